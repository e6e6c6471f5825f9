#!/usr/bin/env python
"""bench.py -- BLS12-381 vote verifications/s (batch 4096 per GPU) through libovhip on MI355X.

Metric (BASELINE.json): "BLS12-381 vote verifications/sec (batch 4096) at 1/2/4/8 MI355X vs
host blst". Workload = BASELINE config 3: 4096 independent precommit votes with distinct
messages per GPU, random-linear-combination batch verify (`ovh_verify_batch_device`, the
batched form of ConsensusCrypto::verify_signature, src/consensus.rs:397-416).

Synthetic inputs: seed 0xC17A; sk_i = SHA-256(seed || i) mod r; vote i =
rlp(Vote{height 1 + i/64, round i%3, Precommit, block_hash SM3(seed || i)}); digest = SM3(rlp);
pk_i = sk_i G1, sigma_i = sk_i H(digest) -- keys and signatures are made on the device (untimed
setup), so inputs are resident in HBM when the timed region starts.

One step = one batch verify of the rank's 4096 votes. N = 1: ovh_verify_batch_device (all
stages + final exponentiation + verdict). N > 1 (one process per GPU, torchrun): each rank
computes its shard partial (Fp12 Miller product + G2 sum, 864 B), the partials are
all-gathered over RCCL, and the combined check runs on the gathered partials (weak scaling:
4096 votes per GPU).

Also reported: "roofline" for the dominant kernel stage (integer VALU: 32x32-bit MAC lane-op
rate from the work model in consensus_overlord_amd/workmodel.json over HIP-event time on the
library's stream, against the microbenchmarked v_mad_u64_u32 rate), and "cpu_baseline" (the
C restatement of the CPU oracle, timed on rank 0 at N = 1: RLC batch on the host threads
plus the serial per-vote call shape on a bounded prefix).
"""
from __future__ import annotations

import argparse
import ctypes
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

SEED = 0xC17A
R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
OVH_FLAG_PROFILE = 0x2
# measured v_mad_u64_u32 lane-op rate on gfx950 (tools/ubench/int_rates.hip,
# profiles/r01_int_rates_ubench.json) and the full-rate 32-bit VALU lane rate
# (256 CU x 4 SIMD x 32 lanes x 2.4 GHz).
PEAK_MAD_U64 = 2.9143e13
PEAK_FULLRATE = 256 * 4 * 32 * 2.4e9
STAGE_TO_WORK = {"hash_to_field": "hash_to_field", "vote": "vote", "fold": "fold_per_partial",
                 "final": "final_per_batch", "fallback": "fallback"}
PER_BATCH_STAGES = {"final"}
NSTAGES = 5


def synth_inputs(lib, lo: int, n: int):
    """sks (n,32) and digests (n,32) for votes lo..lo+n-1."""
    from consensus_overlord_amd.vote import PRECOMMIT, rlp_vote
    sks = np.zeros((n, 32), dtype=np.uint8)
    hs = np.zeros((n, 32), dtype=np.uint8)
    buf = ctypes.create_string_buffer(32)
    for k in range(n):
        i = lo + k
        tag = SEED.to_bytes(8, "big") + i.to_bytes(8, "big")
        sk = int.from_bytes(hashlib.sha256(tag).digest(), "big") % R_ORDER or 1
        sks[k] = np.frombuffer(sk.to_bytes(32, "big"), dtype=np.uint8)
        assert lib.ovh_sm3(tag, len(tag), buf) == 0
        msg = rlp_vote(1 + i // 64, i % 3, PRECOMMIT, buf.raw)
        assert lib.ovh_sm3(msg, len(msg), buf) == 0
        hs[k] = np.frombuffer(buf.raw, dtype=np.uint8)
    return sks, hs


def cpu_baseline(sigs: np.ndarray, hs: np.ndarray, pks: np.ndarray, budget_s: float):
    """The CPU oracle's C restatement (oracle/c/bls_oracle.c, 6x64-bit limbs; NOT blst) on the
    host cores, on the same 4096-vote workload: (a) the RLC batch verify over all the threads
    this job may use (the value), (b) the reference's call shape -- one verify_signature per
    vote, serial, one thread (consensus.rs:397-416) -- on a bounded prefix of the votes."""
    sys.path.insert(0, os.path.join(ROOT, "oracle", "py"))
    import orc
    threads = max(1, min(int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1), 64))
    t0 = time.perf_counter()
    codes, ok = orc.verify_batch_rlc(sigs, hs, pks, seed=0xC17A, threads=threads)
    dt_b = time.perf_counter() - t0
    if not ok or (codes != 0).any():
        raise RuntimeError("CPU oracle rejects GPU-made votes")
    n1 = 0
    t0 = time.perf_counter()
    while n1 < len(sigs) and (n1 < 8 or time.perf_counter() - t0 < budget_s):
        chunk = min(32, len(sigs) - n1)
        c = orc.verify_many(sigs[n1:n1 + chunk], hs[n1:n1 + chunk], pks[n1:n1 + chunk], 1)
        if (c != 0).any():
            raise RuntimeError("CPU oracle rejects GPU-made votes")
        n1 += chunk
    dt_1 = time.perf_counter() - t0
    return {"value": round(len(sigs) / dt_b, 2), "unit": "verifications/s", "cores": threads, "kind": "port",
            "sample": "all %d votes of the workload, RLC batch verify on %d threads (C restatement "
                      "oracle/c/bls_oracle.c, not blst), %.2f s" % (len(sigs), threads, dt_b),
            "serial_1core": {"value": round(n1 / dt_1, 2), "cores": 1,
                             "sample": "first %d votes, per-vote verify_signature serially (the reference's "
                                       "call shape), %.2f s" % (n1, dt_1)}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 30 batches: the pipeline's one-batch drain (the last batch's final check, ~3 ms) is then
    # a small part of the timed region
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=4096, help="votes per GPU per step")
    ap.add_argument("--profile-steps", type=int, default=3, help="untimed unpipelined batches for stage times")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE %d (launch N>1 with torch.distributed.run)" % (args.gpus, world))

    import torch
    import torch.distributed as dist
    from consensus_overlord_amd import device as dev
    from consensus_overlord_amd.crypto import Context
    from consensus_overlord_amd.shard import DeviceBackend, ShardVerifier

    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    ctx = Context(local, flags=OVH_FLAG_PROFILE)
    lib = ctx.lib
    B = args.batch

    # ---- untimed setup: synthetic keys/messages, pks and signatures made on the device ----
    sks_h, hs_h = synth_inputs(lib, rank * B, B)
    sks = torch.from_numpy(sks_h).cuda()
    hs = torch.from_numpy(hs_h).cuda()
    pks = dev.sk_to_pk_batch(ctx, sks)
    sigs = dev.sign_batch(ctx, sks, hs)
    nbatch = args.warmup + args.steps + args.profile_steps
    codes = torch.full((nbatch, B), -1, dtype=torch.int32, device="cuda")   # one verdict row per batch
    shards = ShardVerifier(DeviceBackend(ctx)) if world > 1 else None
    torch.cuda.synchronize()

    nst = NSTAGES
    names = [lib.ovh_stage_name(k).decode() for k in range(nst)]
    stage_ms = np.zeros(nst)
    buf = (ctypes.c_float * nst)()

    def wait_all() -> None:
        if shards:
            shards.wait()
        else:
            dev.batch_wait(ctx)

    def step(s: int) -> None:
        """Enqueue batch s. Pipelined: batch s's combined check / fallback (second stream) overlaps
        batch s + 1's per-vote stages; every batch's codes row is final after batch_wait."""
        seed = (SEED << 32) ^ (s * 0x10001)
        if world == 1:
            dev.verify_batch_async(ctx, sigs, hs, pks, seed, codes[s])
        else:
            shards.submit(s, sigs, hs, pks, seed, codes[s])

    for s in range(args.warmup):
        step(s)
    wait_all()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.steps):
        step(args.warmup + s)
    wait_all()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # per-stage device times of single (unpipelined) batches, untimed: the roofline's kernel time
    # and the per-batch latency breakdown
    lat = []
    for s in range(args.warmup + args.steps, nbatch):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        step(s)
        wait_all()
        lat.append(time.perf_counter() - t1)
        got = lib.ovh_stage_times(ctx.ptr, buf, nst)
        if got != nst:
            raise RuntimeError("ovh_stage_times returned %d" % got)
        stage_ms += np.frombuffer(buf, dtype=np.float32)

    # sanity: every vote of every batch (warmup, timed, profiled) of the synthetic workload is valid
    bad = int((codes != 0).sum().item())
    if bad:
        raise RuntimeError("batch verify rejected %d valid votes" % bad)

    if rank == 0:
        with open(os.path.join(ROOT, "consensus_overlord_amd", "workmodel.json")) as fh:
            wm = json.load(fh)
        macs_per_M = wm["macs_per_M"]
        Mu = wm["M_per_unit"]
        avg_ms = stage_ms / max(1, args.profile_steps)
        stages = {names[k]: round(float(avg_ms[k]), 4) for k in range(nst)}
        dom = max((k for k in range(nst) if names[k] in STAGE_TO_WORK), key=lambda k: avg_ms[k])
        dname = names[dom]
        units = 1 if dname in PER_BATCH_STAGES else B
        # HBM bytes per launch of the dominant kernel from the committed PMC pass
        # (tools/pmc_round.sh; FETCH_SIZE doubled per the gfx950 correction); null if absent
        traffic = None
        tpath = os.path.join(ROOT, "consensus_overlord_amd", "pmc_traffic.json")
        if os.path.exists(tpath):
            with open(tpath) as fh:
                tk = json.load(fh)["kernels"].get("k_vm_" + dname)
            if tk is not None and B == 4096:
                traffic = tk["hbm_bytes_per_launch"]
        macs = Mu[STAGE_TO_WORK[dname]] * units * macs_per_M
        achieved = macs / (avg_ms[dom] * 1e-3) / 1e12
        value = world * B * args.steps / elapsed
        path_M = Mu["hash_to_field"] + Mu["vote"] + Mu["fold_per_partial"] * 4.0 / 3.0 + Mu["final_per_batch"] / B
        line = {
            "metric": "BLS12-381 vote verifications/sec (batch 4096) at 1/2/4/8 MI355X vs host blst",
            "value": round(value, 2),
            "unit": "verifications/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (seed 0xC17A keypairs + RLP precommit votes, SURVEY.md 8(d))",
            "config": {"workload": "config3: %d distinct-message precommit votes per GPU, RLC batch verify" % B,
                       "batch_per_gpu": B, "global_batch": world * B,
                       "parallelism": "vote shards x%d, partials all-gathered over RCCL" % world if world > 1
                       else "single GPU"},
            "roofline": {
                "bound": "valu",
                "kernel": dname,
                "achieved": round(achieved, 3),
                "peak": round(PEAK_MAD_U64 / 1e12, 3),
                "unit": "TOP/s (32x32-bit integer MAC lane-ops; peak = measured v_mad_u64_u32 rate)",
                "frac": round(achieved * 1e12 / PEAK_MAD_U64, 4),
                "frac_of_fullrate_valu": round(achieved * 1e12 / PEAK_FULLRATE, 4),
                "traffic": traffic,
                "traffic_unit": "HBM bytes per launch (PMC FETCH_SIZE x 2 + WRITE_SIZE, pmc_traffic.json)",
                "path_M_per_vote": round(path_M, 1),
                "path_frac": round(value / world * path_M * macs_per_M / PEAK_MAD_U64, 4),
            },
            "stage_ms": stages,
            "batch_latency_ms": round(float(np.median(lat)) * 1e3, 3) if lat else None,
            "pipelined": "batch k's combined check + fallback (second stream) overlap batch k+1's per-vote "
                         "stages; all %d timed batches complete inside the timed region" % args.steps,
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(sigs.cpu().numpy(), hs_h, pks.cpu().numpy(), args.cpu_seconds)
        print(json.dumps(line), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
