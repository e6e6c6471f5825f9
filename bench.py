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
G2_GEN_COMPRESSED = bytes.fromhex(
    "93e02b6052719f607dacd3a088274f65596bd0d09920b61ab5da61bbdc7f5049334cf11213945d57e5ac7d055d042b7e"
    "024aa2b2f08f0a91260805272dc51051c6e47ad4fa403b02b4510b647ae3d1770bac0326a805bbefd48056c8c121bdb8")
R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
OVH_FLAG_PROFILE = 0x2
OVH_FLAG_VM_CLOCK = 0x20
OVH_FLAG_POOL_RESERVE = 0x40
# Roofline denominators (integer VALU):
#  PEAK_FULLRATE  the theoretical full-rate 32-bit VALU lane rate, 256 CU x 64 lanes/clk x
#                 2.4 GHz = 3.93e13 lane-ops/s (one wave instruction per 4 cycles per SIMD)
#  PEAK_MAD_U64   the measured v_mad_u64_u32 lane-op rate (tools/ubench/int_rates.hip, best
#                 occupancy: 8 waves per SIMD, 4.14 cycles per wave instruction;
#                 profiles/r04_int_rates.json), at the clock that run held
#  PEAK_MAD_1WAVE_CHAIN  the same instruction on one dependent chain at one wave per SIMD (the
#                 product's order at the vote kernel's occupancy: 5.93 cycles)
# (r01-r03 used 2.9143e13 from a ubench whose loop carried an s_nop between consecutive mads.)
PEAK_FULLRATE = 256 * 64 * 2.4e9
PEAK_MAD_U64 = 3.7584e13
PEAK_MAD_U64_CLOCK_GHZ = 2.371
PEAK_MAD_1WAVE_CHAIN = 2.6448e13
W_V_CANON = 18300   # algorithmic Montgomery products per verification
W_MSM = 350         # the Pippenger share of sum r_i sigma_i (the k_msm_* kernels)
STAGE_TO_WORK = {"hash_to_field": "hash_to_field", "vote": "vote", "fold": "fold_per_partial",
                 "final": "final_per_batch", "fallback": "fallback"}
PER_BATCH_STAGES = {"final"}
NSTAGES = 6


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


def cpu_allowance():
    """CPUs this process may use: its affinity mask, capped by the cgroup CPU quota (cgroup v2
    cpu.max / v1 cfs_quota_us) -- on a shared GPU box the mask may list the whole machine while
    the quota grants a share of it."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as fh:
                q = int(fh.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as fh:
                per = int(fh.read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    n = aff if quota is None else max(1, min(aff, int(quota)))
    return n, {"affinity_cpus": aff, "cgroup_quota_cpus": quota}


def cpu_baseline(sigs: np.ndarray, hs: np.ndarray, pks: np.ndarray, budget_s: float):
    """The CPU oracle's C restatement (oracle/c/bls_oracle.c, 6x64-bit limbs; NOT blst) on the
    host cores, on the same 4096-vote workload: (a) the RLC batch verify over all the threads
    this job may use (the value), (b) the reference's call shape -- one verify_signature per
    vote, serial, one thread (consensus.rs:397-416) -- on a bounded prefix of the votes."""
    sys.path.insert(0, os.path.join(ROOT, "oracle", "py"))
    import orc
    threads, cpu_info = cpu_allowance()
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
    model = None
    try:
        with open("/proc/cpuinfo") as fh:
            model = next((ln.split(":", 1)[1].strip() for ln in fh if ln.startswith("model name")), None)
    except OSError:
        pass
    mulx = bool(orc.load().orc_mulx_active())
    return {"value": round(len(sigs) / dt_b, 2), "unit": "verifications/s", "cores": threads, "kind": "port",
            "per_core": round(len(sigs) / dt_b / threads, 2),
            # r06: the port's Montgomery product as BMI2 mulx + ADX adcx / adox
            # asm (oracle/c/mont_mulx.h; 1.65x per core on the per-vote verify) at -O3
            "fp_mul": "mulx/adx asm" if mulx else "portable u128 CIOS",
            "cpu_model": model, "host_cpus": os.cpu_count(), "allowance": cpu_info,
            "sample": "all %d votes of the workload, RLC batch verify on %d threads = every CPU this job may "
                      "run on (C restatement oracle/c/bls_oracle.c, %s product, not blst), %.2f s" % (
                          len(sigs), threads, "mulx/adx" if mulx else "portable", dt_b),
            "serial_1core": {"value": round(n1 / dt_1, 2), "cores": 1,
                             "sample": "first %d votes, per-vote verify_signature serially (the reference's "
                                       "call shape), %.2f s" % (n1, dt_1)}}


def latencies(ctx, sigs, hs, pks) -> dict:
    """Untimed latency probes after the throughput run (configs 2 and 5 report
    latency; the reference's own call shape is one verify_signature per vote):
      verify_ms      one ovh_verify (Crypto::verify_signature) of a valid vote on a hash this
                     context has not verified before (message-cache miss), median of 5 votes
      verify_samemsg_ms  the same on a hash it has verified before (every vote of a round after
                     the first signs the same hash: message-cache hit, no hash_to_G2), median of 5
      verify_samemsg_table_ms  the same with the voters in the validator table (update_pubkeys)
      sign_ms        one ovh_sign (Crypto::sign) of a vote digest, median of 3
      aggregate67_ms config 2: aggregate_signatures over 67 signatures, median of 3
      qc67_ms        config 2: verify_aggregated_signature over 67 voters, median of 3
      qc_table_ms    config 2 through the validator table (ovh_verify_qc_batch, one QC)
      cfg5_ms        config 5: 1024 votes with 1% sigma + G2, batch incl. bisection, median of 3
      cfg5_valid_ms  the same 1024 votes all valid (no bisection)
      samemsg4096_ms the 4096 config-3 keys all signing one hash (a round's votes: Vote has no voter
                     field, consensus.rs:169-175): one ovh_verify_batch (host buffers, same-message
                     path: one hash_to_G2 + one Miller loop for the batch), median of 3
      round99_ms     the ingress shim (ingress.VoteIngress at proc_network_msg) on a relayer of a
                     100-validator round: 99 SignedVote messages in, decode + device vote digests
                     + one prefetch (default routing: the small-batch path at 99 votes), the N-1
                     trigger flushing them to overlord; median of 3 rounds; round99_samemsg_ms
                     the same with the same-message path forced (OVH_SAMEMSG=2)"""
    import torch
    from consensus_overlord_amd import device as dev
    lib = ctx.lib
    out = {}
    s0, h0, p0 = (bytes(x[0].cpu().numpy()) for x in (sigs, hs, pks))

    def med(fn, k):
        ts = []
        for _ in range(k):
            t = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t)
        return round(float(np.median(ts)) * 1e3, 3)
    five = [tuple(bytes(x[i].cpu().numpy()) for x in (sigs, hs, pks)) for i in range(5)]
    cold = []
    for sg, hh, pk in five:   # first sight of each hash: vote1 + final1
        t = time.perf_counter()
        assert lib.ovh_verify(ctx.ptr, sg, 96, hh, 32, pk, 48) == 0
        cold.append(time.perf_counter() - t)
    out["verify_ms"] = round(float(np.median(cold)) * 1e3, 3)
    hot = []
    for sg, hh, pk in five:   # the hashes again: vote1h + final1
        t = time.perf_counter()
        assert lib.ovh_verify(ctx.ptr, sg, 96, hh, 32, pk, 48) == 0
        hot.append(time.perf_counter() - t)
    out["verify_samemsg_ms"] = round(float(np.median(hot)) * 1e3, 3)
    # the node's usual case: voters in the validator table (update_pubkeys), hash cached
    assert lib.ovh_set_validators(ctx.ptr, b"".join(x[2] for x in five), 5) == 0
    tab = []
    for sg, hh, pk in five:
        t = time.perf_counter()
        assert lib.ovh_verify(ctx.ptr, sg, 96, hh, 32, pk, 48) == 0
        tab.append(time.perf_counter() - t)
    out["verify_samemsg_table_ms"] = round(float(np.median(tab)) * 1e3, 3)
    assert lib.ovh_set_validators(ctx.ptr, None, 0) == 0
    sk0, sgo = bytes(31) + b"\x05", ctypes.create_string_buffer(96)
    assert lib.ovh_sign(ctx.ptr, sk0, 32, h0, 32, sgo) == 0
    out["sign_ms"] = med(lambda: lib.ovh_sign(ctx.ptr, sk0, 32, h0, 32, sgo), 3)
    # config 2: 67 of 100 validators sign one vote digest; aggregate made with the library
    n = 67
    digest = h0
    sks = torch.from_numpy(np.stack([np.frombuffer(
        (int.from_bytes(hashlib.sha256(b"cfg2" + i.to_bytes(4, "big")).digest(), "big") % R_ORDER or 1)
        .to_bytes(32, "big"), dtype=np.uint8) for i in range(100)])).cuda()
    qp = dev.sk_to_pk_batch(ctx, sks).cpu().numpy()
    qs = dev.sign_batch(ctx, sks[:n], torch.from_numpy(np.tile(np.frombuffer(digest, dtype=np.uint8), (n, 1))).cuda())
    qs = qs.cpu().numpy()
    lens = (ctypes.c_size_t * n)(*([96] * n))
    plen = (ctypes.c_size_t * n)(*([48] * n))
    agg = ctypes.create_string_buffer(96)
    assert lib.ovh_aggregate_sigs(ctx.ptr, qs.tobytes(), lens, n, qp[:n].tobytes(), plen, n, agg) == 0
    out["aggregate67_ms"] = med(lambda: lib.ovh_aggregate_sigs(ctx.ptr, qs.tobytes(), lens, n, qp[:n].tobytes(),
                                                               plen, n, agg), 3)
    assert lib.ovh_verify_aggregated(ctx.ptr, agg.raw, 96, digest, 32, qp[:n].tobytes(), plen, n) == 0
    out["qc67_ms"] = med(lambda: lib.ovh_verify_aggregated(ctx.ptr, agg.raw, 96, digest, 32, qp[:n].tobytes(),
                                                           plen, n), 3)
    assert lib.ovh_set_validators(ctx.ptr, qp.tobytes(), 100) == 0
    order = sorted(range(100), key=lambda i: bytes(qp[i]))
    bm = bytearray(13)
    for pos, i in enumerate(order):
        if i < n:
            bm[pos // 8] |= 0x80 >> (pos % 8)
    qcode = (ctypes.c_int32 * 1)()
    assert lib.ovh_verify_qc_batch(ctx.ptr, 1, agg.raw, digest, bytes(bm), 13, qcode) == 0 and qcode[0] == 0
    out["qc_table_ms"] = med(lambda: lib.ovh_verify_qc_batch(ctx.ptr, 1, agg.raw, digest, bytes(bm), 13, qcode), 3)
    assert lib.ovh_set_validators(ctx.ptr, None, 0) == 0
    # config 5: 1024 votes, 1% sigma + G2 at seeded positions
    import random
    sys.path.insert(0, os.path.join(ROOT, "oracle", "py"))
    m = 1024
    s_h = sigs[:m].cpu().numpy().copy()
    bad = sorted(random.Random(5).sample(range(m), m // 100))
    g2 = G2_GEN_COMPRESSED
    for i in bad:   # sigma + G2 via the library: aggregate(sigma_i, G2) (its voters are only parsed)
        a = ctypes.create_string_buffer(96)
        two = (ctypes.c_size_t * 2)(96, 96)
        pl2 = (ctypes.c_size_t * 2)(48, 48)
        assert lib.ovh_aggregate_sigs(ctx.ptr, bytes(s_h[i]) + g2, two, 2, p0 + p0, pl2, 2, a) == 0
        s_h[i] = np.frombuffer(a.raw, dtype=np.uint8)
    d5 = torch.from_numpy(s_h).cuda()
    c5 = torch.empty((m,), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()

    def cfg5(sg):
        dev.verify_batch(ctx, sg, hs[:m], pks[:m], c5)
    cfg5(d5)
    flagged = [i for i in range(m) if int(c5[i].item()) != 0]
    if flagged != bad:
        raise RuntimeError("config 5: flagged %s, expected %s" % (flagged[:8], bad[:8]))
    out["cfg5_ms"] = med(lambda: cfg5(d5), 3)
    out["cfg5_valid_ms"] = med(lambda: cfg5(sigs[:m]), 3)
    out["cfg5_verifs_per_s"] = round(m / (out["cfg5_ms"] * 1e-3), 1)
    out.update(samemsg_probes(ctx, pks))
    return out


def samemsg_probes(ctx, pks) -> dict:
    """Same-message batches: the config-3 keys signing one hash through
    ovh_verify_batch, and one 100-validator round through the ingress shim (latencies doc)."""
    import torch
    from consensus_overlord_amd import device as dev
    from consensus_overlord_amd import ingress as ig
    from consensus_overlord_amd.crypto import FLAG_SK_RAW, ConsensusCrypto, Context
    from consensus_overlord_amd.vote import PRECOMMIT, rlp_vote
    lib = ctx.lib
    out = {}
    n = pks.shape[0]
    buf = ctypes.create_string_buffer(32)
    msg = rlp_vote(7, 0, PRECOMMIT, hashlib.sha256(b"samemsg block").digest())
    assert lib.ovh_sm3(msg, len(msg), buf) == 0
    digest = buf.raw
    sks_h, _ = synth_inputs(lib, 0, n)
    sks = torch.from_numpy(sks_h).cuda()
    hs1 = torch.from_numpy(np.tile(np.frombuffer(digest, dtype=np.uint8), (n, 1))).cuda()
    sg = dev.sign_batch(ctx, sks, hs1).cpu().numpy()
    pk = pks.cpu().numpy()
    codes = np.zeros(n, dtype=np.int32)
    st0 = (ctypes.c_uint64 * 3)()
    assert lib.ovh_samemsg_stats(ctx.ptr, st0) == 0

    def run():
        assert lib.ovh_verify_batch(ctx.ptr, n, sg.tobytes(), digest * n, pk.tobytes(),
                                    codes.ctypes.data_as(ctypes.c_void_p)) == 0
    run()
    st1 = (ctypes.c_uint64 * 3)()
    assert lib.ovh_samemsg_stats(ctx.ptr, st1) == 0
    if (codes != 0).any() or st1[0] - st0[0] != 1:
        raise RuntimeError("same-message batch: rejected votes or the path was not taken")
    ts = []
    for _ in range(3):
        t = time.perf_counter()
        run()
        ts.append(time.perf_counter() - t)
    out["samemsg4096_ms"] = round(float(np.median(ts)) * 1e3, 3)
    out["samemsg4096_verifs_per_s"] = round(n / float(np.median(ts)), 1)
    stf = (ctypes.c_float * NSTAGES)()
    if lib.ovh_stage_times(ctx.ptr, stf, NSTAGES) == NSTAGES:   # the last call's stages (HIP events)
        out["samemsg4096_stage_ms"] = {lib.ovh_stage_name(k).decode(): round(float(stf[k]), 4) for k in range(NSTAGES)}
    # pipelined: batches of the same votes in device memory through ovh_verify_samemsg_device_async
    # (OVH_BATCH_SLOTS in flight, one codes buffer per batch), timed from the first enqueue to
    # ovh_batch_wait -- the same-message counterpart of the headline value
    kb = 24
    sg_d, pk_d = torch.from_numpy(sg).cuda(), pks.contiguous()
    cd = torch.full((kb, n), -1, dtype=torch.int32, device="cuda")
    for j in range(3):
        dev.verify_samemsg_async(ctx, sg_d, digest, pk_d, cd[j])
    dev.batch_wait(ctx)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for j in range(kb):
        dev.verify_samemsg_async(ctx, sg_d, digest, pk_d, cd[j])
    dev.batch_wait(ctx)
    el = time.perf_counter() - t
    if (cd != 0).any():
        raise RuntimeError("pipelined same-message batches: rejected votes")
    out["samemsg4096_pipelined_ms_per_batch"] = round(el / kb * 1e3, 3)
    out["samemsg4096_pipelined_verifs_per_s"] = round(kb * n / el, 1)
    # the same call with the same-message path off (OVH_SAMEMSG=0 at context creation): the
    # distinct-message batch path on the same votes
    os.environ["OVH_SAMEMSG"] = "0"
    try:
        off = Context(torch.cuda.current_device())
    finally:
        del os.environ["OVH_SAMEMSG"]
    assert lib.ovh_verify_batch(off.ptr, n, sg.tobytes(), digest * n, pk.tobytes(),
                                codes.ctypes.data_as(ctypes.c_void_p)) == 0 and not (codes != 0).any()
    ts = []
    for _ in range(3):
        t = time.perf_counter()
        assert lib.ovh_verify_batch(off.ptr, n, sg.tobytes(), digest * n, pk.tobytes(),
                                    codes.ctypes.data_as(ctypes.c_void_p)) == 0
        ts.append(time.perf_counter() - t)
    out["samemsg4096_off_ms"] = round(float(np.median(ts)) * 1e3, 3)
    off.close()
    # ingress: validator 0 is this node; validators 1..99 send their precommits
    nv = 100
    vs = torch.from_numpy(sks_h[:nv].copy()).cuda()
    vpk = dev.sk_to_pk_batch(ctx, vs).cpu().numpy()
    rts, rts_off = [], []
    for rnd in range(8):
        if rnd in (0, 4):   # rounds 0-3: the default routing (99 votes: the small-batch path);
            if rnd:         # rounds 4-7: OVH_SAMEMSG=2 (the same-message path at any size)
                node.ctx.close()
                os.environ["OVH_SAMEMSG"] = "2"
            try:
                node = ConsensusCrypto(bytes(sks_h[0]), ctx=Context(torch.cuda.current_device(), flags=FLAG_SK_RAW))
            finally:
                os.environ.pop("OVH_SAMEMSG", None)
            node.update_pubkeys([bytes(x) for x in vpk])
        msg = rlp_vote(8, rnd, PRECOMMIT, hashlib.sha256(b"round block").digest())
        assert lib.ovh_sm3(msg, len(msg), buf) == 0
        d = buf.raw
        rs = dev.sign_batch(ctx, vs, torch.from_numpy(np.tile(np.frombuffer(d, dtype=np.uint8), (nv, 1))).cuda())
        rs = rs.cpu().numpy()
        wire = [ig.encode_signed_vote(ig.SignedVote(bytes(rs[i]), 8, rnd, PRECOMMIT,
                                                    hashlib.sha256(b"round block").digest(), bytes(vpk[i])))
                for i in range(1, nv)]
        fwd = []
        sh = ig.VoteIngress(node, lambda k, m: fwd.append(m), max_delay_s=1e9)
        t = time.perf_counter()
        for w in wire:
            sh.proc_network_msg(ig.SIGNED_VOTE, w)
        dt = time.perf_counter() - t
        if len(fwd) != nv - 1 or sh.stats["batches"] != 1:
            raise RuntimeError("ingress round: %d forwarded, %d batches" % (len(fwd), sh.stats["batches"]))
        for m in fwd[:3]:
            ig.overlord_verify(node, ig.SIGNED_VOTE, m)
        if rnd % 4:
            (rts if rnd < 4 else rts_off).append(dt)
    out["round99_ms"] = round(float(np.median(rts)) * 1e3, 3)
    out["round99_samemsg_ms"] = round(float(np.median(rts_off)) * 1e3, 3)
    node.ctx.close()
    return out


def vote_clock(sigs, hs, pks, seconds: float):
    """The clock the vote kernel holds under load (MI355X_MICROARCH.md, DVFS give-back): a
    context with OVH_FLAG_VM_CLOCK runs pipelined batches back to back for `seconds`, then every
    workgroup of the last vote launch reports delta s_memtime / delta s_memrealtime around its
    program (ovh_vm_clock). Untimed diagnostic pass after the measured region; no stamp runs in
    the measured context."""
    import torch
    from consensus_overlord_amd import device as dev
    from consensus_overlord_amd.crypto import Context
    c = Context(torch.cuda.current_device(), flags=OVH_FLAG_VM_CLOCK)
    out = torch.empty((4, sigs.shape[0]), dtype=torch.int32, device="cuda")
    t0 = time.perf_counter()
    k = 0
    while time.perf_counter() - t0 < seconds:
        for _ in range(8):
            dev.verify_batch_async(c, sigs, hs, pks, out[k % 4])
            k += 1
        dev.batch_wait(c)
    n = c.lib.ovh_vm_clock(c.ptr, None, 0)
    buf = (ctypes.c_uint64 * max(1, n))()
    assert c.lib.ovh_vm_clock(c.ptr, buf, n) == n
    st = np.frombuffer(buf, dtype=np.uint64)[:n].reshape(-1, 2).astype(np.float64)
    st = st[st[:, 1] > 0]
    ghz = np.sort(st[:, 0] / st[:, 1] * 0.1)
    c.close()
    if not len(ghz):
        return None
    wg_ms = np.sort(st[:, 1]) * 1e-5     # s_memrealtime ticks at 100 MHz -> ms
    return {"clock_ghz": round(float(np.median(ghz)), 3),
            "wg_ms_median": round(float(np.median(wg_ms)), 4),
            "p10_p90_ghz": [round(float(ghz[len(ghz) // 10]), 3), round(float(ghz[len(ghz) * 9 // 10]), 3)],
            "workgroups": int(len(ghz)), "batches": k, "seconds": round(time.perf_counter() - t0, 2),
            "basis": "median over the last vote launch's workgroups of delta s_memtime / delta s_memrealtime "
                     "x 100 MHz after back-to-back batches (OVH_FLAG_VM_CLOCK diagnostic context)"}


def multi_device_leg(args) -> None:
    """One process over several GPUs through the C ABI alone (ovh_create_multi +
    ovh_verify_batch_async + ovh_batch_wait): what a node linking libovhip.so without torch
    runs. Host buffers: the timed region includes staging into pinned memory and the PCIe copies
    (176 B in, 4 B out per vote); each step is one batch of --batch votes per device."""
    import torch
    from consensus_overlord_amd import device as dev
    from consensus_overlord_amd.crypto import ConsensusCrypto, Context
    devs = list(range(torch.cuda.device_count())) if args.multi_device == "all" else \
        [int(x) for x in args.multi_device.split(",")]
    one = Context(devs[0])
    n = args.batch * len(devs)
    sks_h, hs_h = synth_inputs(one.lib, 0, n)
    sks = torch.from_numpy(sks_h).cuda()
    hs = torch.from_numpy(hs_h).cuda()
    pks = dev.sk_to_pk_batch(one, sks).cpu().numpy()
    sigs = dev.sign_batch(one, sks, hs).cpu().numpy()
    one.close()
    c = ConsensusCrypto(bytes(31) + b"\x01", ctx=Context(devices=devs))
    S, H, P = list(map(bytes, sigs)), list(map(bytes, hs_h)), list(map(bytes, pks))
    outs = [np.full(n, -1, dtype=np.int32) for _ in range(args.warmup + args.steps)]
    for s in range(args.warmup):
        c.verify_batch_async(S, H, P, outs[s])
    c.wait()
    t0 = time.perf_counter()
    for s in range(args.steps):
        c.verify_batch_async(S, H, P, outs[args.warmup + s])
    c.wait()
    elapsed = time.perf_counter() - t0
    if any((o != 0).any() for o in outs):
        raise RuntimeError("multi-device batches rejected valid votes")
    print(json.dumps({
        "metric": "BLS12-381 vote verifications/sec (batch 4096) at 1/2/4/8 MI355X vs host blst",
        "value": round(n * args.steps / elapsed, 2), "unit": "verifications/s", "n_gpus": len(set(devs)),
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic (seed 0xC17A keypairs + RLP precommit votes, SURVEY.md 8(d))",
        "config": {"workload": "config3 votes, %d per device per batch, host buffers" % args.batch,
                   "devices": devs, "parallelism": "one process, ovh_create_multi over %d device pipelines, "
                   "partials peer-copied to a rotating final device" % len(devs)},
        "note": "multi-device leg: includes host staging + PCIe copies; not the driver's metric line"}), flush=True)


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
    ap.add_argument("--no-latency", action="store_true", help="skip the untimed latency probes")
    ap.add_argument("--clock-seconds", type=float, default=2.0,
                    help="diagnostic pass after the timed region: back-to-back batches on a context with "
                         "OVH_FLAG_VM_CLOCK for this long, then the vote kernel's held clock (0 = skip)")
    ap.add_argument("--plain-timed-ctx", action="store_true",
                    help="A/B: time the batches on a context without OVH_FLAG_PROFILE (no HIP events in the timed "
                         "region; vote_spans then absent and the roofline uses the profile batches' stage time)")
    ap.add_argument("--shard-path", action="store_true",
                    help="diagnostic: run the multi-GPU pipeline (partials + RCCL all-gather) even at N=1")
    ap.add_argument("--pool-reserve", action="store_true",
                    help="A/B: contexts with OVH_FLAG_POOL_RESERVE (the pool leaves 8 CUs free; shard batches "
                         "in the persistent pool instead of a pool grid per batch)")
    ap.add_argument("--multi-device", default=None, metavar="DEVS",
                    help="the one-process multi-GPU path a Rust node uses: ovh_create_multi over DEVS "
                         "('all' = every visible GPU, or e.g. '0,0'), host-buffer batches of --batch votes "
                         "per device pipelined through ovh_verify_batch_async")
    args = ap.parse_args()

    if args.multi_device:
        return multi_device_leg(args)
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
    elif args.shard_path:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", local))
    sharded = world > 1 or args.shard_path
    reserve = OVH_FLAG_POOL_RESERVE if args.pool_reserve else 0
    ctx = Context(local, flags=OVH_FLAG_PROFILE | reserve)
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
    shards = ShardVerifier(DeviceBackend(ctx)) if sharded else None
    # the timed batches' context: the profiling one (HIP events around each batch's pool grids
    # and stages: vote_spans) unless --plain-timed-ctx
    tctx = ctx if (shards is not None or not args.plain_timed_ctx) else Context(local, flags=0)
    torch.cuda.synchronize()

    nst = NSTAGES
    names = [lib.ovh_stage_name(k).decode() for k in range(nst)]
    stage_ms = np.zeros(nst)
    buf = (ctypes.c_float * nst)()

    def wait_all() -> None:
        if shards:
            shards.wait()
        else:
            dev.batch_wait(tctx)

    def step(s: int, c=None) -> None:
        """Enqueue batch s. Pipelined: batch s's combined check / bisection (second stream)
        overlaps batch s + 1's per-vote stages; every batch's codes row is final after
        batch_wait. Each batch's RLC coefficients come from a fresh getrandom seed (library)."""
        if shards is None:
            dev.verify_batch_async(c or tctx, sigs, hs, pks, codes[s])
        else:
            shards.submit(s, sigs, hs, pks, codes[s], index_base=rank * B)

    for s in range(args.warmup):
        step(s)
    wait_all()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    lib.ovh_vote_spans(tctx.ptr, None, 0)   # forget the warmup batches' vote kernel events
    t0 = time.perf_counter()
    for s in range(args.steps):
        step(args.warmup + s)
    enqueue_s = time.perf_counter() - t0     # host time to enqueue the K batches (diagnostic)
    wait_all()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # HIP events around every timed vote kernel (OVH_FLAG_PROFILE): pipelined batches' vote grids
    # run two at a time on the per-vote stream pair, so the kernel's device-level time per batch
    # is the union of the spans over the batches, and the mean span is one launch's duration
    sp = (ctypes.c_float * (2 * args.steps))()
    nsp = lib.ovh_vote_spans(tctx.ptr, sp, 2 * args.steps)
    vote_spans = None
    if nsp == args.steps and nsp > 0:
        iv = sorted((sp[2 * k], sp[2 * k + 1]) for k in range(nsp))
        union, cur_a, cur_b = 0.0, iv[0][0], iv[0][1]
        for a, b in iv[1:]:
            if a > cur_b:
                union += cur_b - cur_a
                cur_a, cur_b = a, b
            else:
                cur_b = max(cur_b, b)
        union += cur_b - cur_a
        dsum = sum(b - a for a, b in iv)
        vote_spans = {"launches": nsp, "launch_ms": round(dsum / nsp, 4), "union_ms": round(union, 3),
                      "device_ms_per_launch": round(union / nsp, 4), "concurrency": round(dsum / union, 3)}
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
        step(s, ctx)
        if shards is None:
            dev.batch_wait(ctx)
        else:
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
    clock = vote_clock(sigs, hs, pks, args.clock_seconds) if (rank == 0 and args.clock_seconds > 0) else None

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
        # the vote pool's committed PMC passes (tools/pmc_pool.sh -> tools/pmc_pool_summary.py):
        # HBM bytes per 4,096-vote batch (FETCH_SIZE doubled per the gfx950 correction) and the
        # instruction counts per quad for the counter decomposition below; null if absent
        pmc = None
        ppath = os.path.join(ROOT, "consensus_overlord_amd", "pmc_pool.json")
        if os.path.exists(ppath):
            with open(ppath) as fh:
                pmc = json.load(fh)
        traffic = pmc["hbm_bytes_per_batch"] if (pmc and dname == "vote" and B == 4096) else None
        # algorithmic work of the dominant stage: SURVEY.md 8(d) canonical W_v = 18,300 M per vote
        # (Appendix C) less the Pippenger MSM share (350 M), the Fp12 merge (54 M) and the
        # amortised final exponentiation (4 M), which other kernels do; the program's own count
        # (vote program) is reported beside it, and the MSM kernels' own fraction below
        canon = {"vote": W_V_CANON - W_MSM - 54 - 4}
        work_M = canon.get(dname, Mu[STAGE_TO_WORK[dname]])
        macs = work_M * units * macs_per_M
        # the vote pool's device time per batch over the timed region (vote_spans: the union of
        # the pool streams' HIP-event spans / batches) when recorded, else the unpipelined profile
        # batches' HIP-event stage time
        kern_ms = vote_spans["device_ms_per_launch"] if (dname == "vote" and vote_spans) else avg_ms[dom]
        achieved = macs / (kern_ms * 1e-3) / 1e12
        prog_achieved = Mu[STAGE_TO_WORK[dname]] * units * macs_per_M / (kern_ms * 1e-3) / 1e12
        value = world * B * args.steps / elapsed
        path_M = W_V_CANON
        held = clock["clock_ghz"] if clock else None
        # counter decomposition of frac: frac = VALU busy x v_mad share x
        # useful MACs per issued v_mad lane-op x (4.14 / 4 cycles per v_mad at the peak's rate) x
        # (clock / the peak's clock); VALU busy from the PMC instruction count per quad and this
        # run's time per batch, 1,024 SIMDs at the held clock (2.371 GHz without the clock pass)
        decomp = None
        if pmc and dname == "vote" and B == 4096 and pmc.get("valu_per_quad"):
            ghz = held or PEAK_MAD_U64_CLOCK_GHZ
            quads = B // 4
            busy = quads * pmc["valu_per_quad"] * 4 / (1024 * ghz * 1e9 * kern_ms * 1e-3)
            mad_share = pmc["mad_per_quad_static"] / pmc["valu_per_quad"]
            lane_use = 4 * work_M * macs_per_M / (pmc["mad_per_quad_static"] * 64)
            issue = 4.14 / 4 * ghz / PEAK_MAD_U64_CLOCK_GHZ
            pred = busy * mad_share * lane_use * issue
            decomp = {"valu_busy": round(busy, 4), "mad_share": round(mad_share, 4), "lane_use": round(lane_use, 4),
                      "issue_factor": round(issue, 4), "product": round(pred, 4),
                      "product_over_frac": round(pred / (achieved * 1e12 / PEAK_MAD_U64), 4),
                      "valu_per_quad": pmc["valu_per_quad"], "mad_per_quad": pmc["mad_per_quad_static"],
                      "lanes_per_valu": pmc.get("lanes_per_valu"),
                      "wait_any_share": pmc.get("wait_any_share"), "wait_basis": pmc.get("wait_basis"),
                      "lds_bank_conflict_share": pmc.get("lds_bank_conflict_share"),
                      "write_kb_per_batch": pmc.get("write_kb_per_batch"),
                      "basis": "valu_busy = 1,024 quads x SQ_INSTS_VALU per quad x 4 cycles / (1,024 SIMDs x clock x "
                               "kernel_ms_per_batch); mad_share = static v_mad_u64_u32 per quad / SQ_INSTS_VALU per "
                               "quad; lane_use = algorithmic MACs per quad / (v_mad per quad x 64 lanes); "
                               "issue_factor = 4.14 / 4 x clock / 2.371 GHz (the peak's measured v_mad rate); "
                               "counters: " + pmc["source"]}
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
                       "parallelism": ("vote shards x%d, partials all-gathered over RCCL" % world
                                       + (", persistent pool leaving 8 CUs to the collective" if reserve
                                          else ", a pool grid per batch")) if shards is not None
                       else "single GPU"},
            "roofline": {
                "bound": "valu",
                "kernel": dname,
                "achieved": round(achieved, 3),
                "kernel_ms_per_batch": round(float(kern_ms), 4),
                "time_basis": ("the vote pool's device time per batch: union over the timed batches of the HIP-event "
                               "spans around each batch's pool grids on the two pool streams, / batches (the grids "
                               "are persistent: a batch's span runs from its grids' launch point on the pool streams "
                               "to their exit, and consecutive spans overlap; launch_ms = the mean span)"
                               if (dname == "vote" and vote_spans)
                               else "HIP-event stage time of the unpipelined profile batches"),
                "vote_spans": vote_spans,
                "peak": round(PEAK_MAD_U64 / 1e12, 3),
                "unit": "TOP/s (32x32-bit integer MAC lane-ops; peak = measured v_mad_u64_u32 rate)",
                "frac": round(achieved * 1e12 / PEAK_MAD_U64, 4),
                "peak_basis": "v_mad_u64_u32 lane-op rate measured by tools/ubench/int_rates.hip at its best "
                              "occupancy (profiles/r04_int_rates.json), at the clock that run held (%s GHz)"
                              % (PEAK_MAD_U64_CLOCK_GHZ,),
                "peak_fullrate": round(PEAK_FULLRATE / 1e12, 3),
                "frac_of_fullrate_valu": round(achieved * 1e12 / PEAK_FULLRATE, 4),
                "fullrate_basis": "SURVEY 8(d): 256 CU x 64 lanes/clk x 2.4 GHz (one wave instruction per 4 "
                                  "cycles per SIMD)",
                "vote_clock": clock,
                "frac_of_fullrate_at_held_clock": (round(achieved * 1e12 / (256 * 64 * held * 1e9), 4)
                                                   if held else None),
                "frac_of_1wave_chain_rate": round(achieved * 1e12 / PEAK_MAD_1WAVE_CHAIN, 4),
                "one_wave_chain_basis": "v_mad_u64_u32 on one dependent chain at one wave per SIMD (the vote "
                                        "kernel's occupancy and the product's order), 2.6448e13 lane-ops/s",
                "work_M_per_unit": work_M,
                "work_basis": "SURVEY 8(d) canonical W_v minus MSM + merge + amortised FE" if dname in canon
                              else "program heavy ops (workmodel.json)",
                "program_M_per_unit": Mu[STAGE_TO_WORK[dname]],
                "program_frac": round(prog_achieved * 1e12 / PEAK_MAD_U64, 4),
                "traffic": traffic,
                "traffic_unit": "HBM bytes per 4,096-vote batch of the vote pool (PMC FETCH_SIZE x 2 + WRITE_SIZE, "
                                "consensus_overlord_amd/pmc_pool.json)",
                "pmc": decomp,
                "msm": ({"ms": round(float(avg_ms[names.index("msm")]), 4), "work_M_per_unit": W_MSM,
                         "frac": round(W_MSM * B * macs_per_M / (avg_ms[names.index("msm")] * 1e-3) / PEAK_MAD_U64, 4)}
                        if avg_ms[names.index("msm")] > 0 else None),
                "path_M_per_vote": round(path_M, 1),
                "path_frac": round(value / world * path_M * macs_per_M / PEAK_MAD_U64, 4),
            },
            "stage_ms": stages,
            "batch_latency_ms": round(float(np.median(lat)) * 1e3, 3) if lat else None,
            "enqueue_ms_per_step": round(enqueue_s / args.steps * 1e3, 4),
            "pipelined": "the vote pool runs every batch's per-vote work (persistent grids, quads claimed across "
                         "batches); batch k's fold, MSM, combined check and bisection run on one of four final "
                         "streams beside later batches' votes; all %d timed batches complete inside the timed "
                         "region" % args.steps,
        }
        if world == 1 and not args.no_latency:
            line["latency"] = latencies(ctx, sigs, hs, pks)
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(sigs.cpu().numpy(), hs_h, pks.cpu().numpy(), args.cpu_seconds)
        print(json.dumps(line), flush=True)
    if tctx is not ctx:
        tctx.close()
    ctx.close()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
