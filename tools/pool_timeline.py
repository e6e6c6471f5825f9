#!/usr/bin/env python
"""Pool timeline (diagnostic, no profiler): bench.py's pipelined loop -- config 3, warmup 2 + K
batches through ovh_verify_batch_device_async -- on an OVH_FLAG_VM_CLOCK context, then the
pool log (ovh_pool_log): per batch its publication, first quad start, last quad end and the final
stream's events, plus the quads in flight over time. One JSON object per run on stdout.

    python tools/pool_timeline.py [K] [runs] [shard [rsv]] > gpurun_out/timeline.json

shard: through the shard driver at one RCCL rank; rsv: on an OVH_FLAG_POOL_RESERVE context.
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

RING, QUADS, WORDS = 64, 1024, 16 + 2 * 1024
GRIDS, WGS, WGW = 64, 1024, 4
TOTAL = RING * WORDS + GRIDS * (4 + WGS * WGW)
EV = ["pub", "done", "fold", "msm", "final", "back", "gath", "comb", "fe"]


def one_run(c, dev, sigs, hs, pks, K, codes):
    import numpy as np
    import torch
    for s in range(2):
        dev.verify_batch_async(c, sigs, hs, pks, codes[s])
    dev.batch_wait(c)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(K):
        dev.verify_batch_async(c, sigs, hs, pks, codes[2 + s])
    dev.batch_wait(c)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    buf = (ctypes.c_uint64 * TOTAL)()
    assert c.lib.ovh_pool_log(c.ptr, buf, TOTAL) == TOTAL
    allw = np.frombuffer(buf, dtype=np.uint64)
    a = allw[:RING * WORDS].reshape(RING, WORDS)
    g = allw[RING * WORDS:].reshape(GRIDS, 4 + WGS * WGW)
    seqs = a[:, 15].astype(np.int64)
    last = int(seqs.max())
    recs = sorted([r for r in range(RING) if a[r, 0] and seqs[r] > last - K], key=lambda r: seqs[r])
    t_base = int(a[recs[0], 0])
    rows, spans = [], []
    for r in recs:
        q = a[r, 16:].reshape(QUADS, 2)
        st = (q[:, 0] & ((1 << 48) - 1)).astype(np.int64)
        en = q[:, 1].astype(np.int64)
        ok = (st > 0) & (en > 0)
        st, en = st[ok], en[ok]
        key = ((q[:, 0] >> 48) & 0xFFF).astype(np.int64)[ok]   # the SIMD the quad ran on (simd_key)
        how = (q[:, 0] >> 60).astype(np.int64)[ok]   # the claim's flags (pool_claim)
        _, inv, per = np.unique(key, return_inverse=True, return_counts=True)
        _, cinv, cper = np.unique(key >> 2, return_inverse=True, return_counts=True)
        dur = (en - st) / 100.0
        # quad time by how many of the batch's quads shared its SIMD / its CU
        by_simd = {int(k): round(float(np.median(dur[per[inv] == k])), 1) for k in np.unique(per)}
        by_cu = {int(k): [int((cper[cinv] == k).sum()), round(float(np.median(dur[cper[cinv] == k])), 1)]
                 for k in np.unique(cper)}
        spans.append(np.stack([st, en], 1))
        ev = {EV[k]: round((int(a[r, k]) - t_base) / 100.0, 1) if a[r, k] else None for k in range(len(EV))}
        rows.append({"seq": int(seqs[r]), **ev,
                     "q_first": round((int(st.min()) - t_base) / 100.0, 1),
                     "q_last": round((int(en.max()) - t_base) / 100.0, 1),
                     "quad_us_med": round(float(np.median(en - st)) / 100.0, 1), "quads": int(ok.sum()),
                     "simds": len(per), "quads_per_simd_max": int(per.max()) if len(per) else 0,
                     "claim_flags": {int(k): int(v) for k, v in zip(*np.unique(how, return_counts=True))},
                     "claim_flags_doubled": {int(k): int(v) for k, v in zip(*np.unique(how[per[inv] > 1], return_counts=True))},
                     "quad_us_pct": [round(float(np.percentile(dur, p_)), 1) for p_ in (1, 10, 50, 90, 99, 100)],
                     "quad_us_by_simd_share": by_simd, "quads_and_us_by_cu_share": by_cu,
                     # the slowest 1%: (us, quads on its SIMD, on its CU, start after the first)
                     "slowest": [(round(float(dur[k]), 1), int(per[inv][k]), int(cper[cinv][k]),
                                  round((int(st[k]) - int(st.min())) / 100.0, 1))
                                 for k in np.argsort(-dur)[:max(1, len(dur) // 100)]]})
    sp = np.concatenate(spans)
    t_end = int(sp[:, 1].max())
    grid = np.arange(t_base, t_end, 10000)  # every 100 us
    st_s, en_s = np.sort(sp[:, 0]), np.sort(sp[:, 1])
    inflight = np.searchsorted(st_s, grid, side="right") - np.searchsorted(en_s, grid, side="right")
    grids = []
    for r in sorted(range(GRIDS), key=lambda r: int(g[r, 3])):
        if not g[r, 3] or int(g[r, 0]) <= last - K:
            continue
        w = g[r, 4:].reshape(WGS, WGW).astype(np.int64)
        nw = min(int(g[r, 2]), WGS)
        w = w[:nw]
        ran = w[:, 0] > 0
        rel = lambda x: round((int(x) - t_base) / 100.0, 1)
        grids.append({"seq": int(g[r, 0]), "par": int(g[r, 1]), "launch": rel(g[r, 3]), "wgs": nw,
                      "ran": int(ran.sum()),
                      "enter_pct": [rel(np.percentile(w[ran, 0], p)) for p in (0, 50, 100)] if ran.any() else None,
                      "exit_pct": [rel(np.percentile(w[ran, 1], p)) for p in (0, 50, 100)] if ran.any() else None,
                      "quads_hist": {int(k): int(v) for k, v in zip(*np.unique(w[ran, 2], return_counts=True))},
                      "why": {int(k): int(v) for k, v in zip(*np.unique(w[ran, 3], return_counts=True))}})
    return {"grids": grids, "ms": round(ms, 2), "ms_per_batch": round(ms / K, 3), "batches": rows,
            "inflight_pct": [int(np.percentile(inflight, p)) for p in (5, 25, 50, 75, 95)],
            "inflight_ms": [int(x) for x in inflight[::10]]}


def main():
    import numpy as np
    import torch
    import bench
    from consensus_overlord_amd import device as dev
    from consensus_overlord_amd.crypto import Context
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    runs = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    shard = len(sys.argv) > 3 and sys.argv[3] == "shard"
    rsv = bench.OVH_FLAG_POOL_RESERVE if len(sys.argv) > 4 and sys.argv[4] == "rsv" else 0
    c = Context(0, flags=bench.OVH_FLAG_PROFILE | bench.OVH_FLAG_VM_CLOCK | rsv)
    sks_h, hs_h = bench.synth_inputs(c.lib, 0, 4096)
    sks = torch.from_numpy(sks_h).cuda()
    hs = torch.from_numpy(hs_h).cuda()
    pks = dev.sk_to_pk_batch(c, sks)
    sigs = dev.sign_batch(c, sks, hs)
    codes = torch.full((K + 2, 4096), -1, dtype=torch.int32, device="cuda")
    if shard:   # the per-rank shard path at one rank (bench.py --shard-path): RCCL world of one
        import torch.distributed as dist
        from consensus_overlord_amd.shard import DeviceBackend, ShardVerifier
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        sv = ShardVerifier(DeviceBackend(c))
        nsub = [0]

        class dev:   # one_run's two calls over the shard driver
            @staticmethod
            def verify_batch_async(ctx, s_, h_, p_, cd):
                sv.submit(nsub[0], s_, h_, p_, cd)
                nsub[0] += 1

            @staticmethod
            def batch_wait(ctx):
                sv.wait()
    for _ in range(runs):
        codes.fill_(-1)
        out = one_run(c, dev, sigs, hs, pks, K, codes)
        out["bad_codes"] = int((codes != 0).sum().item())
        print(json.dumps(out), flush=True)
    c.close()


if __name__ == "__main__":
    main()
