#!/usr/bin/env python
"""Per-phase clock of the Fp-VM programs on the GPU (diagnostics).

Runs one 4096-vote batch on a context created with OVH_FLAG_VM_TRACE and saves workgroup 0's
wall-clock stamps (100 MHz) of the vote and final programs to <out>.npz. Analyse on the host
with tools/fpvm/phase_costs.py (joins the stamps with the program's per-phase op mix).

    python tools/vm_trace.py gpurun_out/trace_r01f
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

OVH_FLAG_VM_TRACE = 0x4


def main():
    out = sys.argv[1]
    import torch
    import bench
    from consensus_overlord_amd import device as dev
    from consensus_overlord_amd.crypto import Context

    ctx = Context(0, flags=OVH_FLAG_VM_TRACE)
    lib = ctx.lib
    B = 4096
    sks_h, hs_h = bench.synth_inputs(lib, 0, B)
    sks = torch.from_numpy(sks_h).cuda()
    hs = torch.from_numpy(hs_h).cuda()
    pks = dev.sk_to_pk_batch(ctx, sks)
    sigs = dev.sign_batch(ctx, sks, hs)
    codes = torch.empty((B,), dtype=torch.int32, device="cuda")
    res = {}
    for rep in range(2):  # second run: warm caches
        dev.verify_batch(ctx, sigs, hs, pks, codes)
        torch.cuda.synchronize()
    assert int((codes != 0).sum()) == 0
    for k, name in enumerate(["vote", "fold", "final", "pairchk"]):
        n = lib.ovh_vm_trace(ctx.ptr, k, None, 0)
        buf = (ctypes.c_uint64 * n)()
        assert lib.ovh_vm_trace(ctx.ptr, k, buf, n) == n
        res[name] = np.frombuffer(buf, dtype=np.uint64).copy()
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    np.savez(out, **res)
    v = res["vote"].astype(np.int64)
    f = res["final"].astype(np.int64)
    print("vote: %d phases, %.3f ms; final: %d phases, %.3f ms" %
          (len(v) - 1, (v[-1] - v[0]) / 1e5, len(f) - 1, (f[-1] - f[0]) / 1e5))


if __name__ == "__main__":
    main()
