#!/usr/bin/env python
"""Occupancy A/B of the vote program on real votes (tools/occupancy_ab.py uses zeros): one
ovh_verify_batch of the config-3 workload stages 4,096 real votes (and their hash_to_field
planes in slot 0), then ovh_diag_vm_occupancy runs vote launches over them with
OVH_DIAG_KEEP_IN=1 on one stream, two streams and the per-vote pair.
    python tools/occupancy_real.py"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import bench
    from consensus_overlord_amd import device as dev
    from consensus_overlord_amd.crypto import Context
    os.environ["OVH_DIAG_KEEP_IN"] = "1"
    c = Context(0, flags=bench.OVH_FLAG_VM_CLOCK)
    n = 4096
    sks_h, hs_h = bench.synth_inputs(c.lib, 0, n)
    sks = torch.from_numpy(sks_h).cuda()
    hs = torch.from_numpy(hs_h).cuda()
    pks = dev.sk_to_pk_batch(c, sks).cpu().numpy()
    sigs = dev.sign_batch(c, sks, hs).cpu().numpy()
    codes = np.zeros(n, dtype=np.int32)
    assert c.lib.ovh_verify_batch(c.ptr, n, sigs.tobytes(), hs_h.tobytes(), pks.tobytes(),
                                  codes.ctypes.data_as(ctypes.c_void_p)) == 0 and not codes.any()
    ms = ctypes.c_float()
    out = {}
    for streams in (1, 2, 4, 1, 2, 4):
        assert c.lib.ovh_diag_vm_occupancy(c.ptr, 1, n, 8, streams, ctypes.byref(ms)) == 0
        out.setdefault("vote_real_streams%d_ms_per_launch" % streams, []).append(round(ms.value / 8, 4))
    res = {k: min(v) for k, v in out.items()}
    # per-workgroup program time (s_memrealtime, 100 MHz) of the last launch of each mode
    for streams in (1, 2):
        assert c.lib.ovh_diag_vm_occupancy(c.ptr, 1, n, 8, streams, ctypes.byref(ms)) == 0
        k = c.lib.ovh_vm_clock(c.ptr, None, 0)
        buf = (ctypes.c_uint64 * max(1, k))()
        assert c.lib.ovh_vm_clock(c.ptr, buf, k) == k
        st = np.frombuffer(buf, dtype=np.uint64)[:k].reshape(-1, 2).astype(np.float64)
        st = st[st[:, 1] > 0]
        res["wg_ms_median_streams%d" % streams] = round(float(np.median(st[:, 1])) * 1e-5, 4)
        res["clock_ghz_streams%d" % streams] = round(float(np.median(st[:, 0] / st[:, 1] * 0.1)), 3)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
