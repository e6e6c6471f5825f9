#!/usr/bin/env python
"""Same-message path diagnostics: wall time of ovh_verify_batch on n
votes of one hash (host buffers) and the device time of each stage (OVH_FLAG_PROFILE), for the
same-message path and with OVH_SAMEMSG=0.   python tools/samemsg_probe.py"""
import ctypes
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from consensus_overlord_amd import device as dev
    from consensus_overlord_amd.crypto import Context
    out = {}
    for same in (1, 0):
        os.environ["OVH_SAMEMSG"] = str(same)
        ctx = Context(0, flags=bench.OVH_FLAG_PROFILE)
        del os.environ["OVH_SAMEMSG"]
        lib = ctx.lib
        for n in (99, 1024, 4096):
            sks_h, _ = bench.synth_inputs(lib, 0, n)
            sks = torch.from_numpy(sks_h).cuda()
            d = hashlib.sha256(b"probe %d" % n).digest()
            hs = torch.from_numpy(np.tile(np.frombuffer(d, dtype=np.uint8), (n, 1))).cuda()
            pk = dev.sk_to_pk_batch(ctx, sks).cpu().numpy()
            sg = dev.sign_batch(ctx, sks, hs).cpu().numpy()
            codes = np.zeros(n, dtype=np.int32)
            ts = []
            for _ in range(4):
                t = time.perf_counter()
                assert lib.ovh_verify_batch(ctx.ptr, n, sg.tobytes(), d * n, pk.tobytes(),
                                            codes.ctypes.data_as(ctypes.c_void_p)) == 0
                ts.append(time.perf_counter() - t)
            assert not (codes != 0).any()
            stf = (ctypes.c_float * 6)()
            assert lib.ovh_stage_times(ctx.ptr, stf, 6) == 6
            out["samemsg%d_n%d" % (same, n)] = {
                "wall_ms": round(float(np.median(ts[1:])) * 1e3, 3),
                "stage_ms": {lib.ovh_stage_name(k).decode(): round(float(stf[k]), 4) for k in range(6)}}
        ctx.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
