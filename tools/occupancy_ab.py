#!/usr/bin/env python
"""Occupancy A/B of the Fp-VM: does a second wave per SIMD speed a VM
program up? vsame (75 slots) fits eight workgroups per CU, so two launches over 4,096 votes on two
streams co-reside (two waves per SIMD); the same launches on one stream run one wave per SIMD.
The vote program (159 slots) is the control: its two-stream run cannot co-reside.

    python tools/occupancy_ab.py > gpurun_out/occ.json
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch  # noqa: F401  (one HIP runtime with torch)
    from consensus_overlord_amd.crypto import Context
    c = Context(0)
    ms = ctypes.c_float()
    out = {}
    for prog, name in ((0, "vsame"), (1, "vote")):
        for streams in ((1, 2, 3, 4, 1, 2, 3, 4) if prog else (1, 2, 1, 2)):
            assert c.lib.ovh_diag_vm_occupancy(c.ptr, prog, 4096, 8, streams, ctypes.byref(ms)) == 0
            out.setdefault("%s_streams%d_ms_per_launch" % (name, streams), []).append(round(ms.value / 8, 4))
    for k in list(out):
        out[k] = min(out[k])
    for name in ("vsame", "vote"):
        out["%s_speedup_two_streams" % name] = round(out["%s_streams1_ms_per_launch" % name] /
                                                     out["%s_streams2_ms_per_launch" % name], 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
