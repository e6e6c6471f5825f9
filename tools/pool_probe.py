#!/usr/bin/env python
"""The vote pool alone ("Vote pool"): ovh_diag_vm_occupancy(prog = 1)
publishes `reps` batches of n zero votes back to back (staging, hash_to_field, publication; no
final-stream work) and times them. ms per batch is the pool's device time per batch -- the
diagnostic counterpart of the pipelined bench's `roofline.vote_spans.device_ms_per_launch`.

    python tools/pool_probe.py [n] [reps] [prog] [runs] > gpurun_out/pool.json

prog 2 publishes all reps (<= 6) batches before the pool's grids start (the PMC passes of
tools/pmc_pool.sh).
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
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 24
    prog = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    nrun = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    c = Context(0)
    ms = ctypes.c_float()
    runs = []
    for _ in range(nrun):
        assert c.lib.ovh_diag_vm_occupancy(c.ptr, prog, n, reps, 1, ctypes.byref(ms)) == 0
        runs.append(round(ms.value / reps, 4))
    print(json.dumps({"votes_per_batch": n, "batches": reps, "prog": prog, "ms_per_batch_runs": runs,
                      "ms_per_batch": min(runs), "verifs_per_s": round(n / (min(runs) * 1e-3), 1)}))
    c.close()


if __name__ == "__main__":
    main()
