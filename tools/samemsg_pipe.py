#!/usr/bin/env python
"""Pipelined same-message batches (ovh_verify_samemsg_device_async):
K batches of n config-3 keys signing one hash, enqueued back to back; prints ms per batch.
Run under `rocprofv3 --kernel-trace` to see which stream limits the period.
    python tools/samemsg_pipe.py [K] [n]"""
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
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    ctx = Context(0)
    sks_h, _ = bench.synth_inputs(ctx.lib, 0, n)
    sks = torch.from_numpy(sks_h).cuda()
    d = hashlib.sha256(b"pipe").digest()
    hs = torch.from_numpy(np.tile(np.frombuffer(d, dtype=np.uint8), (n, 1))).cuda()
    pk = dev.sk_to_pk_batch(ctx, sks)
    sg = dev.sign_batch(ctx, sks, hs)
    cd = torch.full((K, n), -1, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    out = {}
    for rep in range(2):
        t = time.perf_counter()
        for j in range(K):
            dev.verify_samemsg_async(ctx, sg, d, pk, cd[j])
        dev.batch_wait(ctx)
        el = time.perf_counter() - t
        assert not (cd != 0).any()
        out["rep%d_ms_per_batch" % rep] = round(el / K * 1e3, 3)
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
