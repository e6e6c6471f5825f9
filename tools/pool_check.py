#!/usr/bin/env python
"""Pipelined-batch consistency probe: K batches of the bench's 4096 synthetic votes through
ovh_verify_batch_device_async into K codes rows, then a histogram of each row's codes (all 0
expected). Prints one JSON line.   python tools/pool_check.py [K]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from bench import synth_inputs
    from consensus_overlord_amd import device as dev
    from consensus_overlord_amd.crypto import Context
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    c = Context(0)
    sks_h, hs_h = synth_inputs(c.lib, 0, 4096)
    sks = torch.from_numpy(sks_h).cuda()
    hs = torch.from_numpy(hs_h).cuda()
    pks = dev.sk_to_pk_batch(c, sks)
    sigs = dev.sign_batch(c, sks, hs)
    out = {}
    for mode in ("single", "pipelined"):
        codes = torch.full((k, 4096), -7, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        for j in range(k):
            dev.verify_batch_async(c, sigs, hs, pks, codes[j])
            if mode == "single":
                dev.batch_wait(c)
        dev.batch_wait(c)
        torch.cuda.synchronize()
        rows = []
        for j in range(k):
            v, n = np.unique(codes[j].cpu().numpy(), return_counts=True)
            rows.append({int(a): int(b) for a, b in zip(v, n)})
        out[mode] = rows
    print(json.dumps(out))
    c.close()


if __name__ == "__main__":
    main()
