import ctypes, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch
from bench import synth_inputs
from consensus_overlord_amd import device as dev
from consensus_overlord_amd.crypto import Context
c = Context(0)
sks_h, hs_h = synth_inputs(c.lib, 0, 4096)
sks = torch.from_numpy(sks_h).cuda(); hs = torch.from_numpy(hs_h).cuda()
pks = dev.sk_to_pk_batch(c, sks); sigs = dev.sign_batch(c, sks, hs)
k = 8
codes = torch.full((k, 4096), -7, dtype=torch.int32, device="cuda")
torch.cuda.synchronize()
for j in range(k):
    dev.verify_batch_async(c, sigs, hs, pks, codes[j])
dev.batch_wait(c)
torch.cuda.synchronize()
buf = (ctypes.c_uint32 * (65536 * 16))()
n = c.lib.ovh_pool_debug_dump(buf, 65536 * 16)
a = np.frombuffer(buf, dtype=np.uint32)[:n * 16].reshape(-1, 16)
out = {"records": int(n)}
ptr = {}
for s in np.unique(a[:, 9]):
    r = a[a[:, 9] == s]
    d = {}
    for col, name in [(1, "slot"), (3, "n"), (4, "codes_lo"), (6, "code"), (7, "pf"), (8, "sf"), (10, "stage_lo"), (11, "state_lo"), (12, "table")]:
        v, cnt = np.unique(r[:, col], return_counts=True)
        d[name] = {int(x): int(y) for x, y in zip(v[:8], cnt[:8])}
    d["i_range"] = [int(r[:, 5].min()), int(r[:, 5].max()), int(len(np.unique(r[:, 5])))]
    ptr[int(s)] = d
out["per_seq"] = ptr
rows = []
for j in range(k):
    v, cnt = np.unique(codes[j].cpu().numpy(), return_counts=True)
    rows.append({int(x): int(y) for x, y in zip(v, cnt)})
out["rows"] = rows
out["codes_rows_lo"] = [int(codes[j].data_ptr() & 0xffffffff) for j in range(k)]
print(json.dumps(out))
