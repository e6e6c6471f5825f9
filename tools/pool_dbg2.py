import ctypes, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch  # noqa
from consensus_overlord_amd.crypto import Context
c = Context(0)
ms = ctypes.c_float()
out = []
for run in range(3):
    c.lib.ovh_pool_debug_reset()
    assert c.lib.ovh_diag_vm_occupancy(c.ptr, 1, 4096, 24, 1, ctypes.byref(ms)) == 0
    buf = (ctypes.c_uint32 * (65536 * 8))()
    n = c.lib.ovh_pool_debug_dump(buf, 65536 * 8)
    a = np.frombuffer(buf, dtype=np.uint32)[:n * 8].reshape(-1, 8).astype(np.uint64)
    t0 = a[:, 2] | (a[:, 3] << 32)
    t1 = a[:, 4] | (a[:, 5] << 32)
    base = t0.min()
    s = (t0 - base) / 100.0  # us
    e = (t1 - base) / 100.0
    work = a[:, 1] > 0
    hw = a[:, 6].astype(np.uint32)
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    xcc = a[:, 7].astype(np.uint32) & 15
    cukey = xcc * 1000 + se * 100 + sh * 20 + cu
    # concurrency of working WGs at several times
    ts = np.linspace(0, e[work].max(), 12)
    conc = [int(((s[work] <= t) & (e[work] > t)).sum()) for t in ts]
    # max per-CU concurrency at the mid time
    mid = e[work].max() / 3
    live = work & (s <= mid) & (e > mid)
    v, cnt = np.unique(cukey[live], return_counts=True)
    hist = {int(k): int(x) for k, x in zip(*np.unique(cnt, return_counts=True))}
    out.append({"ms_per_batch": ms.value / 24, "records": int(n), "working_wgs": int(work.sum()),
                "quads": int(a[:, 1].sum()), "quads_per_wg_pct": [int(np.percentile(a[work, 1], p)) for p in (0, 50, 100)],
                "start_us_pct": [round(float(np.percentile(s[work], p)), 1) for p in (0, 50, 90, 100)],
                "end_us_pct": [round(float(np.percentile(e[work], p)), 1) for p in (0, 10, 50, 100)],
                "concurrency": conc, "cus_live_mid": int(len(v)), "wgs_per_cu_hist_mid": hist})
print(json.dumps(out))
