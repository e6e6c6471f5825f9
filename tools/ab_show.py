"""Summarise an A/B run directory of tools/ab_tmp.sh: pytest tail, pool timelines, bench lines."""
import glob
import json
import os
import sys

d = os.path.join("gpurun_out", sys.argv[1])
for f in sorted(glob.glob(d + "/*.log")):
    lines = open(f).read().splitlines()
    js = [x for x in lines if x.startswith("{")]
    if js:
        b = json.loads(js[0])
        print(os.path.basename(f), b["value"], b["ms_per_step"], b["roofline"]["frac"], b["stage_ms"],
              b["batch_latency_ms"], {k: v for k, v in b.get("latency", {}).items() if k in ("verify_ms", "qc67_ms", "round99_ms", "samemsg4096_pipelined_verifs_per_s")})
    elif lines:
        print(os.path.basename(f), lines[-1])
for f in sorted(glob.glob(d + "/tl*.json")):
    for l in open(f):
        t = json.loads(l)
        print(os.path.basename(f), t["ms"], t["ms_per_batch"], t["inflight_pct"])
        for b in t["batches"][-2:]:
            print("   ", {k: v for k, v in b.items() if k not in ("fold", "msm", "final", "back", "quads_and_us_by_cu_share")})
