#!/usr/bin/env python
"""Summarise the PMC passes of tools/evidence.sh (tools/pmc_round.sh + tools/pmc_vote.sh) for one
tag: per-kernel HBM bytes per launch of the 4096-vote workload (FETCH_SIZE x 2 + WRITE_SIZE, the
gfx950 correction of MI355X_MICROARCH.md) -> consensus_overlord_amd/pmc_traffic.json (bench.py's
roofline.traffic), and per-wave SQ / LDS counters -> profiles/<tag>_pmc_per_wave.json.

    python tools/pmc_summary.py r02am
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the 4096-vote launches (grid size in threads) of the kernels reported
GRIDS = {"k_h2f": 4096, "k_vm_vote": 65536, "k_msm_pair<8, 0>": 139264, "k_msm_pair<8, 1>": 73728,
         "k_msm_pair<8, 2>": 16384, "k_msm_scatter": 4096, "k_vm_final": 64}


def load(pattern):
    """{(kernel, grid): {counter: [values]}}"""
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in glob.glob(pattern):
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            out[(k, int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return out


def mean(v):
    return sum(v) / len(v)


def main(tag):
    base = os.path.join(ROOT, "gpurun_out", tag)
    fetch = load(os.path.join(base, "pmc", "fetch", "*counter_collection.csv"))
    write = load(os.path.join(base, "pmc", "write", "*counter_collection.csv"))
    traffic = {}
    for k, g in GRIDS.items():
        f, w = fetch.get((k, g), {}).get("FETCH_SIZE"), write.get((k, g), {}).get("WRITE_SIZE")
        if f and w:
            traffic[k] = {"grid": g, "launches": len(f), "FETCH_SIZE": round(mean(f), 3), "WRITE_SIZE": round(mean(w), 3),
                          "hbm_bytes_per_launch": int((2 * mean(f) + mean(w)) * 1024)}
    doc = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes (tools/pmc_round.sh) over bench.py "
                     "--steps 2 --warmup 1, %s build; per-dispatch averages (KB as reported) of the 4096-vote "
                     "launches (grid sizes as listed)" % tag,
           "correction": "gfx950: FETCH_SIZE counts 64 B per 128-B request, so hbm_bytes = (2 x FETCH_SIZE + "
                         "WRITE_SIZE) x 1024 (MI355X_MICROARCH.md HBM/rocprofv3 section)",
           "kernels": traffic}
    with open(os.path.join(ROOT, "consensus_overlord_amd", "pmc_traffic.json"), "w") as fh:
        json.dump(doc, fh, indent=1)
    srcs = [load(os.path.join(base, "pmc", "sq", "*counter_collection.csv"))] + \
        [load(os.path.join(base, "pmcv", x, "*counter_collection.csv")) for x in "abc"]
    per_wave = {}
    for k, g in GRIDS.items():
        d = {}
        for src in srcs:
            for cn, vals in src.get((k, g), {}).items():
                d[cn] = mean(vals)
        if not d:
            continue
        waves = d.get("SQ_WAVES", 1.0)
        e = {cn: round(v / waves, 1) for cn, v in d.items() if cn != "SQ_WAVES"}
        e["SQ_WAVES"] = waves
        per_wave["%s grid %d" % (k, g)] = e
    with open(os.path.join(ROOT, "profiles", "%s_pmc_per_wave.json" % tag), "w") as fh:
        json.dump({"source": "rocprofv3 --pmc passes (tools/pmc_round.sh, tools/pmc_vote.sh) over bench.py --steps 2 "
                             "--warmup 1, %s build; per-dispatch counter values divided by SQ_WAVES" % tag,
                   "kernels": per_wave}, fh, indent=1)
    print(json.dumps(traffic, indent=1))
    print(json.dumps(per_wave.get("k_vm_vote grid 65536"), indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
