#!/usr/bin/env python
"""Summarise tools/pmc_pool.sh's passes for one tag: the vote pool's counters per quad (one quad =
one wave's 4 votes through the vote program, the pool's unit of work) over the pre-published
diagnostic (6 batches x 1,024 quads), HBM bytes per batch (FETCH_SIZE x 2 + WRITE_SIZE, the gfx950
correction of MI355X_MICROARCH.md), and the static v_mad_u64_u32 count per quad from the vote
program's schedule. Writes consensus_overlord_amd/pmc_pool.json (read by bench.py for
roofline.pmc) and profiles/<tag>_pmc_pool.json.

    python tools/pmc_pool_summary.py r05ad
"""
import collections
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BATCHES, QUADS_PER_BATCH = 6, 1024


def pool_totals(path):
    tot = collections.defaultdict(float)
    disp = set()
    for f in glob.glob(path):
        for r in csv.DictReader(open(f)):
            if "k_vm_pool" in r["Kernel_Name"]:
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
                disp.add(r["Dispatch_Id"])
    return tot, len(disp)


def product_phases():
    """(product phases, lin_mad phases, unit-lin phases) of the vote program from the scheduled
    stream's stats line in vm_progs.inc"""
    inc = open(os.path.join(ROOT, "consensus_overlord_amd", "csrc", "vm_progs.inc")).read()
    m = re.search(r"^// vote: (\{.*\})$", inc, flags=re.M)
    return json.loads(m.group(1))


def main(tag):
    base = os.path.join(ROOT, "gpurun_out", tag, "pmcpool")
    a, na = pool_totals(os.path.join(base, "a", "*counter_collection.csv"))
    b, nb = pool_totals(os.path.join(base, "b", "*counter_collection.csv"))
    f, _ = pool_totals(os.path.join(base, "fetch", "*counter_collection.csv"))
    w, _ = pool_totals(os.path.join(base, "write", "*counter_collection.csv"))
    quads = BATCHES * QUADS_PER_BATCH
    st = product_phases()
    per_quad = {k: round(v / quads, 1) for k, v in sorted({**a, **b}.items()) if k != "SQ_WAVES"}
    mad_static = st["heavy_phases"] * 392
    doc = {
        "source": "rocprofv3 --pmc passes (tools/pmc_pool.sh, one run per counter group) over tools/pool_probe.py "
                  "4096 6 2 (prog 2: six 4,096-vote batches published before the pool's two grids start), %s build; "
                  "totals over the pool's dispatches / %d quads" % (tag, quads),
        "dispatches": na,
        "quads": quads,
        "per_quad": per_quad,
        "valu_per_quad": per_quad.get("SQ_INSTS_VALU"),
        "lanes_per_valu": round(b["SQ_THREAD_CYCLES_VALU"] / b["SQ_ACTIVE_INST_VALU"], 2)
        if b.get("SQ_ACTIVE_INST_VALU") else None,
        "lds_bank_conflict_share": round(b["SQ_LDS_BANK_CONFLICT"] / b["SQ_LDS_IDX_ACTIVE"], 4)
        if b.get("SQ_LDS_IDX_ACTIVE") else None,
        "wait_any_share": round(a["SQ_WAIT_ANY"] / a["SQ_WAVE_CYCLES"], 4) if a.get("SQ_WAVE_CYCLES") else None,
        "wait_basis": "SQ_WAIT_ANY / SQ_WAVE_CYCLES under rocprofv3's serialised dispatches: the pool's two grids "
                      "then run one after the other, so this is the share at the first grid's occupancy "
                      "(896 workgroups: 3 or 4 of a CU's 8 places, one wave on most SIMDs), not the pipelined one",
        "mad_per_quad_static": mad_static,
        "mad_basis": "392 v_mad_u64_u32 per product phase (csrc/bls/fp_mul28_gfx950.hpp) x the vote program's "
                     "product phases (vm_progs.inc stats); the lin_mad / scale_reduce mads are not counted",
        "int64_per_quad": per_quad.get("SQ_INSTS_VALU_INT64"),
        "hbm_bytes_per_batch": int((2 * f.get("FETCH_SIZE", 0) + w.get("WRITE_SIZE", 0)) * 1024 / BATCHES),
        "fetch_kb_per_batch": round(f.get("FETCH_SIZE", 0) / BATCHES, 1),
        "write_kb_per_batch": round(w.get("WRITE_SIZE", 0) / BATCHES, 1),
        "traffic_basis": "(2 x FETCH_SIZE + WRITE_SIZE) x 1 KiB per 4,096-vote batch (gfx950 FETCH_SIZE correction)",
        "schedule": st,
    }
    for out in (os.path.join(ROOT, "consensus_overlord_amd", "pmc_pool.json"),
                os.path.join(ROOT, "profiles", "%s_pmc_pool.json" % tag)):
        with open(out, "w") as fh:
            json.dump(doc, fh, indent=1)
    print(json.dumps({k: v for k, v in doc.items() if k not in ("schedule", "per_quad")}))


if __name__ == "__main__":
    main(sys.argv[1])
