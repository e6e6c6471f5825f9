#!/usr/bin/env python
"""Summarise a rocprofv3 --kernel-trace --stats run (rocpd SQLite .db, or the CSV
kernel_stats/kernel_trace files) into a markdown table: per kernel calls, average / total
duration, VGPRs, SGPRs, scratch bytes per lane, grid and workgroup size."""
import csv
import glob
import os
import sqlite3
import sys


def from_db(path):
    c = sqlite3.connect(path)
    q = ("select name, count(*), avg(duration), sum(duration), vgpr_count, sgpr_count, scratch_size, "
         "grid_x, workgroup_x from kernels group by name order by sum(duration) desc")
    return [list(r) for r in c.execute(q)]


def from_csv(d):
    tr = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    rows = {}
    for f in tr:
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            e = rows.setdefault(name, [name, 0, 0.0, 0.0, r.get("VGPR_Count") or r.get("Arch_VGPR_Count"),
                                       r.get("SGPR_Count"), r.get("Scratch_Size") or r.get("Private_Segment_Size"),
                                       r.get("Grid_Size_X") or r.get("Grid_Size"), r.get("Workgroup_Size_X") or r.get("Workgroup_Size")])
            e[1] += 1
            e[3] += dur
    out = []
    for e in rows.values():
        e[2] = e[3] / e[1]
        out.append(e)
    return sorted(out, key=lambda e: -e[3])


def main():
    src = sys.argv[1]
    rows = from_db(src) if src.endswith(".db") else from_csv(src)
    tot = sum(r[3] for r in rows)
    print("| kernel | calls | avg us | total ms | % | VGPR | SGPR | scratch B/lane | grid | wg |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for r in rows:
        name = r[0].split("(")[0]
        if len(name) > 60:
            name = name[:57] + "..."
        print("| %s | %d | %.1f | %.3f | %.1f | %s | %s | %s | %s | %s |" % (
            name, r[1], r[2] / 1e3, r[3] / 1e6, 100.0 * r[3] / tot, r[4], r[5], r[6], r[7], r[8]))


if __name__ == "__main__":
    main()
