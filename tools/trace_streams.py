#!/usr/bin/env python
"""Summarise a rocprofv3 --kernel-trace CSV by stream: per kernel its count and mean duration,
per stream its busy time, and for each listed kernel the gaps and overlaps between consecutive
launches (which stream limits a pipelined loop).   python tools/trace_streams.py <kernel_trace.csv> [kernel ...]"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    m = re.match(r"(?:void )?([A-Za-z_0-9]+)", name)
    return m.group(1) if m else name[:40]


def main():
    path = sys.argv[1]
    watch = sys.argv[2:] or ["k_vm_vsame", "k_vm_h2g", "k_vm_gfin"]
    rows = list(csv.DictReader(open(path)))
    sk = "Stream_Id" if "Stream_Id" in rows[0] else "Queue_Id"
    ks = defaultdict(list)
    busy = defaultdict(float)
    t0 = min(int(r["Start_Timestamp"]) for r in rows)
    t1 = max(int(r["End_Timestamp"]) for r in rows)
    for r in rows:
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        ks[short(r["Kernel_Name"])].append((a, b, r[sk]))
        busy[r[sk]] += (b - a) / 1e6
    print("span %.3f ms" % ((t1 - t0) / 1e6))
    for k, v in sorted(ks.items(), key=lambda kv: -sum(b - a for a, b, _ in kv[1])):
        d = [(b - a) / 1e6 for a, b, _ in v]
        print("%-28s n=%4d mean %.4f ms total %.3f ms streams %s" % (k, len(v), sum(d) / len(d), sum(d),
                                                                  sorted(set(s for _, _, s in v))))
    for s, b in sorted(busy.items()):
        print("stream %s busy %.3f ms" % (s, b))
    for k in watch:
        v = sorted(ks.get(k, []))
        print(k, " ".join("%.2f-%.2f" % ((a - t0) / 1e6, (b - t0) / 1e6) for a, b, _ in v))


if __name__ == "__main__":
    main()
