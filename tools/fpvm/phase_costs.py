#!/usr/bin/env python
"""Join a GPU phase trace (tools/vm_trace.py) with the generated programs' per-phase op mix
and fit the cost of each interpreter code path (least squares on path-presence features:
a divergent wave pays for every path any of its lanes takes).

    python tools/fpvm/phase_costs.py gpurun_out/r01f/trace.npz [vote final]
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import gen  # noqa: E402
import sched  # noqa: E402


def _s5(x):
    return x - 32 if x & 16 else x


def lane_paths(w):
    """Interpreter code paths (fpvm.hpp exec) one encoded instruction (w0..w3) takes."""
    opc = w[0] & 31
    k = {v: n for n, v in sched.OPC.items()}[opc]
    if k == "nop":
        return set()
    if k in ("st", "selb", "sel", "inv"):
        return {"rare", k}
    if k in ("and", "or", "xor"):
        return {"rare", "logic"}
    ca, cb, cc, cd = (_s5((w[3] >> (5 * q)) & 31) for q in range(4))
    if k == "lin":
        unit = ca == 1 and all(-1 <= x <= 1 for x in (cb, cc, cd))
        if not unit:
            return {"rare", "lin_acc"}
        p = {"lin"}
        if cb < 0 or cc < 0 or cd < 0:
            p.add("lin_neg")
        if (w[3] >> 20) & 15 > 1:
            p.add("lin_scale")
        return p
    p = {"mul"}
    if cb < 0 or cd < 0:
        p.add("mul_neg")
    if k != "muls":
        p.add("flag")
    return p


def features(sc, words):
    rows = []
    W = sc.W
    for t in range(sc.nrounds):
        s = set()
        for lane in range(W):
            s |= lane_paths(words[(t * W + lane) * 4:(t * W + lane) * 4 + 4])
        rows.append(s)
    names = sorted(set().union(*rows))
    X = np.zeros((len(rows), len(names) + 1))
    X[:, -1] = 1.0
    for t, s in enumerate(rows):
        for n in s:
            X[t, names.index(n)] = 1.0
    return names + ["base"], X


def main():
    path = sys.argv[1]
    which = sys.argv[2:] or ["vote", "final"]
    tr = np.load(path)
    consts, built = gen.build_all()
    for name in which:
        prog, sc, words, ins, outs = built[name]
        st = tr[name].astype(np.int64)
        d = np.diff(st) * 10.0  # ns (100 MHz clock)
        if len(d) != sc.nrounds:
            print("%s: trace has %d phases, program %d -- stale trace?" % (name, len(d), sc.nrounds))
            continue
        names, X = features(sc, words)
        coef, *_ = np.linalg.lstsq(X, d, rcond=None)
        pred = X @ coef
        print("== %s: %d phases, %.3f ms measured, fit rms %.0f ns" %
              (name, len(d), d.sum() / 1e6, np.sqrt(np.mean((pred - d) ** 2))))
        cnt = X.sum(axis=0)
        order = np.argsort(-(coef * cnt))
        for j in order:
            print("  %-14s %7.0f ns x %5d phases = %7.3f ms" % (names[j], coef[j], cnt[j], coef[j] * cnt[j] / 1e6))


if __name__ == "__main__":
    main()
