#!/usr/bin/env python3
"""VALU attribution of the vote program: where the pool kernel's VALU
instructions per quad go, by interpreter path.

    python tools/valu_attr.py [--inc consensus_overlord_amd/csrc/vm_progs.inc] [--build r06] [--md]

Two inputs:
  * how often each interpreter path runs: from the encoded vote program itself (vm_progs.inc
    VM_VOTE_CODE / VM_VOTE_SIDE) -- the phase header bits (fpvm.hpp exec: H_MUL, H_MULNEG,
    H_FLAG, H_LIN, H_LINNEG, H_ACC, H_RARE, H_SELB; one wave runs a block when any lane of the
    phase needs it), the lanes' opcodes for per-lane branches (lex / eq / st), and the side
    words (spills of the phase, fills of the next phase, whose loads the phase issues);
  * how many VALU instructions one pass of each path issues: counted in the gfx950 ISA of
    k_vm_pool's vote loop (hipcc --cuda-device-only -S of csrc/ovhip.hip, the blocks of
    vote_quad<false>'s vm::run<true>), one table per build below.
The product of the two, summed, is the static VALU count per vote program run = per quad (one
wave runs the four slices); tools/pmc_pool_summary.py's SQ_INSTS_VALU per quad measures the same
quantity on the GPU (r05ad: 1.258 M), which pins the table.
"""
from __future__ import annotations

import argparse
import os
import re
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

H_MUL, H_MULNEG, H_FLAG, H_LIN, H_LINNEG, H_ACC, H_RARE, H_SELB = (1 << k for k in range(22, 30))
H_LINNEG2, H_LINNEG3 = 1 << 30, 1 << 31
H_ANY = H_MUL | H_LIN | H_ACC | H_RARE
OPC = {"nop": 0, "muls": 1, "sgn0": 2, "lex": 3, "inv": 4, "lin": 5, "sel": 6, "eq": 7, "and": 8, "or": 9,
       "xor": 10, "st": 11, "selb": 12}

# VALU instructions per pass of each path, per build (ISA block counts).
# class: what the instructions do -- "mac" the v_mad_u64_u32 of the Montgomery product, the rest
# overhead to be cut.
PATHS = {
    "r05": {
        # every phase
        "loop: prefetch ring rotation + loop test": (12, "ring"),
        "loop: instruction / side-word prefetch": (6, "fetch"),
        "fill load issue (next phase fills)": (4, "spill"),
        # H_ANY
        "decode (opcode, dst, imm, coefficients)": (10, "decode"),
        "selb operand rewrite (H_SELB)": (10, "decode"),
        "operand addresses (4 x select + mad)": (24, "address"),
        # H_MUL
        "pre-add, unit signs": (24, "preadd"),
        "pre-add with 2p - x negations (H_MULNEG)": (77, "preadd"),
        "product: v_mad_u64_u32": (392, "mac"),
        "product: split 12x32 -> 14x28": (52, "split"),
        "product: Montgomery digits (mul_lo, and)": (28, "digits"),
        "product: column shifts (lshrrev_b64) + moves": (36, "digits"),
        "product: join 14x28 -> 12x32": (24, "join"),
        "product: conditional subtraction": (26, "condsub"),
        "flag ops (sgn0 / eq / lex, H_FLAG)": (25, "flag"),
        "lex compare (a lane with lex)": (24, "flag"),
        "result store address": (2, "store"),
        # H_LIN / H_ACC / H_RARE
        "lin dispatch (unit / general)": (10, "lin"),
        "lin_sum, unit signs": (37, "lin"),
        "lin_sum with negations (H_LINNEG)": (94, "lin"),
        "scale_reduce + store": (59, "lin"),
        "lin_mad (general coefficients, H_ACC)": (174, "lin"),
        "rare ops (st / sel / logic)": (45, "rare"),
        # side ops
        "spill (slot -> scratch)": (7, "spill"),
        "fill write (scratch -> slot)": (2, "spill"),
    },
    # r06 interpreter (fpvm.hpp): one / two-deep prefetch rings, bfe / bfi operand addresses,
    # negations on y only, per-block field decoding
    "r06": {
        "lin_sum with negations, D only (r06x)": (94, "lin"),
        "lin_sum with negations, C and D (r06x)": (94, "lin"),
        "loop: prefetch ring rotation + loop test": (4, "ring"),
        "loop: instruction / side-word prefetch": (4, "fetch"),
        "fill load issue (next phase fills)": (4, "spill"),
        "decode (opcode, dst, imm, coefficients)": (5, "decode"),
        "selb operand rewrite (H_SELB)": (9, "decode"),
        "operand addresses (4 x select + mad)": (17, "address"),
        "pre-add, unit signs": (24, "preadd"),
        "pre-add with 2p - x negations (H_MULNEG)": (51, "preadd"),
        "product: v_mad_u64_u32": (392, "mac"),
        "product: split 12x32 -> 14x28": (52, "split"),
        "product: Montgomery digits (mul_lo, and)": (28, "digits"),
        "product: column shifts (lshrrev_b64) + moves": (36, "digits"),
        "product: join 14x28 -> 12x32": (24, "join"),
        "product: conditional subtraction": (26, "condsub"),
        "flag ops (sgn0 / eq / lex, H_FLAG)": (28, "flag"),
        "lex compare (a lane with lex)": (24, "flag"),
        "result store address": (3, "store"),
        "lin dispatch (unit / general)": (2, "lin"),
        "lin_sum, unit signs": (37, "lin"),
        "lin_sum with negations (H_LINNEG)": (94, "lin"),
        "scale_reduce + store": (59, "lin"),
        "lin_mad (general coefficients, H_ACC)": (179, "lin"),
        "rare ops (st / sel / logic)": (45, "rare"),
        "spill (slot -> scratch)": (7, "spill"),
        "fill write (scratch -> slot)": (2, "spill"),
    },
}
# r06x: lin_sum XORs only the positions some lane negates (H_LINNEG2 / H_LINNEG3; 12 VALU each)
PATHS["r06x"] = dict(PATHS["r06"])
PATHS["r06x"]["lin_sum with negations, D only (r06x)"] = (70, "lin")
PATHS["r06x"]["lin_sum with negations, C and D (r06x)"] = (82, "lin")


def load_prog(inc, name="VOTE"):
    text = open(inc).read()

    def arr(tag):
        m = re.search(r"static const uint32_t VM_%s_%s\[(\d+)\] = \{(.*?)\};" % (name, tag), text, flags=re.S)
        return [int(x, 16) for x in m.group(2).replace("\n", "").split(",") if x.strip()]
    w = int(re.search(r"#define VM_%s_W (\d+)" % name, text).group(1))
    nph = int(re.search(r"#define VM_%s_NPHASES (\d+)" % name, text).group(1))
    return w, nph, arr("CODE"), arr("SIDE")


def phase_counts(w, nph, code, side):
    """Per path: the number of phases in which one wave runs it."""
    c = Counter()
    for t in range(nph):
        lanes = [code[(t * w + l) * 4:(t * w + l) * 4 + 4] for l in range(w)]
        hdr = lanes[0][0]
        ops = {x[0] & 31 for x in lanes}
        sw = side[t * w:(t + 1) * w]
        nxt = side[(t + 1) * w:(t + 2) * w] if t + 1 < nph else []
        c["loop: prefetch ring rotation + loop test"] += 1
        c["loop: instruction / side-word prefetch"] += 1
        if any(s >> 31 and (s >> 30) & 1 for s in nxt):
            c["fill load issue (next phase fills)"] += 1
            c["fill write (scratch -> slot)"] += 1
        if any(s >> 31 and not (s >> 30) & 1 for s in sw):
            c["spill (slot -> scratch)"] += 1
        if not hdr & H_ANY:
            continue
        c["decode (opcode, dst, imm, coefficients)"] += 1
        c["operand addresses (4 x select + mad)"] += 1
        if hdr & H_SELB:
            c["selb operand rewrite (H_SELB)"] += 1
        if hdr & H_MUL:
            c["pre-add with 2p - x negations (H_MULNEG)" if hdr & H_MULNEG else "pre-add, unit signs"] += 1
            for k in ("product: v_mad_u64_u32", "product: split 12x32 -> 14x28", "product: Montgomery digits (mul_lo, and)",
                      "product: column shifts (lshrrev_b64) + moves", "product: join 14x28 -> 12x32",
                      "product: conditional subtraction", "result store address"):
                c[k] += 1
            if hdr & H_FLAG:
                c["flag ops (sgn0 / eq / lex, H_FLAG)"] += 1
                if OPC["lex"] in ops:
                    c["lex compare (a lane with lex)"] += 1
        c["lin dispatch (unit / general)"] += 1
        if hdr & H_LIN:
            if not hdr & H_LINNEG:
                c["lin_sum, unit signs"] += 1
            elif hdr & H_LINNEG3:
                c["lin_sum with negations (H_LINNEG)"] += 1
            elif hdr & H_LINNEG2:
                c["lin_sum with negations, C and D (r06x)"] += 1
            else:
                c["lin_sum with negations, D only (r06x)"] += 1
            c["scale_reduce + store"] += 1
        if hdr & H_ACC:
            c["lin_mad (general coefficients, H_ACC)"] += 1
        if hdr & H_RARE:
            c["rare ops (st / sel / logic)"] += 1
    return c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--inc", default=os.path.join(ROOT, "consensus_overlord_amd", "csrc", "vm_progs.inc"))
    ap.add_argument("--build", default=max(PATHS))
    ap.add_argument("--md", action="store_true")
    a = ap.parse_args()
    w, nph, code, side = load_prog(a.inc)
    cnt = phase_counts(w, nph, code, side)
    cost = PATHS[a.build]
    rows = [(k, cnt[k], v, cls, cnt[k] * v) for k, (v, cls) in cost.items()]
    total = sum(r[4] for r in rows)
    by_cls = Counter()
    for r in rows:
        by_cls[r[3]] += r[4]
    if a.md:
        print("| path | phases | VALU / pass | VALU / quad | share |")
        print("|---|---:|---:|---:|---:|")
        for k, n, v, cls, tot in sorted(rows, key=lambda r: -r[4]):
            print("| %s | %d | %d | %d | %.1f%% |" % (k, n, v, tot, 100.0 * tot / total))
        print("| **total** | %d | | **%d** | |" % (nph, total))
        print()
        print("| class | VALU / quad | share |")
        print("|---|---:|---:|")
        for cls, tot in by_cls.most_common():
            print("| %s | %d | %.1f%% |" % (cls, tot, 100.0 * tot / total))
    else:
        for k, n, v, cls, tot in sorted(rows, key=lambda r: -r[4]):
            print("%-48s %5d x %4d = %8d  %5.1f%%" % (k, n, v, tot, 100.0 * tot / total))
        print("total VALU per quad (static): %d over %d phases" % (total, nph))
        for cls, tot in by_cls.most_common():
            print("  %-10s %8d  %5.1f%%" % (cls, tot, 100.0 * tot / total))


if __name__ == "__main__":
    main()
