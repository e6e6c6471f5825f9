#!/usr/bin/env python3
"""Generate consensus_overlord_amd/csrc/bls/fp_mul28_gfx950.hpp: the gfx950 Montgomery product on
14 x 28-bit limbs as product scanning with ONE 64-bit accumulator (v[252:253]) in one asm
statement.

Cost model (measured, tools/ubench/fp_mul28.hip + profiles/r01_int_rates_ubench.json): a
v_mad_u64_u32 issues in ~5.4 cycles per wave, other VALU ops in 4. The 12 x 32 form pays 288 mads
+ 288 v_addc (the 96-bit accumulator's third word) + 46 moves per product; here every column of
<= 28 products of 28-bit limbs fits 64 bits (< 2^61 with the carry), so each partial product is
one mad and the column shift is one v_lshrrev_b64: 392 mads + 14 x (mul_lo, and) + 13 ands +
27 shifts. The split of the inputs into 28-bit limbs (a shifted left by 8: with R = 2^392 the
result is a b 2^-384), the join back to 12 x 32 and the final conditional subtraction are C++.
"""
import os

N = 14
ACC, ACC_LO = "v[252:253]", "v252"


def body_1acc():
    """One accumulator: every op depends on the one before (a single chain)."""
    lines = []
    first = True
    for k in range(2 * N - 1):
        terms = [("x%d" % i, "y%d" % (k - i)) for i in range(N) if 0 <= k - i < N]
        terms += [("m%d" % i, "p%d" % (k - i)) for i in range(N) if i < k and 1 <= k - i < N]
        for a, b in terms:
            src = "0" if first else ACC
            lines.append("v_mad_u64_u32 %s, vcc, %%[%s], %%[%s], %s" % (ACC, a, b, src))
            first = False
        if k < N:
            lines.append("v_mul_lo_u32 %%[m%d], %s, %%[pinv]" % (k, ACC_LO))
            lines.append("v_and_b32_e32 %%[m%d], %%[mask], %%[m%d]" % (k, k))
            lines.append("v_mad_u64_u32 %s, vcc, %%[m%d], %%[p0], %s" % (ACC, k, ACC))
        else:
            lines.append("v_and_b32_e32 %%[t%d], %%[mask], %s" % (k - N, ACC_LO))
        lines.append("v_lshrrev_b64 %s, 28, %s" % (ACC, ACC))
    lines.append("v_mov_b32 %%[t%d], %s" % (N - 1, ACC_LO))
    return lines, ["v252", "v253"]


ACC2 = "v[250:251]"


def body_2acc():
    """Two accumulators: a column's products alternate between ACC (which carries the shifted
    previous column) and ACC2 (fresh from 0), joined by one 64-bit add before the column's
    Montgomery digit; the next column's first products (all but m_k p_1, which needs the digit)
    go to ACC2 between the dependent steps of the digit (mul_lo, and, mad, shift), so at one
    wave per SIMD the in-order issue rarely waits on a result (the one-chain form measured ~15%
    slower at 1 wave than at 4 per SIMD, tools/ubench/fp_mul28.hip)."""
    lines = []
    serial = []            # the previous column's digit steps, not yet emitted
    for k in range(2 * N - 1):
        terms = [("x%d" % i, "y%d" % (k - i)) for i in range(N) if 0 <= k - i < N]
        terms += [("m%d" % i, "p%d" % (k - i)) for i in range(N) if i < k and 1 <= k - i < N]
        late = [t for t in terms if t[0] == "m%d" % (k - 1)]          # needs the previous digit
        early = [t for t in terms if t not in late]
        b_used = False
        a_init = k > 0
        # interleave: digit step, ACC2 product, digit step, ...
        while serial:
            lines.append(serial.pop(0))
            if early and k > 0:
                a, b = early.pop(0)
                lines.append("v_mad_u64_u32 %s, vcc, %%[%s], %%[%s], %s" % (ACC2, a, b, ACC2 if b_used else "0"))
                b_used = True
        rest = early + late
        for j, (a, b) in enumerate(rest):
            use_a = (j % 2 == 0)
            if use_a:
                lines.append("v_mad_u64_u32 %s, vcc, %%[%s], %%[%s], %s" % (ACC, a, b, ACC if a_init else "0"))
                a_init = True
            else:
                lines.append("v_mad_u64_u32 %s, vcc, %%[%s], %%[%s], %s" % (ACC2, a, b, ACC2 if b_used else "0"))
                b_used = True
        if b_used:
            lines.append("v_lshl_add_u64 %s, %s, 0, %s" % (ACC, ACC2, ACC))
        if k < N:
            serial = ["v_mul_lo_u32 %%[m%d], %s, %%[pinv]" % (k, ACC_LO),
                      "v_and_b32_e32 %%[m%d], %%[mask], %%[m%d]" % (k, k),
                      "v_mad_u64_u32 %s, vcc, %%[m%d], %%[p0], %s" % (ACC, k, ACC),
                      "v_lshrrev_b64 %s, 28, %s" % (ACC, ACC)]
        else:
            serial = ["v_and_b32_e32 %%[t%d], %%[mask], %s" % (k - N, ACC_LO),
                      "v_lshrrev_b64 %s, 28, %s" % (ACC, ACC)]
    lines += serial
    lines.append("v_mov_b32 %%[t%d], %s" % (N - 1, ACC_LO))
    return lines, ["v250", "v251", "v252", "v253"]


def emit_fn(e, name, lines, clob):
    outs = ['[m%d] "=&v"(m[%d])' % (i, i) for i in range(N)] + ['[t%d] "=&v"(t[%d])' % (i, i) for i in range(N)]
    ins = ['[x%d] "v"(x[%d])' % (i, i) for i in range(N)] + ['[y%d] "v"(y[%d])' % (i, i) for i in range(N)] + \
        ['[p%d] "s"(P28[%d])' % (i, i) for i in range(N)] + ['[pinv] "s"(PINV28)', '[mask] "v"(M28)']
    e("__device__ __forceinline__ void %s(uint32_t* __restrict__ r, const uint32_t* __restrict__ a," % name)
    e("%s const uint32_t* __restrict__ b) {" % (" " * (len(name) + 24)))
    e("  uint32_t x[14], y[14], m[14], t[14];")
    e("  split28<8>(x, a);")
    e("  split28<0>(y, b);")
    e("  asm volatile(")
    for k in range(0, len(lines), 8):
        e('      "%s\\n\\t"' % "\\n\\t".join(lines[k:k + 8]))
    e("      : " + ", ".join(outs))
    e("      : " + ", ".join(ins))
    e('      : "vcc", %s);' % ", ".join('"%s"' % c for c in clob))
    e("  (void)m;")
    e("  join28_reduce(r, t);")
    e("}")


def main():
    out = []
    e = out.append
    e("// GENERATED by tools/gen_fpmul28.py -- do not edit.")
    e("// gfx950 Montgomery product on 14 x 28-bit limbs: product scanning with 64-bit accumulators")
    e("// in one inline-asm statement; split / join / conditional subtraction in C++ (fp_mul28.hpp).")
    e("// fp_mul28_gfx950_1acc: one accumulator (v[252:253]); fp_mul28_gfx950_2acc: two (v[250:253]),")
    e("// see the generator for the issue order.")
    e("#pragma once")
    e("#include <stdint.h>")
    e("#include \"fp_mul28.hpp\"")
    e("namespace ovh {")
    n = {}
    for name, fn in (("fp_mul28_gfx950_1acc", body_1acc), ("fp_mul28_gfx950_2acc", body_2acc)):
        lines, clob = fn()
        n[name] = len(lines)
        emit_fn(e, name, lines, clob)
    e("// one-chain order by default: the two-accumulator order measured 1.5% slower in the vote kernel")
    e("// (profiles/r03g_ab_summary.txt) and 5% slower at 4 waves per SIMD (r03g fp_mul28 ubench)")
    e("#if defined(OVH_FPMUL28_2ACC)")
    e("__device__ __forceinline__ void fp_mul28_gfx950(uint32_t* r, const uint32_t* a, const uint32_t* b) {")
    e("  fp_mul28_gfx950_2acc(r, a, b);")
    e("}")
    e("#else")
    e("__device__ __forceinline__ void fp_mul28_gfx950(uint32_t* r, const uint32_t* a, const uint32_t* b) {")
    e("  fp_mul28_gfx950_1acc(r, a, b);")
    e("}")
    e("#endif")
    e("}  // namespace ovh")
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "consensus_overlord_amd", "csrc", "bls",
                        "fp_mul28_gfx950.hpp")
    with open(path, "w") as fh:
        fh.write("\n".join(out) + "\n")
    print("wrote", os.path.normpath(path), n, "instructions")


if __name__ == "__main__":
    main()
