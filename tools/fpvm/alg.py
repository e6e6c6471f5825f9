"""Branch-free BLS12-381 algorithms traced into the Fp-VM IR (ir.py).

These restate, over traced Fp values, the arithmetic of the CPU oracle
(oracle/py/bls12_381.py -- itself pinned to RFC 9380 and the generator KATs), in forms that
suit a lane-parallel straight-line program:

  * tower Fp2/Fp6/Fp12 (same basis as the oracle), Granger-Scott cyclotomic squaring;
  * branch-free Fp2 square root (norm method, one select);
  * complete projective point formulas (Renes-Costello-Batina 2016, a = 0), so adversarial
    non-subgroup points need no exceptional-case branches;
  * RFC 9380 simplified SWU with the generic sqrt_ratio (Appendix F.2.1.1), 3-isogeny
    homogenised (no inversion), Budroni-Pintore cofactor clearing;
  * optimal-ate Miller loop with T and Q in homogeneous projective coordinates (line scalings
    lie in Fp2 and are removed by the final exponentiation), x-chain final exponentiation.

Every function returns traced values; data-dependent choices are `sel` ops.
"""
from __future__ import annotations

import os
import sys

from ir import P, Prog

X_ABS = 0xD201000000010000
R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
# RLC scalar of a vote: r = a + b * LAMBDA (mod r) with a = bits 0..31, b = bits 32..63 of its
# 64-bit SplitMix64 value. LAMBDA = -x^2 is the eigenvalue of phi on G1 (phi(P) = [-x^2] P)
# and of -psi^2 on G2 (psi(Q) = [x] Q), so [r] P = [a] P + [b] phi(P) and
# [r] Q = [a] Q + [b] (-psi^2(Q)): one 32-step chain instead of 64. The 2^64 (a, b) pairs give
# distinct r (no (da, db) with |da|, |db| < 2^32 has da = LAMBDA db mod r), so the batch check's
# soundness stays 2^-64.
LAMBDA = (-X_ABS * X_ABS) % R_ORDER


def rlc_scalar(z: int) -> int:
    """The effective RLC scalar of a vote from its 64-bit value z."""
    return ((z & 0xFFFFFFFF) + (z >> 32) * LAMBDA) % R_ORDER


def _f2pow(a, e):
    """Python Fp2 power on (c0, c1) ints (constant derivation only)."""
    r = (1, 0)
    b = a
    while e:
        if e & 1:
            r = ((r[0] * b[0] - r[1] * b[1]) % P, (r[0] * b[1] + r[1] * b[0]) % P)
        b = ((b[0] * b[0] - b[1] * b[1]) % P, 2 * b[0] * b[1] % P)
        e >>= 1
    return r


def _f2inv(a):
    n = pow(a[0] * a[0] + a[1] * a[1], P - 2, P)
    return (a[0] * n % P, -a[1] * n % P)


XI = (1, 1)
GAMMA = [_f2pow(XI, k * (P - 1) // 6) for k in range(6)]
PSI_CX = _f2inv(_f2pow(XI, (P - 1) // 3))
PSI_CY = _f2inv(_f2pow(XI, (P - 1) // 2))
INV2 = pow(2, P - 2, P)

# SSWU on E2': A' = 240 u, B' = 1012 (1 + u), Z = -(2 + u)  (RFC 9380 8.8.2)
SSWU_A = (0, 240)
SSWU_B = (1012, 1012)
SSWU_Z = ((-2) % P, (-1) % P)
Q2 = P * P
SR_C1 = 3
assert (Q2 - 1) % 8 == 0 and ((Q2 - 1) // 8) % 2 == 1
SR_C2 = (Q2 - 1) >> SR_C1
SR_C3 = (SR_C2 - 1) // 2
SR_C4 = (1 << SR_C1) - 1
SR_C5 = 1 << (SR_C1 - 1)
SR_C6 = _f2pow(SSWU_Z, SR_C2)
SR_C7 = _f2pow(SSWU_Z, (SR_C2 + 1) // 2)


def _h(s):
    return int(s, 16)


# 3-isogeny E2' -> E2 (RFC 9380 E.3): coefficients k_0..k_n (Fp2 as (c0, c1))
ISO_XNUM = [
    (_h("5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6"),
     _h("5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6")),
    (0, _h("11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71a")),
    (_h("11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71e"),
     _h("8ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38d")),
    (_h("171d6541fa38ccfaed6dea691f5fb614cb14b4e7f4e810aa22d6108f142b85757098e38d0f671c7188e2aaaaaaaa5ed1"), 0),
]
ISO_XDEN = [
    (0, _h("1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaa63")),
    (0xC, _h("1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaa9f")),
    (1, 0),
]
ISO_YNUM = [
    (_h("1530477c7ab4113b59a4c18b076d11930f7da5d4a07f649bf54439d87d27e500fc8c25ebf8c92f6812cfc71c71c6d706"),
     _h("1530477c7ab4113b59a4c18b076d11930f7da5d4a07f649bf54439d87d27e500fc8c25ebf8c92f6812cfc71c71c6d706")),
    (0, _h("5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97be")),
    (_h("11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71c"),
     _h("8ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38f")),
    (_h("124c9ad43b6cf79bfbf7043de3811ad0761b0f37a1e26286b0e977c69aa274524e79097a56dc4bd9e1b371c71c718b10"), 0),
]
ISO_YDEN = [
    (_h("1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffa8fb"),
     _h("1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffa8fb")),
    (0, _h("1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffa9d3")),
    (0x12, _h("1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaa99")),
    (1, 0),
]

G1X = 0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB
G1Y = 0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1


def _beta():
    """Cube root of unity with phi(P) = (beta x, y) == [-x^2] P on G1 (checked on the generator
    with plain affine arithmetic)."""
    def add(p1, p2):
        if p1 is None:
            return p2
        if p2 is None:
            return p1
        (x1, y1), (x2, y2) = p1, p2
        if x1 == x2:
            if (y1 + y2) % P == 0:
                return None
            lam = 3 * x1 * x1 * pow(2 * y1, P - 2, P) % P
        else:
            lam = (y2 - y1) * pow(x2 - x1, P - 2, P) % P
        x3 = (lam * lam - x1 - x2) % P
        return (x3, (lam * (x1 - x3) - y1) % P)

    def mul(pt, k):
        acc = None
        for bit in bin(k)[2:]:
            acc = add(acc, acc)
            if bit == "1":
                acc = add(acc, pt)
        return acc
    g = (G1X, G1Y)
    t = mul(g, X_ABS * X_ABS)
    want = (t[0], (-t[1]) % P)
    b0 = pow(2, (P - 1) // 3, P)
    for b in (b0, b0 * b0 % P):
        if (G1X * b % P, G1Y) == want:
            return b
    raise AssertionError("beta")


BETA = _beta()


JAC_COFACTOR = True
YAO_POW = True        # sqrt_ratio's exponentiation by Yao's method (f2_pow_frob_yao)   # cofactor clearing's [|x|] chains in Jacobian coordinates (see g2_jac_dbl)


# RFC 9380 I.3 sqrt for q = 9 (mod 16), q = p^2: c1 = sqrt(-1) = u, c2 = sqrt(c1), c3 = sqrt(-c1)
SQ9_C2 = (0x6af0e0437ff400b6831e36d6bd17ffe48395dabc2d3435e77f76e17009241c5ee67992f72ec05f4c81084fbede3cc09,
          0x135203e60180a68ee2e9c448d77a2cd91c3dedd930b1cf60ef396489f61eb45e304466cf3e67fa0af1ee7b04121bdea2)
SQ9_C3 = (0x6af0e0437ff400b6831e36d6bd17ffe48395dabc2d3435e77f76e17009241c5ee67992f72ec05f4c81084fbede3cc09,
          0x6af0e0437ff400b6831e36d6bd17ffe48395dabc2d3435e77f76e17009241c5ee67992f72ec05f4c81084fbede3cc09)
SQ9_C4 = (P * P + 7) // 16


def _f2m(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


assert _f2m(SQ9_C2, SQ9_C2) == (0, 1) and _f2m(SQ9_C3, SQ9_C3) == (0, P - 1)


class Alg:
    def __init__(self, prog: Prog, inv_op: bool = False, use_sop: bool = False, fast_sqrt: bool = False):
        self.p = prog
        self.use_sop = use_sop   # Fp2 products as two sum-of-products ops (ir.Prog.sop)
        self.inv_op = inv_op   # Fp inversion by the interpreter's one-lane binary Euclid
        # Fp2 square roots by one Frobenius-split Yao exponentiation (f2_sqrt9): ~390 dependent
        # levels instead of the norm method's two Fp chains (~760), ~300 more products -- the
        # latency programs (one signature or one vote on the GPU) take it
        self.fast_sqrt = fast_sqrt

    # ---------------------------------------------------------------- Fp
    def c(self, v):
        return self.p.const(v)

    def c2(self, v):
        return (self.p.const(v[0]), self.p.const(v[1]))

    def fp_pow(self, a, e: int, w: int = 5):
        """a^e, left-to-right sliding window over precomputed odd powers."""
        p = self.p
        if e == 0:
            return p.one
        sq = a * a
        odd = [a]
        for _ in range((1 << (w - 1)) - 1):
            odd.append(odd[-1] * sq)
        bits = bin(e)[2:]
        acc = None
        i = 0
        while i < len(bits):
            if bits[i] == "0":
                acc = acc * acc
                i += 1
                continue
            j = min(i + w, len(bits))
            while bits[j - 1] == "0":
                j -= 1
            val = int(bits[i:j], 2)
            for _ in range(j - i):
                if acc is not None:
                    acc = acc * acc
            acc = odd[val >> 1] if acc is None else acc * odd[val >> 1]
            i = j
        return acc

    def fp_pow_yao(self, a, e: int, w: int = 3, LAG: int = 2):
        """a^e by Yao's right-to-left k-ary method (as f2_pow_frob_yao, in Fp): the squaring
        chain B_j = a^(2^(w j)) carries the critical path, each window digit d multiplies B_j
        into an accumulator X_d off that path, prod_d X_d^d closes."""
        pp = self.p
        mask = (1 << w) - 1
        nwin = (e.bit_length() + w - 1) // w
        X = [None] * (1 << w)
        B = a
        done = []
        for j in range(nwin):
            if j:
                deps = done[j - 1 - LAG] if j - 1 - LAG >= 0 else []
                if deps:   # the chain at most LAG windows ahead of the accumulations
                    B = pp._op("muls", (B.id, None, B.id, None), (1, 0, 1, 0), deps=tuple(v.id for v in deps))
                else:
                    B = B * B
                for _ in range(w - 1):
                    B = B * B
            d = (e >> (w * j)) & mask
            got = []
            if d:
                X[d] = B if X[d] is None else X[d] * B
                got.append(X[d])
            done.append(got)
        ys, y = [], None
        for d in range(mask, 0, -1):
            if X[d] is None:
                if y is not None:
                    ys.append(y)
                continue
            y = X[d] if y is None else y * X[d]
            ys.append(y)
        while len(ys) > 1:
            ys = [ys[k] * ys[k + 1] if k + 1 < len(ys) else ys[k] for k in range(0, len(ys), 2)]
        return ys[0]

    def fp_inv(self, a):
        if self.inv_op:
            return self.p.inv(a)
        return self.fp_pow(a, P - 2)

    # ---------------------------------------------------------------- Fp2 (tuples)
    def f2_add(self, a, b):
        return (a[0] + b[0], a[1] + b[1])

    def f2_sub(self, a, b):
        return (a[0] - b[0], a[1] - b[1])

    def f2_neg(self, a):
        return (-a[0], -a[1])

    def f2_dbl(self, a):
        return (a[0] + a[0], a[1] + a[1])

    def f2_conj(self, a):
        return (a[0], -a[1])

    def f2_mul(self, a, b):
        p = self.p
        if p.is_const(b[0]) and p.is_const(b[1]):
            return self.f2_mul_c(a, (p.cval(b[0]), p.cval(b[1])))
        if p.is_const(a[0]) and p.is_const(a[1]):
            return self.f2_mul_c(b, (p.cval(a[0]), p.cval(a[1])))
        if self.use_sop:   # schoolbook on two lanes: a0 b0 - a1 b1, a0 b1 + a1 b0 (no post-adds)
            return (p.sop(a[0], b[0], -1, a[1], b[1]), p.sop(a[0], b[1], 1, a[1], b[0]))
        t0 = a[0] * b[0]
        t1 = a[1] * b[1]
        t2 = p.muls(a[0], 1, a[1], b[0], 1, b[1])
        return (t0 - t1, p.lin4(t2, -1, t0, -1, t1))

    def f2_mul_c(self, a, k):
        """a * constant (k0 + k1 u)."""
        p = self.p
        k0, k1 = k[0] % P, k[1] % P
        if k1 == 0:
            return (a[0] * p.const(k0), a[1] * p.const(k0))
        if k0 == 0:
            return (-(a[1] * p.const(k1)), a[0] * p.const(k1))
        if k0 == k1 and k0 <= 15:  # small k (1 + u): linear combinations
            return (p.lin([(k0, a[0]), (-k0, a[1])]), p.lin([(k0, a[0]), (k0, a[1])]))
        if k0 == k1:  # k0 (1 + u): (a0 - a1) k0 + (a0 + a1) k0 u
            kk = p.const(k0)
            return (p.muls(a[0], -1, a[1], kk, 1, None), p.muls(a[0], 1, a[1], kk, 1, None))
        t0 = a[0] * p.const(k0)
        t1 = a[1] * p.const(k1)
        t2 = p.muls(a[0], 1, a[1], p.const(k0 + k1), 1, None)
        return (t0 - t1, p.lin4(t2, -1, t0, -1, t1))

    def f2_sqr(self, a):
        p = self.p
        return (p.muls(a[0], 1, a[1], a[0], -1, a[1]), p.muls(a[0], 1, a[0], a[1], 1, None))

    def f2_mul_fp(self, a, s):
        return (a[0] * s, a[1] * s)

    def f2_mul_xi(self, a):
        return (a[0] - a[1], a[0] + a[1])

    def f2_small(self, a, k):
        return self.f2_mul_c(a, (k, 0))

    def f2_norm(self, a):
        p = self.p
        return p.lin4(a[0] * a[0], 1, a[1] * a[1], 1, None)

    def f2_inv(self, a):
        ni = self.fp_inv(self.f2_norm(a))
        return (a[0] * ni, -(a[1] * ni))

    def f2_eq(self, a, b):
        p = self.p
        return p.f_and(p.eq(a[0], b[0]), p.eq(a[1], b[1]))

    def f2_is_zero(self, a):
        p = self.p
        return p.f_and(p.is_zero(a[0]), p.is_zero(a[1]))

    def f2_sel(self, f, x, y):
        p = self.p
        return (p.sel(f, x[0], y[0]), p.sel(f, x[1], y[1]))

    def f2_pow(self, a, e: int, w: int = 4):
        if e == 0:
            return (self.p.one, self.p.zero)
        sq = self.f2_sqr(a)
        odd = [a]
        for _ in range((1 << (w - 1)) - 1):
            odd.append(self.f2_mul(odd[-1], sq))
        bits = bin(e)[2:]
        acc = None
        i = 0
        while i < len(bits):
            if bits[i] == "0":
                acc = self.f2_sqr(acc)
                i += 1
                continue
            j = min(i + w, len(bits))
            while bits[j - 1] == "0":
                j -= 1
            val = int(bits[i:j], 2)
            for _ in range(j - i):
                if acc is not None:
                    acc = self.f2_sqr(acc)
            acc = odd[val >> 1] if acc is None else self.f2_mul(acc, odd[val >> 1])
            i = j
        return acc

    def f2_pow_frob(self, a, e: int, w: int = 4):
        """a^e for e < p^2 with half the squarings of f2_pow: e = e1 p + e0 and a^p = conj(a),
        so a^e = conj(a)^e1 * a^e0, one shared square chain over max(|e0|, |e1|) bits with
        sliding windows of width w on both exponents (tables of odd powers of a and conj(a))."""
        e1, e0 = divmod(e, P)
        sq = self.f2_sqr(a)
        odd = [a]
        for _ in range((1 << (w - 1)) - 1):
            odd.append(self.f2_mul(odd[-1], sq))
        pp = self.p

        def mul_conj(x, t):   # x * conj(t) by Karatsuba with the signs folded in (no conj slots)
            t0, t1 = x[0] * t[0], x[1] * t[1]
            t2 = pp.muls(x[0], 1, x[1], t[0], -1, t[1])
            return (pp.lin([(1, t0), (1, t1)]), pp.lin([(1, t2), (-1, t0), (1, t1)]))

        def windows(x):   # {bit position: odd window value}, sum(v << pos) == x
            out, i = {}, x.bit_length() - 1
            while i >= 0:
                if not (x >> i) & 1:
                    i -= 1
                    continue
                j = max(i - w + 1, 0)
                while not (x >> j) & 1:
                    j += 1
                out[j] = (x >> j) & ((1 << (i - j + 1)) - 1)
                i = j - 1
            return out
        w0, w1 = windows(e0), windows(e1)
        acc = None
        for pos in range(max(e0.bit_length(), e1.bit_length()) - 1, -1, -1):
            if acc is not None:
                acc = self.f2_sqr(acc)
            for wins, cj in ((w0, False), (w1, True)):
                if pos in wins:
                    t = odd[wins[pos] >> 1]
                    if acc is None:
                        acc = self.f2_conj(t) if cj else t
                    else:
                        acc = mul_conj(acc, t) if cj else self.f2_mul(acc, t)
        return acc

    def f2_pow_frob_yao(self, a, e: int, w: int = 3, LAG: int = 2):
        """a^e for e < p^2 (e = e1 p + e0, a^p = conj(a)) by Yao's right-to-left k-ary method:
        one chain of squarings B_j = a^(2^(w j)) carries the critical path; each window digit d
        of e0 (of e1) multiplies B_j (conj(B_j)) into an accumulator X_d off that path, and
        prod_d X_d^d closes. Against the left-to-right sliding window (f2_pow_frob) the ~150
        window products leave the square chain: ~280 fewer dependent levels, ~70 more products."""
        pp = self.p

        def mul_conj(x, t):   # x * conj(t), signs folded into Karatsuba
            t0, t1 = x[0] * t[0], x[1] * t[1]
            t2 = pp.muls(x[0], 1, x[1], t[0], -1, t[1])
            return (pp.lin([(1, t0), (1, t1)]), pp.lin([(1, t2), (-1, t0), (1, t1)]))
        def sqr_after(x, deps):   # f2_sqr, not scheduled before `deps`
            ids = tuple(v.id for v in deps)
            return (pp._op("muls", (x[0].id, x[1].id, x[0].id, x[1].id), (1, 1, 1, -1), deps=ids),
                    pp._op("muls", (x[0].id, x[0].id, x[1].id, None), (1, 1, 1, 0), deps=ids))
        e1, e0 = divmod(e, P)
        mask = (1 << w) - 1
        nwin = (max(e0.bit_length(), e1.bit_length()) + w - 1) // w
        X = [None] * (1 << w)
        B = a
        done = []   # per window: the accumulator values it produced
        for j in range(nwin):
            if j:
                # the square chain may run at most LAG windows ahead of the accumulations, so the
                # B_j wait in slots only briefly (free list scheduling let the chain race ahead
                # and held ~130 of them)
                deps = done[j - 1 - LAG] if j - 1 - LAG >= 0 else []
                B = sqr_after(B, deps) if deps else self.f2_sqr(B)
                for _ in range(w - 1):
                    B = self.f2_sqr(B)
            got = []
            for d, cj in (((e0 >> (w * j)) & mask, False), ((e1 >> (w * j)) & mask, True)):
                if not d:
                    continue
                if X[d] is None:
                    X[d] = self.f2_conj(B) if cj else B
                else:
                    X[d] = mul_conj(X[d], B) if cj else self.f2_mul(X[d], B)
                got += [X[d][0], X[d][1]]
            done.append(got)
        # prod_d X_d^d = prod_d Y_d with Y_d = prod_{k >= d} X_k (suffix products)
        ys, y = [], None
        for d in range(mask, 0, -1):
            if X[d] is None:
                if y is not None:
                    ys.append(y)
                continue
            y = X[d] if y is None else self.f2_mul(y, X[d])
            ys.append(y)
        while len(ys) > 1:   # product tree
            ys = [self.f2_mul(ys[k], ys[k + 1]) if k + 1 < len(ys) else ys[k] for k in range(0, len(ys), 2)]
        return ys[0]

    def f2_sgn0(self, a):
        """RFC 9380 sgn0 (m = 2): sgn0(a0) or (a0 == 0 and sgn0(a1))."""
        p = self.p
        return p.f_or(p.sgn0(a[0]), p.f_and(p.is_zero(a[0]), p.sgn0(a[1])))

    def f2_lex(self, a):
        """ZCash sort flag: lex(c1) if c1 != 0 else lex(c0)."""
        p = self.p
        return p.sel(p.is_zero(a[1]), p.lex(a[1]), p.lex(a[0]))

    def f2_sqrt(self, a):
        """Branch-free square root (norm method). Returns (ok, root)."""
        p = self.p
        a0, a1 = a
        inv2 = p.const(INV2)
        n = self.fp_pow(self.f2_norm(a), (P + 1) // 4)
        c = p.muls(a0, 1, n, inv2, 1, None)
        c2 = p.muls(a0, -1, n, inv2, 1, None)
        c = p.sel(p.is_zero(c), c, c2)
        t = self.fp_pow(c, (P - 3) // 4)
        tc = t * c
        qr = p.eq(t * tc, p.one)
        ha1t = p.muls(a1, 1, None, t, 1, None) * inv2
        x0 = p.sel(qr, -ha1t, tc)
        x1 = p.sel(qr, tc, ha1t)
        r = (x0, x1)
        ok = self.f2_eq(self.f2_sqr(r), a)
        return ok, r

    def f2_sqrt9(self, a):
        """RFC 9380 Appendix I.3 (q = p^2 = 9 mod 16): z = a^((q+7)/16) times the 8th root of
        unity that makes z^2 = a when a is a square (f2_pow_frob_yao carries the exponentiation).
        Returns (ok, root); ok iff a is a square."""
        p = self.p
        tv1 = self.f2_pow_frob_yao(a, SQ9_C4)
        tv2 = (-tv1[1], tv1[0])                 # c1 tv1 = u tv1
        tv3 = self.f2_mul(tv1, self.c2(SQ9_C2))
        tv4 = self.f2_mul(tv1, self.c2(SQ9_C3))
        e1 = self.f2_eq(self.f2_sqr(tv2), a)
        e2 = self.f2_eq(self.f2_sqr(tv3), a)
        tv1 = self.f2_sel(e1, tv1, tv2)
        tv2 = self.f2_sel(e2, tv4, tv3)
        e3 = self.f2_eq(self.f2_sqr(tv2), a)
        z = self.f2_sel(e3, tv1, tv2)
        return self.f2_eq(self.f2_sqr(z), a), z

    # ---------------------------------------------------------------- Fp6 / Fp12
    def f6_add(self, a, b):
        return tuple(self.f2_add(x, y) for x, y in zip(a, b))

    def f6_sub(self, a, b):
        return tuple(self.f2_sub(x, y) for x, y in zip(a, b))

    def f6_neg(self, a):
        return tuple(self.f2_neg(x) for x in a)

    def f6_mul(self, a, b):
        a0, a1, a2 = a
        b0, b1, b2 = b
        t0 = self.f2_mul(a0, b0)
        t1 = self.f2_mul(a1, b1)
        t2 = self.f2_mul(a2, b2)
        c0 = self.f2_add(t0, self.f2_mul_xi(self.f2_sub(self.f2_mul(self.f2_add(a1, a2), self.f2_add(b1, b2)),
                                                         self.f2_add(t1, t2))))
        c1 = self.f2_add(self.f2_sub(self.f2_mul(self.f2_add(a0, a1), self.f2_add(b0, b1)), self.f2_add(t0, t1)),
                         self.f2_mul_xi(t2))
        c2 = self.f2_add(self.f2_sub(self.f2_mul(self.f2_add(a0, a2), self.f2_add(b0, b2)), self.f2_add(t0, t2)), t1)
        return (c0, c1, c2)

    def f6_mul_v(self, a):
        return (self.f2_mul_xi(a[2]), a[0], a[1])

    def f6_inv(self, a):
        a0, a1, a2 = a
        c0 = self.f2_sub(self.f2_sqr(a0), self.f2_mul_xi(self.f2_mul(a1, a2)))
        c1 = self.f2_sub(self.f2_mul_xi(self.f2_sqr(a2)), self.f2_mul(a0, a1))
        c2 = self.f2_sub(self.f2_sqr(a1), self.f2_mul(a0, a2))
        t = self.f2_add(self.f2_mul(a0, c0), self.f2_mul_xi(self.f2_add(self.f2_mul(a2, c1), self.f2_mul(a1, c2))))
        ti = self.f2_inv(t)
        return (self.f2_mul(c0, ti), self.f2_mul(c1, ti), self.f2_mul(c2, ti))

    def f12_one(self):
        p = self.p
        z = (p.zero, p.zero)
        return (((p.one, p.zero), z, z), (z, z, z))

    def f12_mul(self, a, b):
        t0 = self.f6_mul(a[0], b[0])
        t1 = self.f6_mul(a[1], b[1])
        c1 = self.f6_sub(self.f6_mul(self.f6_add(a[0], a[1]), self.f6_add(b[0], b[1])), self.f6_add(t0, t1))
        c0 = self.f6_add(t0, self.f6_mul_v(t1))
        return (c0, c1)

    def f12_sqr(self, a):
        """complex squaring: 2 Fp6 products"""
        a0, a1 = a
        t = self.f6_mul(a0, a1)
        s = self.f6_mul(self.f6_add(a0, a1), self.f6_add(a0, self.f6_mul_v(a1)))
        c0 = self.f6_sub(self.f6_sub(s, t), self.f6_mul_v(t))
        return (c0, self.f6_add(t, t))

    def f12_conj(self, a):
        return (a[0], self.f6_neg(a[1]))

    def f12_inv(self, a):
        t = self.f6_sub(self.f6_mul(a[0], a[0]), self.f6_mul_v(self.f6_mul(a[1], a[1])))
        ti = self.f6_inv(t)
        return (self.f6_mul(a[0], ti), self.f6_neg(self.f6_mul(a[1], ti)))

    def f12_frob(self, a):
        (a0, a1, a2), (b0, b1, b2) = a
        coeffs = [a0, b0, a1, b1, a2, b2]
        out = [self.f2_mul_c(self.f2_conj(c), GAMMA[k]) if k else self.f2_conj(c) for k, c in enumerate(coeffs)]
        return ((out[0], out[2], out[4]), (out[1], out[3], out[5]))

    def f12_mul_014(self, f, l0, l1, l4):
        """f * (l0 + l1 v + l4 v w)"""
        t0 = self.f6_mul_01(f[0], l0, l1)
        t1 = self.f6_mul_1(f[1], l4)
        s = self.f6_mul_01(self.f6_add(f[0], f[1]), l0, self.f2_add(l1, l4))
        c1 = self.f6_sub(self.f6_sub(s, t0), t1)
        c0 = self.f6_add(t0, self.f6_mul_v(t1))
        return (c0, c1)

    def f6_mul_01(self, a, b0, b1):
        t0 = self.f2_mul(a[0], b0)
        t1 = self.f2_mul(a[1], b1)
        c0 = self.f2_add(t0, self.f2_mul_xi(self.f2_mul(a[2], b1)))
        c1 = self.f2_sub(self.f2_mul(self.f2_add(a[0], a[1]), self.f2_add(b0, b1)), self.f2_add(t0, t1))
        c2 = self.f2_add(t1, self.f2_mul(a[2], b0))
        return (c0, c1, c2)

    def f6_mul_1(self, a, b1):
        return (self.f2_mul_xi(self.f2_mul(a[2], b1)), self.f2_mul(a[0], b1), self.f2_mul(a[1], b1))

    def f12_cyc_sqr(self, a):
        """Granger-Scott squaring in the cyclotomic subgroup: three Fp4 squarings
        (x + y t)^2 = (x^2 + xi y^2) + 2 x y t, each from 7 Fp products whose operands are 2-term
        sums, and every output coefficient one 4-term linear combination (3 t -/+ 2 z)."""
        p = self.p
        r0, r4, r3 = a[0]
        r2, r1, r5 = a[1]

        def fp4_sqr_terms(x, y):
            X0 = p.muls(x[0], 1, x[1], x[0], -1, x[1])      # (x0 + x1)(x0 - x1)
            X1 = p.muls(x[0], 1, x[0], x[1], 1, None)       # 2 x0 x1
            Y0 = p.muls(y[0], 1, y[1], y[0], -1, y[1])
            Y1 = p.muls(y[0], 1, y[0], y[1], 1, None)
            P0 = x[0] * y[0]
            P1 = x[1] * y[1]
            P2 = p.muls(x[0], 1, x[1], y[0], 1, y[1])
            # t0 = x^2 + xi y^2 = (X0 + Y0 - Y1, X1 + Y0 + Y1); t1 = 2 x y = (2P0 - 2P1, 2P2 - 2P0 - 2P1)
            t0 = ([(1, X0), (1, Y0), (-1, Y1)], [(1, X1), (1, Y0), (1, Y1)])
            t1 = ([(2, P0), (-2, P1)], [(2, P2), (-2, P0), (-2, P1)])
            return t0, t1

        def comb(t, z, sign):  # 3 t + sign 2 z, componentwise
            return tuple(p.lin([(3 * c, v) for c, v in ti] + [(2 * sign, zi)]) for ti, zi in zip(t, z))
        t0, t1 = fp4_sqr_terms(r0, r1)
        t2, t3 = fp4_sqr_terms(r2, r3)
        t4, t5 = fp4_sqr_terms(r4, r5)
        # xi t5 = (t5.c0 - t5.c1, t5.c0 + t5.c1)
        xt5 = ([(c, v) for c, v in t5[0]] + [(-c, v) for c, v in t5[1]],
               [(c, v) for c, v in t5[0]] + [(c, v) for c, v in t5[1]])
        z0 = comb(t0, r0, -1)
        z1 = comb(t1, r1, 1)
        z2 = comb(xt5, r2, 1)
        z3 = comb(t4, r3, -1)
        z4 = comb(t2, r4, -1)
        z5 = comb(t3, r5, 1)
        return ((z0, z4, z3), (z2, z1, z5))

    def f12_eq_one(self, a):
        p = self.p
        flat = [c for f6 in a for f2 in f6 for c in f2]
        acc = p.eq(flat[0], p.one)
        for c in flat[1:]:
            acc = p.f_and(acc, p.is_zero(c))
        return acc

    # ---------------------------------------------------------------- curves (homogeneous projective)
    # A point is (X, Y, Z) with x = X/Z, y = Y/Z; infinity = (0, 1, 0). F = "fp" or "f2".
    def _ops(self, F):
        if F == "fp":
            p = self.p
            return dict(add=lambda a, b: a + b, sub=lambda a, b: a - b, mul=lambda a, b: a * b,
                        b3=lambda a: a * p.const(12), neg=lambda a: -a, zero=p.zero, one=p.one)
        return dict(add=self.f2_add, sub=self.f2_sub, mul=self.f2_mul,
                    b3=lambda a: self.f2_mul_c(a, (12, 12)), neg=self.f2_neg,
                    zero=(self.p.zero, self.p.zero), one=(self.p.one, self.p.zero))

    def pt_add(self, F, A, B):
        """RCB 2016 Algorithm 7 (complete addition, a = 0)."""
        o = self._ops(F)
        add, sub, mul, b3 = o["add"], o["sub"], o["mul"], o["b3"]
        X1, Y1, Z1 = A
        X2, Y2, Z2 = B
        t0 = mul(X1, X2)
        t1 = mul(Y1, Y2)
        t2 = mul(Z1, Z2)
        t3 = mul(add(X1, Y1), add(X2, Y2))
        t4 = add(t0, t1)
        t3 = sub(t3, t4)
        t4 = mul(add(Y1, Z1), add(Y2, Z2))
        X3 = add(t1, t2)
        t4 = sub(t4, X3)
        X3 = mul(add(X1, Z1), add(X2, Z2))
        Y3 = add(t0, t2)
        Y3 = sub(X3, Y3)
        X3 = add(t0, t0)
        t0 = add(X3, t0)
        t2 = b3(t2)
        Z3 = add(t1, t2)
        t1 = sub(t1, t2)
        Y3 = b3(Y3)
        X3 = mul(t4, Y3)
        t2 = mul(t3, t1)
        X3 = sub(t2, X3)
        Y3 = mul(Y3, t0)
        t1 = mul(t1, Z3)
        Y3 = add(t1, Y3)
        t0 = mul(t0, t3)
        Z3 = mul(Z3, t4)
        Z3 = add(Z3, t0)
        return (X3, Y3, Z3)

    def pt_dbl(self, F, A):
        """RCB 2016 Algorithm 9 (complete doubling, a = 0)."""
        o = self._ops(F)
        add, sub, mul, b3 = o["add"], o["sub"], o["mul"], o["b3"]
        X, Y, Z = A
        t0 = mul(Y, Y)
        Z3 = add(t0, t0)
        Z3 = add(Z3, Z3)
        Z3 = add(Z3, Z3)
        t1 = mul(Y, Z)
        t2 = mul(Z, Z)
        t2 = b3(t2)
        X3 = mul(t2, Z3)
        Y3 = add(t0, t2)
        Z3 = mul(t1, Z3)
        t1 = add(t2, t2)
        t2 = add(t1, t2)
        t0 = sub(t0, t2)
        Y3 = mul(t0, Y3)
        Y3 = add(X3, Y3)
        t1 = mul(X, Y)
        X3 = mul(t0, t1)
        X3 = add(X3, X3)
        return (X3, Y3, Z3)

    def pt_neg(self, F, A):
        return (A[0], self._ops(F)["neg"](A[1]), A[2])

    def pt_inf(self, F):
        o = self._ops(F)
        return (o["zero"], o["one"], o["zero"])

    def pt_mul_fixed(self, F, A, k: int):
        """[k] A, k > 0 fixed (public), double-and-add on complete formulas."""
        bits = bin(k)[2:]
        acc = A
        for b in bits[1:]:
            acc = self.pt_dbl(F, acc)
            if b == "1":
                acc = self.pt_add(F, acc, A)
        return acc

    def pt_mul_rbits(self, F, A, nbits: int = 64):
        """[r] A for the vote's secret-free RLC scalar r (bits via rbit), double-and-add-always."""
        p = self.p
        acc = self.pt_inf(F)
        for k in range(nbits - 1, -1, -1):
            if k != nbits - 1:
                acc = self.pt_dbl(F, acc)
            t = self.pt_add(F, acc, A)
            if F == "fp":
                acc = tuple(p.selb(k, a_, t_) for a_, t_ in zip(acc, t))
            else:
                acc = tuple((p.selb(k, a_[0], t_[0]), p.selb(k, a_[1], t_[1])) for a_, t_ in zip(acc, t))
        return acc

    def pt_selb(self, F, k, A, B, after=None):
        """bit k of the vote's 64-bit RLC value ? B : A (not scheduled before `after`)"""
        p = self.p
        if F == "fp":
            return tuple(p.selb(k, a, b, after) for a, b in zip(A, B))
        return tuple((p.selb(k, a[0], b[0], after), p.selb(k, a[1], b[1], after)) for a, b in zip(A, B))

    def pt_mul_glv(self, F, A, B, nbits: int = 32):
        """[a] A + [b] B for the vote's RLC value (a = bits 0..31, b = bits 32..63), B = [LAMBDA] A
        by an endomorphism (see LAMBDA): one double-and-add-always chain over 32 bits whose
        addend (O, A, B or A + B) is picked by two selb levels; complete formulas."""
        AB = self.pt_add(F, A, B)
        O = self.pt_inf(F)
        acc = None
        for k in range(nbits - 1, -1, -1):
            # the step's addend is selected once the previous step's sum exists
            dep = None if acc is None else (acc[2] if F == "fp" else acc[2][0])
            lo = self.pt_selb(F, k, O, A, dep)
            hi = self.pt_selb(F, k, B, AB, dep)
            ad = self.pt_selb(F, k + nbits, lo, hi, dep)
            acc = ad if acc is None else self.pt_add(F, self.pt_dbl(F, acc), ad)
        return acc

    def g1_phi(self, A):
        """phi(P) = (beta X : Y : Z) = [-x^2] P on G1."""
        return (A[0] * self.p.const(BETA), A[1], A[2])

    def g2_neg_psi2(self, A):
        """-psi^2(Q) = [-x^2] Q on G2."""
        return self.pt_neg("f2", self.g2_psi(self.g2_psi(A)))

    def pt_sel(self, F, f, A, B):
        p = self.p
        if F == "fp":
            return tuple(p.sel(f, a, b) for a, b in zip(A, B))
        return tuple(self.f2_sel(f, a, b) for a, b in zip(A, B))

    def pt_eq(self, F, A, B):
        """projective equality (both non-infinity or both infinity handled by the callers)."""
        o = self._ops(F)
        mul = o["mul"]
        p = self.p
        if F == "fp":
            e1 = p.eq(mul(A[0], B[2]), mul(B[0], A[2]))
            e2 = p.eq(mul(A[1], B[2]), mul(B[1], A[2]))
        else:
            e1 = self.f2_eq(mul(A[0], B[2]), mul(B[0], A[2]))
            e2 = self.f2_eq(mul(A[1], B[2]), mul(B[1], A[2]))
        return p.f_and(e1, e2)

    def g2_psi(self, A):
        X, Y, Z = A
        return (self.f2_mul_c(self.f2_conj(X), PSI_CX), self.f2_mul_c(self.f2_conj(Y), PSI_CY), self.f2_conj(Z))

    def g1_in_group(self, A):
        """phi(P) == [-x^2] P  (P not infinity)."""
        t1 = self.pt_mul_fixed("fp", A, X_ABS)
        t2 = self.pt_mul_fixed("fp", t1, X_ABS)
        return self.pt_eq("fp", self.g1_phi(A), self.pt_neg("fp", t2)), t1

    def g2_in_group(self, A):
        """psi(Q) == [x] Q = -[|x|] Q  (Q not infinity)."""
        t = self.pt_mul_fixed("f2", A, X_ABS)
        return self.pt_eq("f2", self.g2_psi(A), self.pt_neg("f2", t))

    def to_affine(self, F, A):
        if F == "fp":
            zi = self.fp_inv(A[2])
            return (A[0] * zi, A[1] * zi)
        zi = self.f2_inv(A[2])
        return (self.f2_mul(A[0], zi), self.f2_mul(A[1], zi))

    # ---------------------------------------------------------------- decompression
    def g1_decompress(self, x_plain, sort_flag):
        """x from plain limbs (-> Montgomery via the product with R^2 done by the prologue op
        `tomont`), y = sqrt(x^3 + 4) with the ZCash sign. Returns (on_curve, (x, y))."""
        p = self.p
        x = x_plain
        rhs = p.lin4(x * (x * x), 1, p.const(4), 1, None)
        y = self.fp_pow_yao(rhs, (P + 1) // 4) if self.fast_sqrt else self.fp_pow(rhs, (P + 1) // 4)
        ok = p.eq(y * y, rhs)
        flip = p.f_xor(p.lex(y), sort_flag)
        y = p.sel(flip, y, -y)
        return ok, (x, y)

    def g2_decompress(self, x, sort_flag):
        p = self.p
        rhs = self.f2_add(self.f2_mul(x, self.f2_sqr(x)), self.c2((4, 4)))
        ok, y = self.f2_sqrt9(rhs) if self.fast_sqrt else self.f2_sqrt(rhs)
        flip = p.f_xor(self.f2_lex(y), sort_flag)
        y = self.f2_sel(flip, y, self.f2_neg(y))
        return ok, (x, y)

    # ---------------------------------------------------------------- hash to G2
    def sqrt_ratio(self, u, v):
        """RFC 9380 F.2.1.1 over Fp2 (q = p^2, c1 = 3). Returns (isQR, y)."""
        p = self.p
        tv1 = self.c2(SR_C6)
        tv2 = self.f2_pow(v, SR_C4)
        tv3 = self.f2_sqr(tv2)
        tv3 = self.f2_mul(tv3, v)
        tv5 = self.f2_mul(u, tv3)
        tv5 = self.f2_pow_frob_yao(tv5, SR_C3) if YAO_POW else self.f2_pow_frob(tv5, SR_C3)
        tv5 = self.f2_mul(tv5, tv2)
        tv2 = self.f2_mul(tv5, v)
        tv3 = self.f2_mul(tv5, u)
        tv4 = self.f2_mul(tv3, tv2)
        tv5 = self.f2_pow(tv4, SR_C5)
        is_qr = self.f2_eq(tv5, (p.one, p.zero))
        tv2 = self.f2_mul_c(tv3, SR_C7)
        tv5 = self.f2_mul(tv4, tv1)
        tv3 = self.f2_sel(is_qr, tv2, tv3)
        tv4 = self.f2_sel(is_qr, tv5, tv4)
        for k in range(SR_C1, 1, -1):
            tv5 = self.f2_pow(tv4, 1 << (k - 2)) if k > 2 else tv4
            e1 = self.f2_eq(tv5, (p.one, p.zero))
            tv2 = self.f2_mul(tv3, tv1)
            tv1 = self.f2_sqr(tv1)
            tv5 = self.f2_mul(tv4, tv1)
            tv3 = self.f2_sel(e1, tv2, tv3)
            tv4 = self.f2_sel(e1, tv5, tv4)
        return is_qr, tv3

    def map_to_curve_sswu(self, u):
        """RFC 9380 6.6.2 (optimized, F.2). Returns (xn, xd, y) with x = xn / xd on E2'."""
        p = self.p
        A, B, Z = SSWU_A, SSWU_B, SSWU_Z
        tv1 = self.f2_mul_c(self.f2_sqr(u), Z)
        tv2 = self.f2_add(self.f2_sqr(tv1), tv1)
        tv3 = self.f2_mul_c(self.f2_add(tv2, (p.one, p.zero)), B)
        tv4 = self.f2_sel(self.f2_is_zero(tv2), self.f2_neg(tv2), self.c2(Z))
        tv4 = self.f2_mul_c(tv4, A)
        tv2 = self.f2_sqr(tv3)
        tv6 = self.f2_sqr(tv4)
        tv5 = self.f2_mul_c(tv6, A)
        tv2 = self.f2_add(tv2, tv5)
        tv2 = self.f2_mul(tv2, tv3)
        tv6 = self.f2_mul(tv6, tv4)
        tv5 = self.f2_mul_c(tv6, B)
        tv2 = self.f2_add(tv2, tv5)
        x = self.f2_mul(tv1, tv3)
        is_gx1_sq, y1 = self.sqrt_ratio(tv2, tv6)
        y = self.f2_mul(self.f2_mul(tv1, u), y1)
        x = self.f2_sel(is_gx1_sq, x, tv3)
        y = self.f2_sel(is_gx1_sq, y, y1)
        e1 = p.f_xor(self.f2_sgn0(u), self.f2_sgn0(y))  # 1 when signs differ
        y = self.f2_sel(e1, y, self.f2_neg(y))
        return x, tv4, y

    def _poly_h(self, coeffs, xn, xd, deg):
        """xd^deg * poly(xn/xd) = sum k_i xn^i xd^(deg-i)"""
        xn_p = [None, xn]
        xd_p = [None, xd]
        for i in range(2, deg + 1):
            xn_p.append(self.f2_mul(xn_p[-1], xn))
            xd_p.append(self.f2_mul(xd_p[-1], xd))
        acc = None
        for i, k in enumerate(coeffs):
            if i == 0:
                term = self.f2_mul_c(xd_p[deg], k)
            elif i == deg:
                term = xn_p[deg] if k == (1, 0) else self.f2_mul_c(xn_p[deg], k)
            else:
                term = self.f2_mul_c(self.f2_mul(xn_p[i], xd_p[deg - i]), k)
            acc = term if acc is None else self.f2_add(acc, term)
        return acc

    def iso_map(self, xn, xd, y):
        """3-isogeny to E2, homogenised: returns a projective point (X, Y, Z)."""
        XN = self._poly_h(ISO_XNUM, xn, xd, 3)          # xd^3 xnum(x)
        XD2 = self._poly_h(ISO_XDEN, xn, xd, 2)         # xd^2 xden(x)
        YN = self._poly_h(ISO_YNUM, xn, xd, 3)          # xd^3 ynum(x)
        YD = self._poly_h(ISO_YDEN, xn, xd, 3)          # xd^3 yden(x)
        # x' = XN / (xd XD2), y' = y YN / YD
        xdXD2 = self.f2_mul(xd, XD2)
        Z = self.f2_mul(xdXD2, YD)
        X = self.f2_mul(XN, YD)
        Y = self.f2_mul(self.f2_mul(y, YN), xdXD2)
        return (X, Y, Z)

    # Jacobian (x = X/Z^2, y = Y/Z^3) chains for cofactor clearing only: dbl-2009-l doubling
    # (a = 0) is 3 product levels deep against ~5 for the complete homogeneous formula, so the
    # two 63-doubling chains of h_eff, which sit on the vote program's critical path, shorten.
    # The additions (add-2007-bl) are not complete: they fail only when an intermediate [k]A
    # equals +-A, i.e. when the hash point's order is below 2^64 -- never, for a point derived
    # from a hash. Subgroup checks keep the complete formulas (their inputs are adversarial).
    def _f2_lin(self, terms):
        p = self.p
        return (p.lin([(c, v[0]) for c, v in terms]), p.lin([(c, v[1]) for c, v in terms]))

    def g2_hom_to_jac(self, A):
        X, Y, Z = A
        return (self.f2_mul(X, Z), self.f2_mul(Y, self.f2_sqr(Z)), Z)

    def g2_jac_to_hom(self, A):
        X, Y, Z = A
        return (self.f2_mul(X, Z), Y, self.f2_mul(Z, self.f2_sqr(Z)))

    def g2_jac_dbl(self, A):
        """S = 4 X Y^2 as the product X (Y^2) rather than (X + Y^2)^2 - X^2 - Y^4 (dbl-2009-l):
        one product more, but no sum ahead of a square, so the chain through Y is two products,
        a linear combination, a product and a linear combination deep."""
        X, Y, Z = A
        a = self.f2_sqr(X)
        b = self.f2_sqr(Y)
        yz = self.f2_mul(Y, Z)
        c = self.f2_sqr(b)
        # X b by Karatsuba, its three Fp products combined straight into X3 and u (xb is used
        # twice, so a shared post-addition would add a level)
        p = self.p
        t0, t1 = X[0] * b[0], X[1] * b[1]
        t2 = p.muls(X[0], 1, X[1], b[0], 1, b[1])
        f = self.f2_sqr(a)
        # X3 = M^2 - 2S = 9 f - 8 xb (M = 3 X^2), u = S - X3 = 12 xb - 9 f; xb = (t0 - t1, t2 - t0 - t1)
        X3 = (p.lin([(9, f[0]), (-8, t0), (8, t1)]), p.lin([(9, f[1]), (-8, t2), (8, t0), (8, t1)]))
        u = (p.lin([(-9, f[0]), (12, t0), (-12, t1)]), p.lin([(-9, f[1]), (12, t2), (-12, t0), (-12, t1)]))
        Y3 = self._f2_lin([(3, self.f2_mul(a, u)), (-8, c)])
        Z3 = self._f2_lin([(2, yz)])
        return (X3, Y3, Z3)

    def g2_jac_add(self, A, B):
        X1, Y1, Z1 = A
        X2, Y2, Z2 = B
        z1z1 = self.f2_sqr(Z1)
        z2z2 = self.f2_sqr(Z2)
        u1 = self.f2_mul(X1, z2z2)
        u2 = self.f2_mul(X2, z1z1)
        s1 = self.f2_mul(Y1, self.f2_mul(Z2, z2z2))
        s2 = self.f2_mul(Y2, self.f2_mul(Z1, z1z1))
        h = self.f2_sub(u2, u1)
        i = self.f2_sqr(self.f2_dbl(h))
        j = self.f2_mul(h, i)
        r = self._f2_lin([(2, s2), (-2, s1)])
        v = self.f2_mul(u1, i)
        X3 = self._f2_lin([(1, self.f2_sqr(r)), (-1, j), (-2, v)])
        Y3 = self._f2_lin([(1, self.f2_mul(r, self.f2_sub(v, X3))), (-2, self.f2_mul(s1, j))])
        Z3 = self.f2_mul(self._f2_lin([(1, self.f2_sqr(self.f2_add(Z1, Z2))), (-1, z1z1), (-1, z2z2)]), h)
        return (X3, Y3, Z3)

    def g2_mul_fixed_jac(self, A, k: int):
        """[k] A (homogeneous in and out) by a Jacobian double-and-add chain."""
        J = self.g2_hom_to_jac(A)
        acc = J
        for b in bin(k)[3:]:
            acc = self.g2_jac_dbl(acc)
            if b == "1":
                acc = self.g2_jac_add(acc, J)
        return self.g2_jac_to_hom(acc)

    def clear_cofactor(self, A):
        """h_eff A = [x^2 - x - 1] A + [x - 1] psi(A) + psi^2(2A), x = -X_ABS (RFC 9380 G.3).
        With t1 = [X_ABS] A and psi commuting with scalars:
          h_eff A = [X_ABS] B + K,  B = t1 - psi(A),  K = B - A + psi^2(2A),
        so only K (one point) is held across the second scalar chain."""
        mul = self.g2_mul_fixed_jac if JAC_COFACTOR else (lambda P_, k: self.pt_mul_fixed("f2", P_, k))
        t1 = mul(A, X_ABS)
        B = self.pt_add("f2", t1, self.pt_neg("f2", self.g2_psi(A)))
        K = self.pt_add("f2", self.pt_add("f2", B, self.pt_neg("f2", A)),
                        self.g2_psi(self.g2_psi(self.pt_dbl("f2", A))))
        return self.pt_add("f2", mul(B, X_ABS), K)

    def hash_to_g2(self, u0, u1):
        q0 = self.iso_map(*self.map_to_curve_sswu(u0))
        q1 = self.iso_map(*self.map_to_curve_sswu(u1))
        return self.clear_cofactor(self.pt_add("f2", q0, q1))

    # ---------------------------------------------------------------- pairing
    def miller_loop(self, Pa, Q):
        """f_{|x|,Q}(P) conjugated. Pa = (xP, yP) affine or (XP, YP, ZP) homogeneous projective
        in Fp (every line then carries the factor ZP in Fp, which the final exponentiation
        removes: no inversion); Q = (X, Y, Z) projective in E2."""
        return self.miller_loop_multi([(Pa, Q)])

    def miller_loop_multi(self, pairs):
        """prod_j f_{|x|,Q_j}(P_j) conjugated, one shared f: every iteration squares f once and
        multiplies in each pair's line (the n = 1 vote program's two pairs)."""
        st = []
        for Pa, Q in pairs:
            xP, yP = Pa[0], Pa[1]
            ZP = Pa[2] if len(Pa) == 3 else None
            st.append({"ZP": ZP, "Q": Q, "T": Q, "m3x": -(xP + xP + xP), "y2": yP + yP,
                       "xPZ": self.f2_mul_fp(Q[2], xP), "yPZ": self.f2_mul_fp(Q[2], yP)})
        f = None
        for b in range(62, -1, -1):
            lines = []
            for d in st:
                X, Y, Z = d["T"]
                XX = self.f2_sqr(X)
                YY = self.f2_sqr(Y)
                ZZ = self.f2_sqr(Z)
                E = self.f2_mul_c(ZZ, (12, 12))          # 3 b' Z^2
                l0 = self.f2_sub(YY, E)
                if d["ZP"] is not None:
                    l0 = self.f2_mul_fp(l0, d["ZP"])
                l1 = self.f2_mul_fp(XX, d["m3x"])
                YZ = self.f2_mul(Y, Z)
                l4 = self.f2_mul_fp(YZ, d["y2"])
                A = self.f2_mul(X, Y)
                Fv = self.f2_add(self.f2_dbl(E), E)
                X3 = self.f2_dbl(self.f2_mul(A, self.f2_sub(YY, Fv)))
                G = self.f2_add(YY, Fv)
                Y3 = self.f2_sub(self.f2_sqr(G), self.f2_small(self.f2_sqr(E), 12))
                Z3 = self.f2_mul_c(self.f2_mul(YY, YZ), (8, 0))
                d["T"] = (X3, Y3, Z3)
                lines.append((l0, l1, l4))
            for k, (l0, l1, l4) in enumerate(lines):
                if f is None:
                    f = self.f12_mul_014(self.f12_one(), l0, l1, l4)
                elif k == 0:
                    f = self.f12_mul_014(self.f12_sqr(f), l0, l1, l4)
                else:
                    f = self.f12_mul_014(f, l0, l1, l4)
            if (X_ABS >> b) & 1:
                for d in st:
                    X, Y, Z = d["T"]
                    XQ, YQ, ZQ = d["Q"]
                    th = self.f2_sub(self.f2_mul(Y, ZQ), self.f2_mul(YQ, Z))
                    lm = self.f2_sub(self.f2_mul(X, ZQ), self.f2_mul(XQ, Z))
                    l0 = self.f2_sub(self.f2_mul(th, XQ), self.f2_mul(lm, YQ))
                    if d["ZP"] is not None:
                        l0 = self.f2_mul_fp(l0, d["ZP"])
                    l1 = self.f2_neg(self.f2_mul(th, d["xPZ"]))
                    l4 = self.f2_mul(lm, d["yPZ"])
                    d["T"] = self.pt_add("f2", d["T"], d["Q"])
                    f = self.f12_mul_014(f, l0, l1, l4)
        return self.f12_conj(f)

    def f12_exp_x(self, f):
        acc = f
        for b in range(62, -1, -1):
            acc = self.f12_cyc_sqr(acc)
            if (X_ABS >> b) & 1:
                acc = self.f12_mul(acc, f)
        return self.f12_conj(acc)

    def final_exp(self, fin):
        """f^(3 (p^12 - 1)/r) (x-chain)."""
        f = self.f12_mul(self.f12_conj(fin), self.f12_inv(fin))
        f = self.f12_mul(self.f12_frob(self.f12_frob(f)), f)
        t = self.f12_mul(self.f12_exp_x(f), self.f12_conj(f))
        t = self.f12_mul(self.f12_exp_x(t), self.f12_conj(t))
        t = self.f12_mul(self.f12_exp_x(t), self.f12_frob(t))
        t = self.f12_mul(self.f12_mul(self.f12_exp_x(self.f12_exp_x(t)), self.f12_frob(self.f12_frob(t))),
                         self.f12_conj(t))
        return self.f12_mul(t, self.f12_mul(self.f12_cyc_sqr(f), f))
