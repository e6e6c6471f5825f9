// Extension tower: Fp2 = Fp[u]/(u^2+1), Fp6 = Fp2[v]/(v^3 - xi) with xi = 1+u,
// Fp12 = Fp6[w]/(w^2 - v). Same tower as the oracle (oracle/py/bls12_381.py).
#pragma once
#include "fp.hpp"

namespace ovh {

struct Fp2 {
  Fp c0, c1;
};
struct Fp6 {
  Fp2 c0, c1, c2;
};
struct Fp12 {
  Fp6 c0, c1;
};

// ------------------------------------------------------------------------------ Fp2
OVH_HD Fp2 fp2_const(const uint32_t* a0, const uint32_t* a1) {
  Fp2 r;
  fp_load(r.c0, a0);
  fp_load(r.c1, a1);
  return r;
}
OVH_HD void fp2_zero(Fp2& r) {
  fp_zero(r.c0);
  fp_zero(r.c1);
}
OVH_HD void fp2_one(Fp2& r) {
  fp_one(r.c0);
  fp_zero(r.c1);
}
OVH_HD bool fp2_is_zero(const Fp2& a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
OVH_HD bool fp2_eq(const Fp2& a, const Fp2& b) { return fp_eq(a.c0, b.c0) && fp_eq(a.c1, b.c1); }
OVH_HD void fp2_select(Fp2& r, bool cond, const Fp2& a, const Fp2& b) {
  fp_select(r.c0, cond, a.c0, b.c0);
  fp_select(r.c1, cond, a.c1, b.c1);
}
OVH_HD void fp2_add(Fp2& r, const Fp2& a, const Fp2& b) {
  fp_add(r.c0, a.c0, b.c0);
  fp_add(r.c1, a.c1, b.c1);
}
OVH_HD void fp2_sub(Fp2& r, const Fp2& a, const Fp2& b) {
  fp_sub(r.c0, a.c0, b.c0);
  fp_sub(r.c1, a.c1, b.c1);
}
OVH_HD void fp2_dbl(Fp2& r, const Fp2& a) {
  fp_add(r.c0, a.c0, a.c0);
  fp_add(r.c1, a.c1, a.c1);
}
OVH_HD void fp2_neg(Fp2& r, const Fp2& a) {
  fp_neg(r.c0, a.c0);
  fp_neg(r.c1, a.c1);
}
OVH_HD void fp2_conj(Fp2& r, const Fp2& a) {
  r.c0 = a.c0;
  fp_neg(r.c1, a.c1);
}
// Karatsuba: 3 Fp products
OVH_HD void fp2_mul(Fp2& r, const Fp2& a, const Fp2& b) {
  Fp t0, t1, s0, s1;
  fp_mul(t0, a.c0, b.c0);
  fp_mul(t1, a.c1, b.c1);
  fp_add(s0, a.c0, a.c1);
  fp_add(s1, b.c0, b.c1);
  fp_mul(s0, s0, s1);
  fp_sub(r.c0, t0, t1);
  fp_sub(s0, s0, t0);
  fp_sub(r.c1, s0, t1);
}
// (a0 + a1 u)^2 = (a0+a1)(a0-a1) + 2 a0 a1 u : 2 Fp products
OVH_HD void fp2_sqr(Fp2& r, const Fp2& a) {
  Fp s, d, m;
  fp_add(s, a.c0, a.c1);
  fp_sub(d, a.c0, a.c1);
  fp_mul(m, a.c0, a.c1);
  fp_mul(r.c0, s, d);
  fp_add(r.c1, m, m);
}
OVH_HD void fp2_mul_fp(Fp2& r, const Fp2& a, const Fp& b) {
  fp_mul(r.c0, a.c0, b);
  fp_mul(r.c1, a.c1, b);
}
// a * (1 + u) = (a0 - a1) + (a0 + a1) u
OVH_HD void fp2_mul_xi(Fp2& r, const Fp2& a) {
  Fp t0, t1;
  fp_sub(t0, a.c0, a.c1);
  fp_add(t1, a.c0, a.c1);
  r.c0 = t0;
  r.c1 = t1;
}
OVH_HD void fp2_mul_small(Fp2& r, const Fp2& a, uint32_t k) {
  fp_mul_small(r.c0, a.c0, k);
  fp_mul_small(r.c1, a.c1, k);
}
OVH_HD void fp2_norm(Fp& r, const Fp2& a) {
  Fp t0, t1;
  fp_sqr(t0, a.c0);
  fp_sqr(t1, a.c1);
  fp_add(r, t0, t1);
}
OVH_HD void fp2_inv(Fp2& r, const Fp2& a) {
  Fp n, ni;
  fp2_norm(n, a);
  fp_inv(ni, n);
  fp_mul(r.c0, a.c0, ni);
  fp_mul(ni, a.c1, ni);
  fp_neg(r.c1, ni);
}
// ZCash sort flag: compare c1 first, c0 only when c1 == 0.
OVH_HD bool fp2_lex_largest(const Fp2& a) {
  if (!fp_is_zero(a.c1)) return fp_lex_largest(a.c1);
  return fp_lex_largest(a.c0);
}
// RFC 9380 sgn0 for m = 2.
OVH_HD uint32_t fp2_sgn0(const Fp2& a) {
  uint32_t s0 = fp_sgn0(a.c0);
  uint32_t z0 = fp_is_zero(a.c0) ? 1u : 0u;
  uint32_t s1 = fp_sgn0(a.c1);
  return s0 | (z0 & s1);
}

// Square root in Fp2 (p = 3 mod 4) through the norm:
//   n = sqrt(a0^2 + a1^2) in Fp (fails <=> a is a non-square),
//   c = (a0 + n)/2; s = c^((p+1)/4). If s^2 == c: x0 = s, else s = sqrt(-c) and
//   x0 = (a1/2)/s (then c' = (a0 - n)/2 = -(a1/2)^2/c is the square);  x1 = a1 / (2 x0).
// Returns true and some root on success (callers fix the sign).
OVH_HDNI bool fp2_sqrt(Fp2& r, const Fp2& a) {
  if (fp_is_zero(a.c1)) {
    Fp s;
    if (fp_sqrt(s, a.c0)) {
      r.c0 = s;
      fp_zero(r.c1);
      return true;
    }
    Fp na;
    fp_neg(na, a.c0);
    if (fp_sqrt(s, na)) {
      fp_zero(r.c0);
      r.c1 = s;
      return true;
    }
    return false;
  }
  Fp nrm, n;
  fp2_norm(nrm, a);
  if (!fp_sqrt(n, nrm)) return false;
  const Fp inv2 = fp_const(INV2_M);
  Fp c, s, s2, x0, x1, t;
  fp_add(c, a.c0, n);
  fp_mul(c, c, inv2);
  fp_pow(s, c, EXP_SQRT);
  fp_sqr(s2, s);
  Fp half_a1;
  fp_mul(half_a1, a.c1, inv2);
  if (fp_eq(s2, c)) {
    x0 = s;
  } else {
    // s = sqrt(-c): x0 = (a1/2) / s
    fp_inv(t, s);
    fp_mul(x0, half_a1, t);
  }
  // x1 = (a1/2) / x0
  fp_inv(t, x0);
  fp_mul(x1, half_a1, t);
  r.c0 = x0;
  r.c1 = x1;
  Fp2 chk;
  fp2_sqr(chk, r);
  return fp2_eq(chk, a);
}

// ------------------------------------------------------------------------------ Fp6
OVH_HD void fp6_zero(Fp6& r) {
  fp2_zero(r.c0);
  fp2_zero(r.c1);
  fp2_zero(r.c2);
}
OVH_HD void fp6_one(Fp6& r) {
  fp2_one(r.c0);
  fp2_zero(r.c1);
  fp2_zero(r.c2);
}
OVH_HD void fp6_add(Fp6& r, const Fp6& a, const Fp6& b) {
  fp2_add(r.c0, a.c0, b.c0);
  fp2_add(r.c1, a.c1, b.c1);
  fp2_add(r.c2, a.c2, b.c2);
}
OVH_HD void fp6_sub(Fp6& r, const Fp6& a, const Fp6& b) {
  fp2_sub(r.c0, a.c0, b.c0);
  fp2_sub(r.c1, a.c1, b.c1);
  fp2_sub(r.c2, a.c2, b.c2);
}
OVH_HD void fp6_neg(Fp6& r, const Fp6& a) {
  fp2_neg(r.c0, a.c0);
  fp2_neg(r.c1, a.c1);
  fp2_neg(r.c2, a.c2);
}
OVH_HD bool fp6_eq(const Fp6& a, const Fp6& b) { return fp2_eq(a.c0, b.c0) && fp2_eq(a.c1, b.c1) && fp2_eq(a.c2, b.c2); }
// Karatsuba-style, 6 Fp2 products
OVH_HDNI void fp6_mul(Fp6& r, const Fp6& a, const Fp6& b) {
  Fp2 t0, t1, t2, s0, s1, c0, c1, c2;
  fp2_mul(t0, a.c0, b.c0);
  fp2_mul(t1, a.c1, b.c1);
  fp2_mul(t2, a.c2, b.c2);
  // c0 = t0 + xi((a1+a2)(b1+b2) - t1 - t2)
  fp2_add(s0, a.c1, a.c2);
  fp2_add(s1, b.c1, b.c2);
  fp2_mul(c0, s0, s1);
  fp2_sub(c0, c0, t1);
  fp2_sub(c0, c0, t2);
  fp2_mul_xi(c0, c0);
  fp2_add(c0, c0, t0);
  // c1 = (a0+a1)(b0+b1) - t0 - t1 + xi t2
  fp2_add(s0, a.c0, a.c1);
  fp2_add(s1, b.c0, b.c1);
  fp2_mul(c1, s0, s1);
  fp2_sub(c1, c1, t0);
  fp2_sub(c1, c1, t1);
  fp2_mul_xi(s0, t2);
  fp2_add(c1, c1, s0);
  // c2 = (a0+a2)(b0+b2) - t0 - t2 + t1
  fp2_add(s0, a.c0, a.c2);
  fp2_add(s1, b.c0, b.c2);
  fp2_mul(c2, s0, s1);
  fp2_sub(c2, c2, t0);
  fp2_sub(c2, c2, t2);
  fp2_add(c2, c2, t1);
  r.c0 = c0;
  r.c1 = c1;
  r.c2 = c2;
}
// a * v = xi a2 + a0 v + a1 v^2
OVH_HD void fp6_mul_v(Fp6& r, const Fp6& a) {
  Fp2 t;
  fp2_mul_xi(t, a.c2);
  r.c2 = a.c1;
  r.c1 = a.c0;
  r.c0 = t;
}
// a * (b0 + b1 v): 5 Fp2 products
OVH_HD void fp6_mul_01(Fp6& r, const Fp6& a, const Fp2& b0, const Fp2& b1) {
  Fp2 t0, t1, c0, c1, c2, s;
  fp2_mul(t0, a.c0, b0);
  fp2_mul(t1, a.c1, b1);
  // c0 = a0 b0 + xi a2 b1
  fp2_mul(s, a.c2, b1);
  fp2_mul_xi(s, s);
  fp2_add(c0, t0, s);
  // c1 = a0 b1 + a1 b0
  fp2_mul(c1, a.c0, b1);
  fp2_mul(s, a.c1, b0);
  fp2_add(c1, c1, s);
  // c2 = a1 b1 + a2 b0
  fp2_mul(s, a.c2, b0);
  fp2_add(c2, t1, s);
  r.c0 = c0;
  r.c1 = c1;
  r.c2 = c2;
}
// a * (b1 v): xi a2 b1 + a0 b1 v + a1 b1 v^2
OVH_HD void fp6_mul_1(Fp6& r, const Fp6& a, const Fp2& b1) {
  Fp2 c0, c1, c2;
  fp2_mul(c0, a.c2, b1);
  fp2_mul_xi(c0, c0);
  fp2_mul(c1, a.c0, b1);
  fp2_mul(c2, a.c1, b1);
  r.c0 = c0;
  r.c1 = c1;
  r.c2 = c2;
}
OVH_HDNI void fp6_inv(Fp6& r, const Fp6& a) {
  Fp2 c0, c1, c2, t, s;
  fp2_sqr(c0, a.c0);
  fp2_mul(t, a.c1, a.c2);
  fp2_mul_xi(t, t);
  fp2_sub(c0, c0, t);
  fp2_sqr(c1, a.c2);
  fp2_mul_xi(c1, c1);
  fp2_mul(t, a.c0, a.c1);
  fp2_sub(c1, c1, t);
  fp2_sqr(c2, a.c1);
  fp2_mul(t, a.c0, a.c2);
  fp2_sub(c2, c2, t);
  fp2_mul(t, a.c2, c1);
  fp2_mul(s, a.c1, c2);
  fp2_add(t, t, s);
  fp2_mul_xi(t, t);
  fp2_mul(s, a.c0, c0);
  fp2_add(t, t, s);
  fp2_inv(t, t);
  fp2_mul(r.c0, c0, t);
  fp2_mul(r.c1, c1, t);
  fp2_mul(r.c2, c2, t);
}

// ------------------------------------------------------------------------------ Fp12
OVH_HD void fp12_one(Fp12& r) {
  fp6_one(r.c0);
  fp6_zero(r.c1);
}
OVH_HD bool fp12_eq(const Fp12& a, const Fp12& b) { return fp6_eq(a.c0, b.c0) && fp6_eq(a.c1, b.c1); }
OVH_HD bool fp12_is_one(const Fp12& a) {
  Fp12 one;
  fp12_one(one);
  return fp12_eq(a, one);
}
OVH_HD void fp12_conj(Fp12& r, const Fp12& a) {
  r.c0 = a.c0;
  fp6_neg(r.c1, a.c1);
}
OVH_HDNI void fp12_mul(Fp12& r, const Fp12& a, const Fp12& b) {
  Fp6 t0, t1, s0, s1;
  fp6_mul(t0, a.c0, b.c0);
  fp6_mul(t1, a.c1, b.c1);
  fp6_add(s0, a.c0, a.c1);
  fp6_add(s1, b.c0, b.c1);
  fp6_mul(s0, s0, s1);
  fp6_sub(s0, s0, t0);
  fp6_sub(r.c1, s0, t1);
  fp6_mul_v(t1, t1);
  fp6_add(r.c0, t0, t1);
}
// complex squaring: 2 Fp6 products
OVH_HDNI void fp12_sqr(Fp12& r, const Fp12& a) {
  Fp6 t, s0, s1, vt;
  fp6_mul(t, a.c0, a.c1);
  fp6_add(s0, a.c0, a.c1);
  fp6_mul_v(s1, a.c1);
  fp6_add(s1, s1, a.c0);
  fp6_mul(s0, s0, s1);
  fp6_mul_v(vt, t);
  fp6_sub(s0, s0, t);
  fp6_sub(r.c0, s0, vt);
  fp6_add(r.c1, t, t);
}
// f * (l0 + l1 v + l4 v w): sparse line product, 13 Fp2 products
OVH_HDNI void fp12_mul_by_014(Fp12& f, const Fp2& l0, const Fp2& l1, const Fp2& l4) {
  Fp6 t0, t1, s;
  Fp2 l14;
  fp6_mul_01(t0, f.c0, l0, l1);
  fp6_mul_1(t1, f.c1, l4);
  fp6_add(s, f.c0, f.c1);
  fp2_add(l14, l1, l4);
  fp6_mul_01(s, s, l0, l14);
  fp6_sub(s, s, t0);
  fp6_sub(f.c1, s, t1);
  fp6_mul_v(t1, t1);
  fp6_add(f.c0, t0, t1);
}
OVH_HDNI void fp12_inv(Fp12& r, const Fp12& a) {
  Fp6 t0, t1;
  fp6_mul(t0, a.c0, a.c0);
  fp6_mul(t1, a.c1, a.c1);
  fp6_mul_v(t1, t1);
  fp6_sub(t0, t0, t1);
  fp6_inv(t0, t0);
  fp6_mul(r.c0, a.c0, t0);
  fp6_mul(t1, a.c1, t0);
  fp6_neg(r.c1, t1);
}
// Frobenius f^p: coefficient of w^k (k = 2i + j for v^i w^j) -> conj(coef) * gamma_k.
OVH_HDNI void fp12_frob(Fp12& r, const Fp12& a) {
  Fp2 t;
  fp2_conj(r.c0.c0, a.c0.c0);                      // w^0
  fp2_conj(t, a.c1.c0);                            // w^1
  fp2_mul(r.c1.c0, t, fp2_const(FROB_G1_C0, FROB_G1_C1));
  fp2_conj(t, a.c0.c1);                            // w^2
  fp2_mul(r.c0.c1, t, fp2_const(FROB_G2_C0, FROB_G2_C1));
  fp2_conj(t, a.c1.c1);                            // w^3
  fp2_mul(r.c1.c1, t, fp2_const(FROB_G3_C0, FROB_G3_C1));
  fp2_conj(t, a.c0.c2);                            // w^4
  fp2_mul(r.c0.c2, t, fp2_const(FROB_G4_C0, FROB_G4_C1));
  fp2_conj(t, a.c1.c2);                            // w^5
  fp2_mul(r.c1.c2, t, fp2_const(FROB_G5_C0, FROB_G5_C1));
}
// Granger-Scott squaring, valid in the cyclotomic subgroup (after the easy part).
OVH_HDNI void fp12_cyc_sqr(Fp12& f, const Fp12& a) {
  const Fp2& r0 = a.c0.c0;
  const Fp2& r4 = a.c0.c1;
  const Fp2& r3 = a.c0.c2;
  const Fp2& r2 = a.c1.c0;
  const Fp2& r1 = a.c1.c1;
  const Fp2& r5 = a.c1.c2;
  Fp2 t0, t1, t2, t3, t4, t5, tmp, s, u;
  // (t0 + t1 y) = (r0 + r1 y)^2
  fp2_mul(tmp, r0, r1);
  fp2_add(s, r0, r1);
  fp2_mul_xi(u, r1);
  fp2_add(u, u, r0);
  fp2_mul(t0, s, u);
  fp2_sub(t0, t0, tmp);
  fp2_mul_xi(u, tmp);
  fp2_sub(t0, t0, u);
  fp2_dbl(t1, tmp);
  // (t2 + t3 y) = (r2 + r3 y)^2
  fp2_mul(tmp, r2, r3);
  fp2_add(s, r2, r3);
  fp2_mul_xi(u, r3);
  fp2_add(u, u, r2);
  fp2_mul(t2, s, u);
  fp2_sub(t2, t2, tmp);
  fp2_mul_xi(u, tmp);
  fp2_sub(t2, t2, u);
  fp2_dbl(t3, tmp);
  // (t4 + t5 y) = (r4 + r5 y)^2
  fp2_mul(tmp, r4, r5);
  fp2_add(s, r4, r5);
  fp2_mul_xi(u, r5);
  fp2_add(u, u, r4);
  fp2_mul(t4, s, u);
  fp2_sub(t4, t4, tmp);
  fp2_mul_xi(u, tmp);
  fp2_sub(t4, t4, u);
  fp2_dbl(t5, tmp);
  Fp2 z0 = a.c0.c0, z4 = a.c0.c1, z3 = a.c0.c2, z2 = a.c1.c0, z1 = a.c1.c1, z5 = a.c1.c2;
  // z0 = 3 t0 - 2 z0
  fp2_sub(z0, t0, z0);
  fp2_dbl(z0, z0);
  fp2_add(z0, z0, t0);
  // z1 = 3 t1 + 2 z1
  fp2_add(z1, t1, z1);
  fp2_dbl(z1, z1);
  fp2_add(z1, z1, t1);
  // z2 = 3 xi t5 + 2 z2
  fp2_mul_xi(tmp, t5);
  fp2_add(z2, z2, tmp);
  fp2_dbl(z2, z2);
  fp2_add(z2, z2, tmp);
  // z3 = 3 t4 - 2 z3
  fp2_sub(z3, t4, z3);
  fp2_dbl(z3, z3);
  fp2_add(z3, z3, t4);
  // z4 = 3 t2 - 2 z4
  fp2_sub(z4, t2, z4);
  fp2_dbl(z4, z4);
  fp2_add(z4, z4, t2);
  // z5 = 3 t3 + 2 z5
  fp2_add(z5, z5, t3);
  fp2_dbl(z5, z5);
  fp2_add(z5, z5, t3);
  f.c0.c0 = z0;
  f.c0.c1 = z4;
  f.c0.c2 = z3;
  f.c1.c0 = z2;
  f.c1.c1 = z1;
  f.c1.c2 = z5;
}

}  // namespace ovh
