// Curve arithmetic on E1 : y^2 = x^3 + 4 over Fp (G1, public keys) and the M-type twist
// E2 : y^2 = x^3 + 4(1+u) over Fp2 (G2, signatures). Jacobian coordinates (x = X/Z^2,
// y = Y/Z^3), Z == 0 is the point at infinity.
#pragma once
#include "tower.hpp"

namespace ovh {

// ---- field-generic shims so point code is written once ----
OVH_HD void f_add(Fp& r, const Fp& a, const Fp& b) { fp_add(r, a, b); }
OVH_HD void f_sub(Fp& r, const Fp& a, const Fp& b) { fp_sub(r, a, b); }
OVH_HD void f_dbl(Fp& r, const Fp& a) { fp_add(r, a, a); }
OVH_HD void f_mul(Fp& r, const Fp& a, const Fp& b) { fp_mul(r, a, b); }
OVH_HD void f_sqr(Fp& r, const Fp& a) { fp_sqr(r, a); }
OVH_HD void f_neg(Fp& r, const Fp& a) { fp_neg(r, a); }
OVH_HD bool f_is_zero(const Fp& a) { return fp_is_zero(a); }
OVH_HD bool f_eq(const Fp& a, const Fp& b) { return fp_eq(a, b); }
OVH_HD void f_one(Fp& r) { fp_one(r); }
OVH_HD void f_zero(Fp& r) { fp_zero(r); }
OVH_HD void f_inv(Fp& r, const Fp& a) { fp_inv(r, a); }
OVH_HD void f_add(Fp2& r, const Fp2& a, const Fp2& b) { fp2_add(r, a, b); }
OVH_HD void f_sub(Fp2& r, const Fp2& a, const Fp2& b) { fp2_sub(r, a, b); }
OVH_HD void f_dbl(Fp2& r, const Fp2& a) { fp2_dbl(r, a); }
OVH_HD void f_mul(Fp2& r, const Fp2& a, const Fp2& b) { fp2_mul(r, a, b); }
OVH_HD void f_sqr(Fp2& r, const Fp2& a) { fp2_sqr(r, a); }
OVH_HD void f_neg(Fp2& r, const Fp2& a) { fp2_neg(r, a); }
OVH_HD bool f_is_zero(const Fp2& a) { return fp2_is_zero(a); }
OVH_HD bool f_eq(const Fp2& a, const Fp2& b) { return fp2_eq(a, b); }
OVH_HD void f_one(Fp2& r) { fp2_one(r); }
OVH_HD void f_zero(Fp2& r) { fp2_zero(r); }
OVH_HD void f_inv(Fp2& r, const Fp2& a) { fp2_inv(r, a); }

template <class F>
struct Jac {
  F X, Y, Z;
};
template <class F>
struct Aff {
  F x, y;
};
typedef Jac<Fp> G1J;
typedef Jac<Fp2> G2J;
typedef Aff<Fp> G1A;
typedef Aff<Fp2> G2A;

template <class F>
OVH_HD void jac_set_inf(Jac<F>& r) {
  f_one(r.X);
  f_one(r.Y);
  f_zero(r.Z);
}
template <class F>
OVH_HD bool jac_is_inf(const Jac<F>& a) {
  return f_is_zero(a.Z);
}
template <class F>
OVH_HD void jac_from_aff(Jac<F>& r, const Aff<F>& a) {
  r.X = a.x;
  r.Y = a.y;
  f_one(r.Z);
}
template <class F>
OVH_HD void jac_neg(Jac<F>& r, const Jac<F>& a) {
  r.X = a.X;
  f_neg(r.Y, a.Y);
  r.Z = a.Z;
}

// dbl-2009-l (a = 0)
template <class F>
OVH_HDNI void jac_dbl(Jac<F>& r, const Jac<F>& p) {
  F A, B, C, D, E, Fv, t;
  f_sqr(A, p.X);
  f_sqr(B, p.Y);
  f_sqr(C, B);
  f_add(t, p.X, B);
  f_sqr(t, t);
  f_sub(t, t, A);
  f_sub(t, t, C);
  f_dbl(D, t);
  f_dbl(E, A);
  f_add(E, E, A);
  f_sqr(Fv, E);
  F Z3;
  f_mul(Z3, p.Y, p.Z);
  f_dbl(Z3, Z3);
  F X3;
  f_dbl(t, D);
  f_sub(X3, Fv, t);
  F Y3;
  f_sub(t, D, X3);
  f_mul(Y3, E, t);
  f_dbl(C, C);
  f_dbl(C, C);
  f_dbl(C, C);
  f_sub(Y3, Y3, C);
  r.X = X3;
  r.Y = Y3;
  r.Z = Z3;
}

// madd-2007-bl: r = p + q with q affine (q not infinity)
template <class F>
OVH_HDNI void jac_add_aff(Jac<F>& r, const Jac<F>& p, const Aff<F>& q) {
  if (jac_is_inf(p)) {
    jac_from_aff(r, q);
    return;
  }
  F Z1Z1, U2, S2, H, HH, I, J, rr, V, t;
  f_sqr(Z1Z1, p.Z);
  f_mul(U2, q.x, Z1Z1);
  f_mul(S2, q.y, p.Z);
  f_mul(S2, S2, Z1Z1);
  f_sub(H, U2, p.X);
  f_sub(rr, S2, p.Y);
  if (f_is_zero(H)) {
    if (f_is_zero(rr)) {
      Jac<F> qq;
      jac_from_aff(qq, q);
      jac_dbl(r, qq);
    } else {
      jac_set_inf(r);
    }
    return;
  }
  f_dbl(rr, rr);
  f_sqr(HH, H);
  f_dbl(I, HH);
  f_dbl(I, I);
  f_mul(J, H, I);
  f_mul(V, p.X, I);
  F X3, Y3, Z3;
  f_sqr(X3, rr);
  f_sub(X3, X3, J);
  f_sub(X3, X3, V);
  f_sub(X3, X3, V);
  f_sub(t, V, X3);
  f_mul(Y3, rr, t);
  f_mul(t, p.Y, J);
  f_dbl(t, t);
  f_sub(Y3, Y3, t);
  f_add(Z3, p.Z, H);
  f_sqr(Z3, Z3);
  f_sub(Z3, Z3, Z1Z1);
  f_sub(Z3, Z3, HH);
  r.X = X3;
  r.Y = Y3;
  r.Z = Z3;
}

// add-2007-bl: general Jacobian addition with all special cases
template <class F>
OVH_HDNI void jac_add(Jac<F>& r, const Jac<F>& p, const Jac<F>& q) {
  if (jac_is_inf(p)) {
    r = q;
    return;
  }
  if (jac_is_inf(q)) {
    r = p;
    return;
  }
  F Z1Z1, Z2Z2, U1, U2, S1, S2, H, I, J, rr, V, t;
  f_sqr(Z1Z1, p.Z);
  f_sqr(Z2Z2, q.Z);
  f_mul(U1, p.X, Z2Z2);
  f_mul(U2, q.X, Z1Z1);
  f_mul(S1, p.Y, q.Z);
  f_mul(S1, S1, Z2Z2);
  f_mul(S2, q.Y, p.Z);
  f_mul(S2, S2, Z1Z1);
  f_sub(H, U2, U1);
  f_sub(rr, S2, S1);
  if (f_is_zero(H)) {
    if (f_is_zero(rr)) {
      jac_dbl(r, p);
    } else {
      jac_set_inf(r);
    }
    return;
  }
  f_dbl(rr, rr);
  f_dbl(I, H);
  f_sqr(I, I);
  f_mul(J, H, I);
  f_mul(V, U1, I);
  F X3, Y3, Z3;
  f_sqr(X3, rr);
  f_sub(X3, X3, J);
  f_sub(X3, X3, V);
  f_sub(X3, X3, V);
  f_sub(t, V, X3);
  f_mul(Y3, rr, t);
  f_mul(t, S1, J);
  f_dbl(t, t);
  f_sub(Y3, Y3, t);
  f_add(Z3, p.Z, q.Z);
  f_sqr(Z3, Z3);
  f_sub(Z3, Z3, Z1Z1);
  f_sub(Z3, Z3, Z2Z2);
  f_mul(Z3, Z3, H);
  r.X = X3;
  r.Y = Y3;
  r.Z = Z3;
}

// Equality of two Jacobian points (projective comparison).
template <class F>
OVH_HDNI bool jac_eq(const Jac<F>& p, const Jac<F>& q) {
  bool pi = jac_is_inf(p), qi = jac_is_inf(q);
  if (pi || qi) return pi && qi;
  F z1z1, z2z2, a, b, c, d;
  f_sqr(z1z1, p.Z);
  f_sqr(z2z2, q.Z);
  f_mul(a, p.X, z2z2);
  f_mul(b, q.X, z1z1);
  if (!f_eq(a, b)) return false;
  f_mul(c, p.Y, q.Z);
  f_mul(c, c, z2z2);
  f_mul(d, q.Y, p.Z);
  f_mul(d, d, z1z1);
  return f_eq(c, d);
}

// Affine conversion: returns false for infinity.
template <class F>
OVH_HDNI bool jac_to_aff(Aff<F>& r, const Jac<F>& p) {
  if (jac_is_inf(p)) return false;
  F zi, zi2, zi3;
  f_inv(zi, p.Z);
  f_sqr(zi2, zi);
  f_mul(zi3, zi2, zi);
  f_mul(r.x, p.X, zi2);
  f_mul(r.y, p.Y, zi3);
  return true;
}

// r = [k] p for a 64-bit scalar, double-and-add from the MSB (p affine, not infinity).
template <class F>
OVH_HDNI void jac_mul_u64(Jac<F>& r, const Aff<F>& p, uint64_t k) {
  Jac<F> acc;
  jac_set_inf(acc);
#pragma unroll 1
  for (int b = 63; b >= 0; --b) {
    jac_dbl(acc, acc);
    if ((k >> b) & 1) jac_add_aff(acc, acc, p);
  }
  r = acc;
}

// r = [k] p for a 64-bit scalar with p in Jacobian coordinates.
template <class F>
OVH_HDNI void jac_mul_u64_jac(Jac<F>& r, const Jac<F>& p, uint64_t k) {
  Jac<F> acc;
  jac_set_inf(acc);
#pragma unroll 1
  for (int b = 63; b >= 0; --b) {
    jac_dbl(acc, acc);
    if ((k >> b) & 1) jac_add(acc, acc, p);
  }
  r = acc;
}

// r = [k] p for a multi-word scalar (nwords little-endian 32-bit words), p Jacobian.
template <class F>
OVH_HDNI void jac_mul_words(Jac<F>& r, const Jac<F>& p, const uint32_t* k, int nwords) {
  Jac<F> acc;
  jac_set_inf(acc);
#pragma unroll 1
  for (int w = nwords - 1; w >= 0; --w) {
    const uint32_t kw = k[w];
#pragma unroll 1
    for (int b = 31; b >= 0; --b) {
      jac_dbl(acc, acc);
      if ((kw >> b) & 1) jac_add(acc, acc, p);
    }
  }
  r = acc;
}

// r = [|x|] p, |x| = 0xd201000000010000 (63 doublings + 5 additions).
template <class F>
OVH_HD void jac_mul_xabs(Jac<F>& r, const Jac<F>& p) { jac_mul_u64_jac(r, p, X_ABS); }

// ------------------------------------------------------------------ G2 endomorphisms
OVH_HD void g2_psi(G2J& r, const G2J& p) {
  Fp2 t;
  fp2_conj(t, p.X);
  fp2_mul(r.X, t, fp2_const(PSI_CX_C0, PSI_CX_C1));
  fp2_conj(t, p.Y);
  fp2_mul(r.Y, t, fp2_const(PSI_CY_C0, PSI_CY_C1));
  fp2_conj(r.Z, p.Z);
}
OVH_HD void g2_psi2(G2J& r, const G2J& p) {
  fp2_mul(r.X, p.X, fp2_const(PSI2_CX_C0, PSI2_CX_C1));
  fp2_mul(r.Y, p.Y, fp2_const(PSI2_CY_C0, PSI2_CY_C1));
  r.Z = p.Z;
}

// Q in G2  <=>  psi(Q) == [x] Q  (Scott 2021; x = -|x|)
OVH_HDNI bool g2_in_subgroup(const G2J& q) {
  if (jac_is_inf(q)) return true;
  G2J xq, pq;
  jac_mul_xabs(xq, q);
  jac_neg(xq, xq);
  g2_psi(pq, q);
  return jac_eq(pq, xq);
}

// P in G1  <=>  phi(P) == [-x^2] P with phi(x, y) = (beta x, y)
OVH_HDNI bool g1_in_subgroup(const G1J& p) {
  if (jac_is_inf(p)) return true;
  G1J t, phi;
  jac_mul_xabs(t, p);
  jac_mul_xabs(t, t);
  jac_neg(t, t);
  fp_mul(phi.X, p.X, fp_const(BETA_M));
  phi.Y = p.Y;
  phi.Z = p.Z;
  return jac_eq(phi, t);
}

// h_eff * P = [x^2 - x - 1] P + [x - 1] psi(P) + psi^2(2P)   (RFC 9380 8.8.2)
OVH_HDNI void g2_clear_cofactor(G2J& r, const G2J& p) {
  G2J t1, t2, t3, u;
  jac_mul_xabs(t1, p);
  jac_neg(t1, t1);  // t1 = [x] P
  g2_psi(t2, p);    // t2 = psi(P)
  jac_dbl(t3, p);
  g2_psi2(t3, t3);  // t3 = psi2(2P)
  jac_neg(u, t2);
  jac_add(t3, t3, u);  // t3 = psi2(2P) - psi(P)
  jac_add(t2, t1, t2);  // t2 = [x]P + psi(P)
  jac_mul_xabs(t2, t2);
  jac_neg(t2, t2);  // t2 = [x]([x]P + psi(P))
  jac_add(t3, t3, t2);
  jac_neg(u, t1);
  jac_add(t3, t3, u);  // - [x] P
  jac_neg(u, p);
  jac_add(r, t3, u);  // - P
}

// ------------------------------------------------------------------ serialization
enum : int {
  BLST_SUCCESS = 0,
  BLST_BAD_ENCODING = 1,
  BLST_POINT_NOT_ON_CURVE = 2,
  BLST_POINT_NOT_IN_GROUP = 3,
  BLST_AGGR_TYPE_MISMATCH = 4,
  BLST_VERIFY_FAIL = 5,
  BLST_PK_IS_INFINITY = 6,
  BLST_BAD_SCALAR = 7,
};

OVH_HD bool bytes_zero(const uint8_t* b, int n) {
  uint32_t acc = 0;
  for (int i = 0; i < n; ++i) acc |= b[i];
  return acc == 0;
}

// Parse a field element from 48 BE bytes with the top 3 bits masked off; returns false if >= p.
OVH_HD bool fp_from_be48_masked(Fp& r, const uint8_t* in, bool mask_top) {
  uint32_t l[12];
  limbs_from_be48(l, in);
  if (mask_top) l[11] &= 0x1fffffffu;
  if (!limbs_lt_p(l)) return false;
  Fp t;
  for (int i = 0; i < 12; ++i) t.v[i] = l[i];
  fp_to_mont(r, t);
  return true;
}

// blst PublicKey::from_bytes semantics: 48-byte compressed (0x80 set) or 96-byte
// uncompressed (0x80 clear). On success *inf says whether it is the point at infinity.
OVH_HDNI int g1_from_bytes(G1A& out, bool& inf, const uint8_t* in, uint32_t len) {
  inf = false;
  if (len == 0) return BLST_BAD_ENCODING;
  const uint8_t b0 = in[0];
  if (len == 48 && (b0 & 0x80)) {
    if (b0 & 0x40) {
      if ((b0 & 0x3f) == 0 && bytes_zero(in + 1, 47)) {
        inf = true;
        return BLST_SUCCESS;
      }
      return BLST_BAD_ENCODING;
    }
    Fp x;
    if (!fp_from_be48_masked(x, in, true)) return BLST_BAD_ENCODING;
    Fp y2, y;
    fp_sqr(y2, x);
    fp_mul(y2, y2, x);
    fp_add(y2, y2, fp_const(B1_M));
    if (!fp_sqrt(y, y2)) return BLST_POINT_NOT_ON_CURVE;
    const bool want = (b0 & 0x20) != 0;
    if (fp_lex_largest(y) != want) fp_neg(y, y);
    out.x = x;
    out.y = y;
    if (fp_is_zero(x)) return BLST_POINT_NOT_IN_GROUP;
    return BLST_SUCCESS;
  }
  if (len == 96 && !(b0 & 0x80)) {
    if (b0 & 0x40) {
      if ((b0 & 0x3f) == 0 && bytes_zero(in + 1, 95)) {
        inf = true;
        return BLST_SUCCESS;
      }
      return BLST_BAD_ENCODING;
    }
    if (b0 & 0x20) return BLST_BAD_ENCODING;
    Fp x, y;
    if (!fp_from_be48_masked(x, in, true)) return BLST_BAD_ENCODING;
    if (!fp_from_be48_masked(y, in + 48, false)) return BLST_BAD_ENCODING;
    Fp l, rr;
    fp_sqr(l, y);
    fp_sqr(rr, x);
    fp_mul(rr, rr, x);
    fp_add(rr, rr, fp_const(B1_M));
    if (!fp_eq(l, rr)) return BLST_POINT_NOT_ON_CURVE;
    out.x = x;
    out.y = y;
    if (fp_is_zero(x)) return BLST_POINT_NOT_IN_GROUP;
    return BLST_SUCCESS;
  }
  return BLST_BAD_ENCODING;
}

// blst Signature::from_bytes semantics: 96-byte compressed or 192-byte uncompressed.
OVH_HDNI int g2_from_bytes(G2A& out, bool& inf, const uint8_t* in, uint32_t len) {
  inf = false;
  if (len == 0) return BLST_BAD_ENCODING;
  const uint8_t b0 = in[0];
  if (len == 96 && (b0 & 0x80)) {
    if (b0 & 0x40) {
      if ((b0 & 0x3f) == 0 && bytes_zero(in + 1, 95)) {
        inf = true;
        return BLST_SUCCESS;
      }
      return BLST_BAD_ENCODING;
    }
    Fp2 x;
    if (!fp_from_be48_masked(x.c1, in, true)) return BLST_BAD_ENCODING;
    if (!fp_from_be48_masked(x.c0, in + 48, false)) return BLST_BAD_ENCODING;
    Fp2 y2, y;
    fp2_sqr(y2, x);
    fp2_mul(y2, y2, x);
    fp2_add(y2, y2, fp2_const(B2_C0, B2_C1));
    if (!fp2_sqrt(y, y2)) return BLST_POINT_NOT_ON_CURVE;
    const bool want = (b0 & 0x20) != 0;
    if (fp2_lex_largest(y) != want) fp2_neg(y, y);
    out.x = x;
    out.y = y;
    if (fp2_is_zero(x)) return BLST_POINT_NOT_IN_GROUP;
    return BLST_SUCCESS;
  }
  if (len == 192 && !(b0 & 0x80)) {
    if (b0 & 0x40) {
      if ((b0 & 0x3f) == 0 && bytes_zero(in + 1, 191)) {
        inf = true;
        return BLST_SUCCESS;
      }
      return BLST_BAD_ENCODING;
    }
    if (b0 & 0x20) return BLST_BAD_ENCODING;
    Fp2 x, y;
    if (!fp_from_be48_masked(x.c1, in, true)) return BLST_BAD_ENCODING;
    if (!fp_from_be48_masked(x.c0, in + 48, false)) return BLST_BAD_ENCODING;
    if (!fp_from_be48_masked(y.c1, in + 96, false)) return BLST_BAD_ENCODING;
    if (!fp_from_be48_masked(y.c0, in + 144, false)) return BLST_BAD_ENCODING;
    Fp2 l, rr;
    fp2_sqr(l, y);
    fp2_sqr(rr, x);
    fp2_mul(rr, rr, x);
    fp2_add(rr, rr, fp2_const(B2_C0, B2_C1));
    if (!fp2_eq(l, rr)) return BLST_POINT_NOT_ON_CURVE;
    out.x = x;
    out.y = y;
    if (fp2_is_zero(x)) return BLST_POINT_NOT_IN_GROUP;
    return BLST_SUCCESS;
  }
  return BLST_BAD_ENCODING;
}

// Compressed encodings (ZCash). Infinity -> 0xc0 || zeros.
OVH_HD void g1_compress(uint8_t* out, const G1J& p) {
  G1A a;
  if (!jac_to_aff(a, p)) {
    out[0] = 0xc0;
    for (int i = 1; i < 48; ++i) out[i] = 0;
    return;
  }
  fp_to_be48(out, a.x);
  out[0] |= 0x80 | (fp_lex_largest(a.y) ? 0x20 : 0);
}
OVH_HD void g2_compress(uint8_t* out, const G2J& p) {
  G2A a;
  if (!jac_to_aff(a, p)) {
    out[0] = 0xc0;
    for (int i = 1; i < 96; ++i) out[i] = 0;
    return;
  }
  fp_to_be48(out, a.x.c1);
  fp_to_be48(out + 48, a.x.c0);
  out[0] |= 0x80 | (fp2_lex_largest(a.y) ? 0x20 : 0);
}
// Uncompressed (96/192 bytes), used for point hand-off in tests.
OVH_HD void g2_serialize(uint8_t* out, const G2J& p) {
  G2A a;
  if (!jac_to_aff(a, p)) {
    out[0] = 0x40;
    for (int i = 1; i < 192; ++i) out[i] = 0;
    return;
  }
  fp_to_be48(out, a.x.c1);
  fp_to_be48(out + 48, a.x.c0);
  fp_to_be48(out + 96, a.y.c1);
  fp_to_be48(out + 144, a.y.c0);
}

}  // namespace ovh
