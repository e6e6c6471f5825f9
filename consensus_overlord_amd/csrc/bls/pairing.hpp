// Optimal-ate pairing pieces: Miller loop f_{|x|,Q}(P) (conjugated, x < 0) with T in
// homogeneous projective coordinates and sparse "014" lines, and the final exponentiation
// f^(3(p^12-1)/r) through the x-chain 3 Phi12(p)/r = (x-1)^2 (x+p)(x^2+p^2-1) + 3.
// Formulas are restated from oracle/py/bls12_381.py (miller_loop_proj,
// final_exponentiation_x_chain), where they are checked against the textbook definitions.
#pragma once
#include "ec.hpp"

namespace ovh {

struct MillerP {  // per-P constants for line evaluation
  Fp m3x;        // -3 xP
  Fp nx;         // -xP
  Fp y;          // yP
  Fp y2;         // 2 yP
};

OVH_HD void miller_prep(MillerP& mp, const G1A& p) {
  Fp t;
  fp_add(t, p.x, p.x);
  fp_add(t, t, p.x);
  fp_neg(mp.m3x, t);
  fp_neg(mp.nx, p.x);
  mp.y = p.y;
  fp_add(mp.y2, p.y, p.y);
}

struct ProjT {
  Fp2 X, Y, Z;
};

// T <- 2T, returns line coefficients (l0, l1, l4)
OVH_HDNI void miller_dbl_step(ProjT& T, Fp2& l0, Fp2& l1, Fp2& l4, const MillerP& mp) {
  Fp2 XX, YY, ZZ, E, YZ, A, Fv, G, t;
  fp2_sqr(XX, T.X);
  fp2_sqr(YY, T.Y);
  fp2_sqr(ZZ, T.Z);
  fp2_mul(E, ZZ, fp2_const(B2X3_C0, B2X3_C1));  // 3 b' Z^2
  fp2_sub(l0, YY, E);
  fp2_mul_fp(l1, XX, mp.m3x);
  fp2_mul(YZ, T.Y, T.Z);
  fp2_mul_fp(l4, YZ, mp.y2);
  fp2_mul(A, T.X, T.Y);
  fp2_dbl(Fv, E);
  fp2_add(Fv, Fv, E);  // 9 b' Z^2
  fp2_sub(t, YY, Fv);
  fp2_mul(t, A, t);
  fp2_dbl(T.X, t);  // X3 = 2 X Y (Y^2 - 9b'Z^2)
  fp2_add(G, YY, Fv);
  fp2_sqr(G, G);
  fp2_sqr(t, E);
  fp2_mul_small(t, t, 12);
  fp2_sub(T.Y, G, t);  // Y3 = (Y^2 + 9b'Z^2)^2 - 12 (3b'Z^2)^2
  fp2_mul(t, YY, YZ);
  fp2_dbl(t, t);
  fp2_dbl(t, t);
  fp2_dbl(T.Z, t);  // Z3 = 8 Y^3 Z
}

// T <- T + Q (Q affine), returns line coefficients
OVH_HDNI void miller_add_step(ProjT& T, Fp2& l0, Fp2& l1, Fp2& l4, const G2A& q, const MillerP& mp) {
  Fp2 theta, lam, t, C, D, E, F, G, H;
  fp2_mul(t, q.y, T.Z);
  fp2_sub(theta, T.Y, t);
  fp2_mul(t, q.x, T.Z);
  fp2_sub(lam, T.X, t);
  fp2_mul(l0, theta, q.x);
  fp2_mul(t, lam, q.y);
  fp2_sub(l0, l0, t);
  fp2_mul_fp(l1, theta, mp.nx);
  fp2_mul_fp(l4, lam, mp.y);
  fp2_sqr(C, theta);
  fp2_sqr(D, lam);
  fp2_mul(E, D, lam);
  fp2_mul(F, T.Z, C);
  fp2_mul(G, T.X, D);
  fp2_add(H, E, F);
  fp2_sub(H, H, G);
  fp2_sub(H, H, G);
  fp2_mul(T.X, lam, H);
  fp2_sub(t, G, H);
  fp2_mul(t, theta, t);
  fp2_mul(C, T.Y, E);
  fp2_sub(T.Y, t, C);
  fp2_mul(T.Z, T.Z, E);
}

// f = Miller(P, Q) for P in G1 affine, Q in G2 affine (neither infinity).
OVH_HDNI void miller_loop(Fp12& f, const G1A& p, const G2A& q) {
  MillerP mp;
  miller_prep(mp, p);
  ProjT T;
  T.X = q.x;
  T.Y = q.y;
  fp2_one(T.Z);
  Fp2 l0, l1, l4;
  fp12_one(f);
  bool first = true;
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    miller_dbl_step(T, l0, l1, l4, mp);
    if (!first) fp12_sqr(f, f);
    fp12_mul_by_014(f, l0, l1, l4);
    first = false;
    if ((X_ABS >> b) & 1) {
      miller_add_step(T, l0, l1, l4, q, mp);
      fp12_mul_by_014(f, l0, l1, l4);
    }
  }
  fp12_conj(f, f);
}

// f^|x| in the cyclotomic subgroup
OVH_HDNI void fp12_cyc_exp_xabs(Fp12& r, const Fp12& f) {
  Fp12 acc = f;
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    fp12_cyc_sqr(acc, acc);
    if ((X_ABS >> b) & 1) fp12_mul(acc, acc, f);
  }
  r = acc;
}
// f^x = conj(f^|x|)
OVH_HD void fp12_cyc_exp_x(Fp12& r, const Fp12& f) {
  fp12_cyc_exp_xabs(r, f);
  fp12_conj(r, r);
}

// f^(3 (p^12 - 1)/r)
OVH_HDNI void final_exponentiation(Fp12& r, const Fp12& fin) {
  Fp12 f, t, u;
  // easy part: f^(p^6 - 1)(p^2 + 1)
  fp12_inv(t, fin);
  fp12_conj(f, fin);
  fp12_mul(f, f, t);
  fp12_frob(t, f);
  fp12_frob(t, t);
  fp12_mul(f, t, f);
  // t = f^((x-1)^2)
  fp12_cyc_exp_x(t, f);
  fp12_conj(u, f);
  fp12_mul(t, t, u);
  fp12_cyc_exp_x(u, t);
  fp12_conj(t, t);
  fp12_mul(t, u, t);
  // t = t^(x + p)
  fp12_cyc_exp_x(u, t);
  fp12_frob(t, t);
  fp12_mul(t, u, t);
  // t = t^(x^2 + p^2 - 1)
  fp12_cyc_exp_x(u, t);
  fp12_cyc_exp_x(u, u);
  Fp12 w;
  fp12_frob(w, t);
  fp12_frob(w, w);
  fp12_mul(u, u, w);
  fp12_conj(t, t);
  fp12_mul(t, u, t);
  // * f^3
  fp12_cyc_sqr(u, f);
  fp12_mul(u, u, f);
  fp12_mul(r, t, u);
}

}  // namespace ovh
