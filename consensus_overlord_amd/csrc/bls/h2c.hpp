// Hash to G2 (RFC 9380, suite BLS12381G2_XMD:SHA-256_SSWU_RO_), message = the 32-byte
// vote digest (ophelia HashValue, src/consensus.rs:403, 412). expand_message_xmd runs on
// per-DST block templates prepared once on the host (XmdTemplates), so the device only
// injects the 32 variable bytes per block chain and runs the SHA-256 compressions.
#pragma once
#include "ec.hpp"

namespace ovh {

// ------------------------------------------------------------------ SHA-256
OVH_HD uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

OVH_HD void sha256_compress(uint32_t st[8], const uint32_t blk[16]) {
  const uint32_t K[64] = {
      0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
      0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
      0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
      0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
      0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
      0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
      0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
      0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) w[i] = blk[i];
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      const uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
      const uint32_t s0 = rotr32(w15, 7) ^ rotr32(w15, 18) ^ (w15 >> 3);
      const uint32_t s1 = rotr32(w2, 17) ^ rotr32(w2, 19) ^ (w2 >> 10);
      wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
      w[i & 15] = wi;
    }
    const uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
    const uint32_t ch = (e & f) ^ (~e & g);
    const uint32_t t1 = h + S1 + ch + K[i] + wi;
    const uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
    const uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    const uint32_t t2 = S0 + mj;
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  st[0] += a;
  st[1] += b;
  st[2] += c;
  st[3] += d;
  st[4] += e;
  st[5] += f;
  st[6] += g;
  st[7] += h;
}

OVH_HD void sha256_iv(uint32_t st[8]) {
  st[0] = 0x6a09e667u;
  st[1] = 0xbb67ae85u;
  st[2] = 0x3c6ef372u;
  st[3] = 0xa54ff53au;
  st[4] = 0x510e527fu;
  st[5] = 0x9b05688cu;
  st[6] = 0x1f83d9abu;
  st[7] = 0x5be0cd19u;
}

// Padded SHA-256 blocks for expand_message_xmd(msg[32], DST, 256) with the variable 32
// bytes at words 0..7 of the first template block of each chain.
//   b_0 = H(Z_pad || msg || I2OSP(256,2) || 0x00 || DST || len)   -> state after Z_pad = mid0
//   b_i = H(strxor(b_0, b_{i-1}) || I2OSP(i,1) || DST || len)      -> counter byte at byte 32
#define OVH_XMD_MAX_BLOCKS 4
struct XmdTemplates {
  uint32_t mid0[8];                        // SHA-256 state after the all-zero Z_pad block
  uint32_t b0[OVH_XMD_MAX_BLOCKS][16];     // blocks after Z_pad (words 0..7 of b0[0] <- msg)
  uint32_t bi[OVH_XMD_MAX_BLOCKS][16];     // words 0..7 of bi[0] <- xor; word 8 |= i << 24
  uint32_t nb0, nbi;
};

// Host-side template construction (also callable in the host test build).
inline bool xmd_build_templates(XmdTemplates& t, const uint8_t* dst, uint32_t dst_len) {
  if (dst_len > 255) return false;
  uint8_t buf[OVH_XMD_MAX_BLOCKS * 64];
  // b0 tail: msg(32) | 0x01 0x00 | 0x00 | DST | len, then padding; total message = 64 + 36 + L
  {
    const uint32_t body = 36 + dst_len, total = 64 + body;
    const uint32_t nb = (body + 9 + 63) / 64;
    if (nb > OVH_XMD_MAX_BLOCKS) return false;
    for (uint32_t i = 0; i < nb * 64; ++i) buf[i] = 0;
    buf[32] = 0x01;
    buf[33] = 0x00;
    buf[34] = 0x00;
    for (uint32_t i = 0; i < dst_len; ++i) buf[35 + i] = dst[i];
    buf[35 + dst_len] = (uint8_t)dst_len;
    buf[body] = 0x80;
    const uint64_t bits = (uint64_t)total * 8;
    for (int i = 0; i < 8; ++i) buf[nb * 64 - 1 - i] = (uint8_t)(bits >> (8 * i));
    for (uint32_t b = 0; b < OVH_XMD_MAX_BLOCKS; ++b)
      for (int w = 0; w < 16; ++w) {
        uint32_t v = 0;
        if (b < nb) {
          const uint8_t* p = buf + b * 64 + 4 * w;
          v = ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
        }
        t.b0[b][w] = v;
      }
    t.nb0 = nb;
  }
  {
    const uint32_t body = 34 + dst_len;
    const uint32_t nb = (body + 9 + 63) / 64;
    if (nb > OVH_XMD_MAX_BLOCKS) return false;
    for (uint32_t i = 0; i < nb * 64; ++i) buf[i] = 0;
    for (uint32_t i = 0; i < dst_len; ++i) buf[33 + i] = dst[i];
    buf[33 + dst_len] = (uint8_t)dst_len;
    buf[body] = 0x80;
    const uint64_t bits = (uint64_t)body * 8;
    for (int i = 0; i < 8; ++i) buf[nb * 64 - 1 - i] = (uint8_t)(bits >> (8 * i));
    for (uint32_t b = 0; b < OVH_XMD_MAX_BLOCKS; ++b)
      for (int w = 0; w < 16; ++w) {
        uint32_t v = 0;
        if (b < nb) {
          const uint8_t* p = buf + b * 64 + 4 * w;
          v = ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
        }
        t.bi[b][w] = v;
      }
    t.nbi = nb;
  }
  uint32_t zero[16] = {0};
  sha256_iv(t.mid0);
  sha256_compress(t.mid0, zero);
  return true;
}

// msg32 as 8 big-endian words -> 64 big-endian words of uniform bytes.
OVH_HD void expand_message_xmd_256(uint32_t out[64], const uint32_t msg[8], const XmdTemplates& t) {
  uint32_t b0[8], st[8], blk[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) st[i] = t.mid0[i];
#pragma unroll 1
  for (uint32_t b = 0; b < t.nb0; ++b) {
#pragma unroll
    for (int w = 0; w < 16; ++w) blk[w] = t.b0[b][w];
    if (b == 0) {
#pragma unroll
      for (int w = 0; w < 8; ++w) blk[w] = msg[w];
    }
    sha256_compress(st, blk);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) b0[i] = st[i];
  uint32_t prev[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) prev[i] = 0;
#pragma unroll 1
  for (uint32_t k = 1; k <= 8; ++k) {
    sha256_iv(st);
#pragma unroll 1
    for (uint32_t b = 0; b < t.nbi; ++b) {
#pragma unroll
      for (int w = 0; w < 16; ++w) blk[w] = t.bi[b][w];
      if (b == 0) {
#pragma unroll
        for (int w = 0; w < 8; ++w) blk[w] = b0[w] ^ prev[w];
        blk[8] |= k << 24;
      }
      sha256_compress(st, blk);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      prev[i] = st[i];
      out[(k - 1) * 8 + i] = st[i];
    }
  }
}

// 64 big-endian bytes (16 BE words) -> Fp (Montgomery): (H * 2^384 + L) mod p.
OVH_HD void fp_from_be64_words(Fp& r, const uint32_t* w) {
  Fp L, H, a, b;
#pragma unroll
  for (int i = 0; i < 12; ++i) L.v[i] = w[15 - i];
#pragma unroll
  for (int i = 0; i < 12; ++i) H.v[i] = i < 4 ? w[3 - i] : 0u;
  // first operand must be < p (CIOS bound); the raw limbs go second
  fp_mul(a, fp_const(R2_M), L);
  fp_mul(b, fp_const(R3_M), H);
  fp_add(r, a, b);
}

OVH_HD void hash_to_field_fp2x2(Fp2& u0, Fp2& u1, const uint32_t uniform[64]) {
  fp_from_be64_words(u0.c0, uniform + 0);
  fp_from_be64_words(u0.c1, uniform + 16);
  fp_from_be64_words(u1.c0, uniform + 32);
  fp_from_be64_words(u1.c1, uniform + 48);
}

// ------------------------------------------------------------------ SSWU + iso map
OVH_HD void g2p_rhs(Fp2& r, const Fp2& x) {  // x^3 + A' x + B'
  Fp2 t;
  fp2_sqr(t, x);
  fp2_mul(t, t, x);
  Fp2 ax;
  fp2_mul(ax, x, fp2_const(SSWU_A_C0, SSWU_A_C1));
  fp2_add(t, t, ax);
  fp2_add(r, t, fp2_const(SSWU_B_C0, SSWU_B_C1));
}

// Simplified SWU onto E2' (RFC 9380 6.6.2); output affine (x, y) on E2'.
OVH_HDNI void map_to_curve_sswu(Fp2& xo, Fp2& yo, const Fp2& u) {
  Fp2 u2, zu2, tv1, x1, gx, y;
  fp2_sqr(u2, u);
  fp2_mul(zu2, u2, fp2_const(SSWU_Z_C0, SSWU_Z_C1));
  fp2_sqr(tv1, zu2);
  fp2_add(tv1, tv1, zu2);
  if (fp2_is_zero(tv1)) {
    x1 = fp2_const(SSWU_B_OVER_ZA_C0, SSWU_B_OVER_ZA_C1);
  } else {
    Fp2 inv;
    fp2_inv(inv, tv1);
    Fp2 one;
    fp2_one(one);
    fp2_add(inv, inv, one);
    fp2_mul(x1, inv, fp2_const(SSWU_NEG_B_OVER_A_C0, SSWU_NEG_B_OVER_A_C1));
  }
  g2p_rhs(gx, x1);
  if (fp2_sqrt(y, gx)) {
    xo = x1;
  } else {
    fp2_mul(xo, zu2, x1);
    g2p_rhs(gx, xo);
    fp2_sqrt(y, gx);
  }
  if (fp2_sgn0(u) != fp2_sgn0(y)) fp2_neg(y, y);
  yo = y;
}

OVH_HD void iso_horner(Fp2& acc, const Fp2& x, const uint32_t* const* c0, const uint32_t* const* c1, int n) {
  acc = fp2_const(c0[n - 1], c1[n - 1]);
  for (int k = n - 2; k >= 0; --k) {
    fp2_mul(acc, acc, x);
    fp2_add(acc, acc, fp2_const(c0[k], c1[k]));
  }
}

// 3-isogeny E2' -> E2, straight into Jacobian coordinates (no inversion):
//   Z = xd yd, X = xn xd yd^2, Y = y yn yd^2 xd^3  (x = xn/xd, y = y yn/yd).
OVH_HDNI void iso_map_g2(G2J& r, const Fp2& x, const Fp2& y) {
  const uint32_t* xn0[4] = {ISO_XNUM0_C0, ISO_XNUM1_C0, ISO_XNUM2_C0, ISO_XNUM3_C0};
  const uint32_t* xn1[4] = {ISO_XNUM0_C1, ISO_XNUM1_C1, ISO_XNUM2_C1, ISO_XNUM3_C1};
  const uint32_t* xd0[3] = {ISO_XDEN0_C0, ISO_XDEN1_C0, ISO_XDEN2_C0};
  const uint32_t* xd1[3] = {ISO_XDEN0_C1, ISO_XDEN1_C1, ISO_XDEN2_C1};
  const uint32_t* yn0[4] = {ISO_YNUM0_C0, ISO_YNUM1_C0, ISO_YNUM2_C0, ISO_YNUM3_C0};
  const uint32_t* yn1[4] = {ISO_YNUM0_C1, ISO_YNUM1_C1, ISO_YNUM2_C1, ISO_YNUM3_C1};
  const uint32_t* yd0[4] = {ISO_YDEN0_C0, ISO_YDEN1_C0, ISO_YDEN2_C0, ISO_YDEN3_C0};
  const uint32_t* yd1[4] = {ISO_YDEN0_C1, ISO_YDEN1_C1, ISO_YDEN2_C1, ISO_YDEN3_C1};
  Fp2 xn, xd, yn, yd, t, yd2;
  iso_horner(xn, x, xn0, xn1, 4);
  iso_horner(xd, x, xd0, xd1, 3);
  iso_horner(yn, x, yn0, yn1, 4);
  iso_horner(yd, x, yd0, yd1, 4);
  fp2_mul(r.Z, xd, yd);
  fp2_sqr(yd2, yd);
  fp2_mul(t, xn, xd);
  fp2_mul(r.X, t, yd2);
  fp2_sqr(t, xd);
  fp2_mul(t, t, xd);
  fp2_mul(t, t, yd2);
  fp2_mul(t, t, yn);
  fp2_mul(r.Y, t, y);
}

// Full hash_to_curve for one 32-byte message (single lane).
OVH_HDNI void hash_to_g2(G2J& r, const uint32_t msg[8], const XmdTemplates& t) {
  uint32_t uni[64];
  expand_message_xmd_256(uni, msg, t);
  Fp2 u0, u1, x, y;
  hash_to_field_fp2x2(u0, u1, uni);
  G2J q0, q1;
  map_to_curve_sswu(x, y, u0);
  iso_map_g2(q0, x, y);
  map_to_curve_sswu(x, y, u1);
  iso_map_g2(q1, x, y);
  jac_add(q0, q0, q1);
  g2_clear_cofactor(r, q0);
}

}  // namespace ovh
