// Fp = GF(p), p the BLS12-381 base prime, as 12 x 32-bit limbs in Montgomery form.
//
// Device representation chosen for CDNA4: 32-bit limbs so every partial product is one
// v_mad_u64_u32 (measured on gfx950 at ~1.24x the issue cost of a v_add_u32,
// profiles/r01_int_rates_ubench.json), values kept fully reduced in [0, p). Because the top
// limb of p is < 2^31, the CIOS Montgomery product needs no 13th carry word.
//
// This header compiles for the gfx950 device (hipcc) and for the host (g++), so the exact
// device arithmetic can be unit-tested on a CPU; the host build is a test harness only and
// is never linked into the product library.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define OVH_HD __host__ __device__ __forceinline__
#define OVH_HDNI __host__ __device__ inline __attribute__((noinline))
#else
#define OVH_HD inline
#define OVH_HDNI inline
#endif

#include "consts.hpp"
#if defined(__HIP_DEVICE_COMPILE__)
#include "fp_mul_gfx950.hpp"
#include "fp_mul28.hpp"
#include "fp_mul28_gfx950.hpp"
#endif

namespace ovh {

// Host-only op counter for the work model (tools/count_muls.cpp); compiled out everywhere else.
#if defined(OVH_COUNT_MULS) && !defined(__HIP_DEVICE_COMPILE__)
extern unsigned long long g_fp_mul_count;
#define OVH_COUNT_MUL() (++::ovh::g_fp_mul_count)
#else
#define OVH_COUNT_MUL() ((void)0)
#endif

// 32-bit add/sub with carry: clang lowers the builtins to v_add_co/v_addc_co chains.
OVH_HD uint32_t addc32(uint32_t a, uint32_t b, uint32_t cin, uint32_t* cout) {
#if defined(__clang__)
  return __builtin_addc(a, b, cin, cout);
#else
  const uint64_t s = (uint64_t)a + b + cin;
  *cout = (uint32_t)(s >> 32);
  return (uint32_t)s;
#endif
}
OVH_HD uint32_t subc32(uint32_t a, uint32_t b, uint32_t bin, uint32_t* bout) {
#if defined(__clang__)
  return __builtin_subc(a, b, bin, bout);
#else
  const uint64_t d = (uint64_t)a - b - bin;
  *bout = (uint32_t)(d >> 63);
  return (uint32_t)d;
#endif
}

struct Fp {
  uint32_t v[12];
};

OVH_HD void fp_load(Fp& r, const uint32_t* c) {
#pragma unroll
  for (int i = 0; i < 12; ++i) r.v[i] = c[i];
}

OVH_HD Fp fp_const(const uint32_t* c) {
  Fp r;
  fp_load(r, c);
  return r;
}

OVH_HD void fp_zero(Fp& r) {
#pragma unroll
  for (int i = 0; i < 12; ++i) r.v[i] = 0;
}

OVH_HD void fp_one(Fp& r) { fp_load(r, ONE_M); }

OVH_HD bool fp_is_zero(const Fp& a) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) acc |= a.v[i];
  return acc == 0;
}

OVH_HD bool fp_eq(const Fp& a, const Fp& b) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) acc |= a.v[i] ^ b.v[i];
  return acc == 0;
}

OVH_HD bool fp_is_one(const Fp& a) { return fp_eq(a, fp_const(ONE_M)); }

// r = cond ? b : a   (cond uniform or per-lane; compiles to v_cndmask)
OVH_HD void fp_select(Fp& r, bool cond, const Fp& a, const Fp& b) {
#pragma unroll
  for (int i = 0; i < 12; ++i) r.v[i] = cond ? b.v[i] : a.v[i];
}

// r = a + b mod p
OVH_HD void fp_add(Fp& r, const Fp& a, const Fp& b) {
  uint32_t s[12], d[12], c = 0, br = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) s[i] = addc32(a.v[i], b.v[i], c, &c);
#pragma unroll
  for (int i = 0; i < 12; ++i) d[i] = subc32(s[i], P_LIMBS[i], br, &br);
#pragma unroll
  for (int i = 0; i < 12; ++i) r.v[i] = br ? s[i] : d[i];  // s < p -> keep s
}

// r = a - b mod p
OVH_HD void fp_sub(Fp& r, const Fp& a, const Fp& b) {
  uint32_t d[12], br = 0, c = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) d[i] = subc32(a.v[i], b.v[i], br, &br);
  const uint32_t mask = 0u - br;
#pragma unroll
  for (int i = 0; i < 12; ++i) r.v[i] = addc32(d[i], P_LIMBS[i] & mask, c, &c);
}

OVH_HD void fp_dbl(Fp& r, const Fp& a) { fp_add(r, a, a); }

OVH_HD void fp_neg(Fp& r, const Fp& a) {
  Fp z;
  fp_zero(z);
  fp_sub(r, z, a);
}

// Montgomery product r = a * b * 2^-384 mod p. Device: fp_mul28_gfx950 (14 x 28-bit limbs, one
// 64-bit accumulator per column, no carry word). Host: CIOS on 12 x 32-bit limbs (p[11] < 2^31).
OVH_HD void fp_mul(Fp& r, const Fp& a, const Fp& b) {
#if defined(__HIP_DEVICE_COMPILE__) && defined(OVH_FPMUL32)
  fp_mul_gfx950(r.v, a.v, b.v);  // A/B builds: the 12 x 32-bit product scanning form
#elif defined(__HIP_DEVICE_COMPILE__)
  // 14 x 28-bit limbs, one 64-bit accumulator (r03c: vote kernel 3.76 -> 3.56 ms, 1,060k ->
  // 1,115k verifs/s; tools/ubench/fp_mul28.hip 1.10-1.14x per product)
  fp_mul28_gfx950(r.v, a.v, b.v);
#else
  OVH_COUNT_MUL();
  uint32_t t[12];
#pragma unroll
  for (int j = 0; j < 12; ++j) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const uint32_t bi = b.v[i];
    uint64_t c = (uint64_t)a.v[0] * bi + t[0];
    t[0] = (uint32_t)c;
    const uint32_t m = t[0] * P_INV32;
    uint64_t c2 = (uint64_t)m * P_LIMBS[0] + t[0];
#pragma unroll
    for (int j = 1; j < 12; ++j) {
      c = (uint64_t)a.v[j] * bi + t[j] + (c >> 32);
      c2 = (uint64_t)m * P_LIMBS[j] + (uint32_t)c + (c2 >> 32);
      t[j - 1] = (uint32_t)c2;
    }
    t[11] = (uint32_t)(c >> 32) + (uint32_t)(c2 >> 32);
  }
  // conditional subtraction: t < 2p
  uint32_t d[12], br = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) d[i] = subc32(t[i], P_LIMBS[i], br, &br);
#pragma unroll
  for (int i = 0; i < 12; ++i) r.v[i] = br ? t[i] : d[i];
#endif
}

OVH_HD void fp_sqr(Fp& r, const Fp& a) { fp_mul(r, a, a); }

// r = a * small (small < 2^16), via repeated doubling-free Montgomery-free path:
OVH_HD void fp_mul_small(Fp& r, const Fp& a, uint32_t k) {
  Fp acc, base = a;
  fp_zero(acc);
  while (k) {
    if (k & 1) fp_add(acc, acc, base);
    fp_add(base, base, base);
    k >>= 1;
  }
  r = acc;
}

// r = a^e for a plain (non-Montgomery) 384-bit exponent given as 12 LE limbs.
OVH_HDNI void fp_pow(Fp& r, const Fp& a, const uint32_t* e) {
  Fp acc;
  fp_one(acc);
  bool started = false;
#pragma unroll 1
  for (int i = 11; i >= 0; --i) {
    const uint32_t w = e[i];
#pragma unroll 1
    for (int b = 31; b >= 0; --b) {
      if (started) fp_sqr(acc, acc);
      if ((w >> b) & 1) {
        if (started) {
          fp_mul(acc, acc, a);
        } else {
          acc = a;
          started = true;
        }
      }
    }
  }
  r = acc;
}

// Modular inverse of a canonical Montgomery value, then back to Montgomery form with one product
// by raw R^3 (r3). 0 -> 0. Used by fp_inv (every one-lane kernel) and the Fp-VM's inv op.
// Bernstein-Yang divsteps, variable time (the inverted value is public batch data): batches of
// 30 divsteps on the low limbs give a 2x2 transition matrix, applied to (f, g) exactly and to
// (d, e) modulo p (plus the multiple of p that makes the division by 2^30 exact). Values in 13
// signed 30-bit limbs (limbs 0..11 in [0, 2^30), limb 12 signed). Invariants: f = d x, g = e x
// (mod p); f starts at p, g at x; when g reaches 0, f = +-1 and x^-1 = +-d.
namespace inv {
constexpr int NL = 13;
constexpr int32_t M30 = 0x3FFFFFFF;
constexpr int32_t PL[NL] = {0x3fffaaab, 0x27fbffff, 0x153ffffb, 0x2affffac, 0x30f6241e, 0x034a83da, 0x112bf673,
                            0x12e13ce1, 0x2cd76477, 0x1ed90d2e, 0x29a4b1ba, 0x3a8e5ff9, 0x001a0111};
constexpr uint32_t PINV30 = 0x30003;  // p^-1 mod 2^30
struct Trans {
  int32_t u, v, q, r;
};

OVH_HD int ctz32(uint32_t x) { return __builtin_ctz(x); }

// -(f^-1) mod 2^32, f odd (Newton: 3 -> 6 -> 12 -> 24 -> 48 correct bits)
OVH_HD uint32_t neg_inv32(uint32_t f) {
  uint32_t x = f;
  x *= 2u - f * x;
  x *= 2u - f * x;
  x *= 2u - f * x;
  x *= 2u - f * x;
  return 0u - x;
}

// 30 divsteps on the low bits of f and g (eta = -delta); t: 2^30 [f', g'] = t [f, g]
OVH_HD int32_t divsteps30(int32_t eta, uint32_t f, uint32_t g, Trans& t) {
  uint32_t u = 1, v = 0, q = 0, r = 1, finv = neg_inv32(f);
  int i = 30;
#pragma unroll 1
  for (;;) {
    // zero low bits of g: halvings (the f row doubles instead), at most i of them
    const int z = ctz32(g | (0xFFFFFFFFu << i));
    g >>= z;
    u <<= z;
    v <<= z;
    eta -= z;
    i -= z;
    if (i == 0) break;
    if (eta < 0) {  // swap: (f, g) = (g, -f)
      eta = -eta;
      uint32_t x = f;
      f = g;
      g = 0u - x;
      x = u;
      u = q;
      q = 0u - x;
      x = v;
      v = r;
      r = 0u - x;
      finv = neg_inv32(f);
    }
    // cancel up to min(eta + 1, i) low bits of g with a multiple of f
    const int limit = (eta + 1) > i ? i : (eta + 1);
    const uint32_t w = (g * finv) & (0xFFFFFFFFu >> (32 - limit));
    g += f * w;
    q += u * w;
    r += v * w;
  }
  t.u = (int32_t)u;
  t.v = (int32_t)v;
  t.q = (int32_t)q;
  t.r = (int32_t)r;
  return eta;
}

// (f, g) = t (f, g) / 2^30 (exact)
OVH_HD void update_fg(int32_t* f, int32_t* g, const Trans& t) {
  const int64_t u = t.u, v = t.v, q = t.q, r = t.r;
  int64_t cf = u * f[0] + v * g[0], cg = q * f[0] + r * g[0];
  cf >>= 30;
  cg >>= 30;
#pragma unroll
  for (int i = 1; i < NL; ++i) {
    cf += u * f[i] + v * g[i];
    cg += q * f[i] + r * g[i];
    f[i - 1] = (int32_t)cf & M30;
    cf >>= 30;
    g[i - 1] = (int32_t)cg & M30;
    cg >>= 30;
  }
  f[NL - 1] = (int32_t)cf;
  g[NL - 1] = (int32_t)cg;
}

// (d, e) = (t (d, e) + p (md, me)) / 2^30, md / me making the division exact and keeping
// d, e in (-2p, p)
OVH_HD void update_de(int32_t* d, int32_t* e, const Trans& t) {
  const int32_t sd = d[NL - 1] >> 31, se = e[NL - 1] >> 31;
  int32_t md = (t.u & sd) + (t.v & se), me = (t.q & sd) + (t.r & se);
  const int64_t u = t.u, v = t.v, q = t.q, r = t.r;
  int64_t cd = u * d[0] + v * e[0], ce = q * d[0] + r * e[0];
  md -= (int32_t)((PINV30 * (uint32_t)cd + (uint32_t)md) & (uint32_t)M30);
  me -= (int32_t)((PINV30 * (uint32_t)ce + (uint32_t)me) & (uint32_t)M30);
  cd += (int64_t)PL[0] * md;
  ce += (int64_t)PL[0] * me;
  cd >>= 30;
  ce >>= 30;
#pragma unroll
  for (int i = 1; i < NL; ++i) {
    cd += u * d[i] + v * e[i] + (int64_t)PL[i] * md;
    ce += q * d[i] + r * e[i] + (int64_t)PL[i] * me;
    d[i - 1] = (int32_t)cd & M30;
    cd >>= 30;
    e[i - 1] = (int32_t)ce & M30;
    ce >>= 30;
  }
  d[NL - 1] = (int32_t)cd;
  e[NL - 1] = (int32_t)ce;
}

// d in (-2p, p) -> (neg ? -d : d) in [0, p)
OVH_HD void normalize(int32_t* d, bool neg) {
  int32_t c = d[NL - 1] >> 31;
#pragma unroll
  for (int i = 0; i < NL; ++i) d[i] += PL[i] & c;
  const int32_t n = neg ? -1 : 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) d[i] = (d[i] ^ n) - n;
#pragma unroll
  for (int i = 0; i < NL - 1; ++i) {
    d[i + 1] += d[i] >> 30;
    d[i] &= M30;
  }
  c = d[NL - 1] >> 31;
#pragma unroll
  for (int i = 0; i < NL; ++i) d[i] += PL[i] & c;
#pragma unroll
  for (int i = 0; i < NL - 1; ++i) {
    d[i + 1] += d[i] >> 30;
    d[i] &= M30;
  }
}
}  // namespace inv

OVH_HD void fp_inv_divsteps(Fp& r, const Fp& a, const Fp& r3) {
  using namespace inv;
  int32_t f[NL], g[NL], d[NL], e[NL];
  uint32_t any = 0;
#pragma unroll
  for (int k = 0; k < NL; ++k) {  // 12 x 32 -> 13 x 30 bits
    const int b = 30 * k, w = b >> 5, sh = b & 31;
    uint32_t x = a.v[w] >> sh;
    if (sh > 2 && w + 1 < 12) x |= a.v[w + 1] << (32 - sh);
    g[k] = (int32_t)(x & (uint32_t)M30);
    f[k] = PL[k];
    d[k] = 0;
    e[k] = 0;
    any |= a.v[k < 12 ? k : 11];
  }
  e[0] = 1;
  if (!any) {
    fp_zero(r);
    return;
  }
  int32_t eta = -1;
#pragma unroll 1
  for (int it = 0; it < 80; ++it) {  // converges in well under 1102 / 30 batches
    Trans t;
    eta = divsteps30(eta, (uint32_t)f[0], (uint32_t)g[0], t);
    update_de(d, e, t);
    update_fg(f, g, t);
    if (g[0] == 0) {
      int32_t z = 0;
#pragma unroll
      for (int i = 1; i < NL; ++i) z |= g[i];
      if (z == 0) break;
    }
  }
  normalize(d, f[NL - 1] < 0);
  Fp x;
#pragma unroll
  for (int w = 0; w < 12; ++w) {  // 13 x 30 -> 12 x 32 bits
    const int b = 32 * w, k = b / 30, sh = b % 30;
    uint32_t y = (uint32_t)d[k] >> sh;
    if (k + 1 < NL) y |= (uint32_t)d[k + 1] << (30 - sh);
    if (sh > 28 && k + 2 < NL) y |= (uint32_t)d[k + 2] << (60 - sh);
    x.v[w] = y;
  }
  fp_mul(r, x, r3);
}

// a^-1 (0 -> 0) by divsteps: ~37 batches of 30 steps on 13 x 30-bit limbs instead of the ~450
// dependent products of a^(p-2) (k_g2p_compress and every other one-lane inversion)
OVH_HD void fp_inv(Fp& r, const Fp& a) {
  Fp c, r3;
  uint32_t d[12], br = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) d[i] = subc32(a.v[i], P_LIMBS[i], br, &br);
#pragma unroll
  for (int i = 0; i < 12; ++i) c.v[i] = br ? a.v[i] : d[i];
#pragma unroll
  for (int i = 0; i < 12; ++i) r3.v[i] = R3_M[i];
  fp_inv_divsteps(r, c, r3);
}

// Square root candidate a^((p+1)/4); returns true iff it squares back to a.
OVH_HD bool fp_sqrt(Fp& r, const Fp& a) {
  Fp s, s2;
  fp_pow(s, a, EXP_SQRT);
  fp_sqr(s2, s);
  r = s;
  return fp_eq(s2, a);
}

// Conversion between plain and Montgomery form.
OVH_HD void fp_to_mont(Fp& r, const Fp& a) { fp_mul(r, a, fp_const(R2_M)); }
OVH_HD void fp_from_mont(Fp& r, const Fp& a) {
  Fp one;
  fp_zero(one);
  one.v[0] = 1;
  fp_mul(r, a, one);
}

// plain-integer compare a > b (both plain limbs)
OVH_HD bool limbs_gt(const uint32_t* a, const uint32_t* b) {
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) (void)subc32(b[i], a[i], br, &br);
  return br != 0;
}

// plain a < p ?
OVH_HD bool limbs_lt_p(const uint32_t* a) {
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) (void)subc32(a[i], P_LIMBS[i], br, &br);
  return br != 0;
}

// Lexicographic "sign" of a Montgomery-form element: value > (p-1)/2.
OVH_HD bool fp_lex_largest(const Fp& a) {
  Fp plain;
  fp_from_mont(plain, a);
  return limbs_gt(plain.v, HALF_P);
}

// RFC 9380 sgn0 (parity of the canonical value).
OVH_HD uint32_t fp_sgn0(const Fp& a) {
  Fp plain;
  fp_from_mont(plain, a);
  return plain.v[0] & 1u;
}

// 48 big-endian bytes -> plain limbs (no reduction).
OVH_HD void limbs_from_be48(uint32_t* out, const uint8_t* in) {
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const uint8_t* p = in + 44 - 4 * i;
    out[i] = ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
  }
}

OVH_HD void limbs_to_be48(uint8_t* out, const uint32_t* in) {
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    uint8_t* p = out + 44 - 4 * i;
    p[0] = (uint8_t)(in[i] >> 24);
    p[1] = (uint8_t)(in[i] >> 16);
    p[2] = (uint8_t)(in[i] >> 8);
    p[3] = (uint8_t)in[i];
  }
}

// Montgomery element -> 48 BE bytes of its canonical value.
OVH_HD void fp_to_be48(uint8_t* out, const Fp& a) {
  Fp plain;
  fp_from_mont(plain, a);
  limbs_to_be48(out, plain.v);
}

}  // namespace ovh
