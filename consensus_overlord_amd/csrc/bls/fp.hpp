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

// Montgomery product r = a * b * 2^-384 mod p (CIOS, no extra carry word: p[11] < 2^31).
OVH_HD void fp_mul(Fp& r, const Fp& a, const Fp& b) {
#if defined(__HIP_DEVICE_COMPILE__)
  fp_mul_gfx950(r.v, a.v, b.v);
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

OVH_HD void fp_inv(Fp& r, const Fp& a) { fp_pow(r, a, EXP_P_MINUS_2); }

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
