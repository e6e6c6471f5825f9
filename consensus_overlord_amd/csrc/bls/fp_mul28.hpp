// Montgomery product a b 2^-384 mod p on 14 x 28-bit limbs, gfx950 device code. Interface of
// fp_mul_gfx950: 12 x 32-bit limbs in / out, a, b < 4p, r < 1.63p after one conditional
// subtraction. A column of 14 + 14 products of 28-bit limbs plus the carry stays below 2^61, so
// every partial product is one v_mad_u64_u32 into a 64-bit accumulator, with no carry word
// (the 12 x 32 product scanning pays one v_addc per v_mad). R = 2^392; a enters shifted left by
// 8 bits, so the result is a b 2^-384 (the Montgomery form everywhere else is unchanged).
// tools/ubench/fp_mul28.hip times it against fp_mul_gfx950 and checks them against each other.
#pragma once
#include <stdint.h>

#include "consts.hpp"

namespace ovh {

constexpr uint32_t M28 = 0x0FFFFFFFu;
constexpr uint32_t P28[14] = {0xfffaaabu, 0xfefffffu, 0x3ffffb9u, 0xfffeb15u, 0x6241eabu, 0xa0f6b0fu, 0xf6730d2u,
                              0xf38512bu, 0x4774b84u, 0x4bacd76u, 0xba7b643u, 0xe69a4b1u, 0x1ea397fu, 0x001a011u};
constexpr uint32_t PINV28 = 0xffcfffdu;  // -p^-1 mod 2^28

// x = (a << sh) as 14 limbs of 28 bits (a < 2^384 - sh)
template <int SH>
__device__ __forceinline__ void split28(uint32_t* x, const uint32_t* a) {
#if defined(OVH_UBENCH_NOSPLIT)  // microbenchmark only (tools/ubench/vm_phase.hip): wrong values
#pragma unroll
  for (int k = 0; k < 14; ++k) x[k] = a[k % 12];
  return;
#endif
#pragma unroll
  for (int k = 0; k < 14; ++k) {
    const int lo = 28 * k - SH;
    uint32_t v;
    if (lo < 0) {
      v = a[0] << (-lo);
    } else {
      const int w = lo >> 5, s = lo & 31;
      v = a[w] >> s;
      if (s > 4 && w + 1 < 12) v |= a[w + 1] << (32 - s);
    }
    x[k] = v & M28;
  }
}

// 14 x 28 -> 12 x 32, then one conditional subtraction (the value is < 2.63 p)
__device__ __forceinline__ void join28_reduce(uint32_t* r, const uint32_t* t) {
#if defined(OVH_UBENCH_NOSPLIT)
#pragma unroll
  for (int j = 0; j < 12; ++j) r[j] = t[j];
  return;
#endif
  uint32_t u[12];
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    const int k = (32 * j) / 28, s = (32 * j) % 28;
    uint32_t v = (t[k] >> s) | (t[k + 1] << (28 - s));
    if (s > 24 && k + 2 < 14) v |= t[k + 2] << (56 - s);
    u[j] = v;
  }
  uint32_t d[12], br = 0;
#pragma unroll
  for (int j = 0; j < 12; ++j) d[j] = __builtin_subc(u[j], P_LIMBS[j], br, &br);  // v_sub(b)_co chain
#pragma unroll
  for (int j = 0; j < 12; ++j) r[j] = br ? u[j] : d[j];
}

__device__ __forceinline__ void fp_mul28(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  uint32_t x[14], y[14], m[14], t[14];
  split28<8>(x, a);  // a 2^8: with R = 2^392 the product is a b 2^-384
  split28<0>(y, b);
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 27; ++k) {
#pragma unroll
    for (int i = 0; i < 14; ++i)
      if (k - i >= 0 && k - i < 14) acc += (uint64_t)x[i] * y[k - i];
#pragma unroll
    for (int i = 0; i < 14; ++i)
      if (i < k && k - i < 14) acc += (uint64_t)m[i] * P28[k - i];
    if (k < 14) {
      m[k] = ((uint32_t)acc * PINV28) & M28;
      acc += (uint64_t)m[k] * P28[0];
    } else {
      t[k - 14] = (uint32_t)acc & M28;
    }
    acc >>= 28;
  }
  t[13] = (uint32_t)acc;
  join28_reduce(r, t);
}

}  // namespace ovh
