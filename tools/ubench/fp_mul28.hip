// Montgomery product on 14 x 28-bit limbs (product scanning, 64-bit accumulators, no carry
// word; one-chain and two-accumulator issue orders, tools/gen_fpmul28.py) against the production 12 x 32-bit product (csrc/bls/fp_mul_gfx950.hpp): same interface
// (12 x 32-bit limbs in and out, a, b < 4p, result < 1.63p), bit-checked against each other mod p
// and timed as dependent product chains at 1 and 4 waves per SIMD.
//   hipcc -O3 --offload-arch=gfx950 -o tools/ubench/fp_mul28 tools/ubench/fp_mul28.hip
// Why 28 bits: a column of 14 + 14 products of 28-bit limbs plus the carry stays below 2^61, so
// every partial product is one v_mad_u64_u32 into the accumulator with no v_addc for a third
// word (the 12 x 32 form pays one v_addc per v_mad). R = 2^392; the operand a enters shifted left
// by 8 bits, so the product is a b 2^-384 as before (the VM's Montgomery form is unchanged).
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../../consensus_overlord_amd/csrc/bls/fp.hpp"
#include "../../consensus_overlord_amd/csrc/bls/fp_mul28.hpp"
#include "../../consensus_overlord_amd/csrc/bls/fp_mul28_gfx950.hpp"

namespace ovh {
__device__ __forceinline__ void vm_canon(Fp& r, const Fp& a) {
  uint32_t d[12], br = 0;
#pragma unroll
  for (int j = 0; j < 12; ++j) d[j] = subc32(a.v[j], P_LIMBS[j], br, &br);
#pragma unroll
  for (int j = 0; j < 12; ++j) r.v[j] = br ? a.v[j] : d[j];
}

}  // namespace ovh

using namespace ovh;

template <int V>
__global__ __launch_bounds__(64) void k_chain(uint32_t iters, uint32_t* out) {
  Fp x, y;
  for (int k = 0; k < 12; ++k) {
    x.v[k] = (k < 11) ? 0x9abcdefu * (threadIdx.x + k + 1 + blockIdx.x) : 0x0100000u;
    y.v[k] = (k < 11) ? 0x1234567u * (threadIdx.x + k + 7) : 0x0200000u;
  }
  for (uint32_t i = 0; i < iters; ++i) {
    if (V == 0) fp_mul(x, x, y);
    else if (V == 1) fp_mul28_gfx950_1acc(x.v, x.v, y.v);
    else fp_mul28_gfx950_2acc(x.v, x.v, y.v);
  }
  Fp c;
  vm_canon(c, x);
  for (int k = 0; k < 12; ++k) out[(blockIdx.x * 64 + threadIdx.x) * 12 + k] = c.v[k];
}

int main() {
  uint32_t *d0, *d1;
  const int maxg = 4096;
  if (hipMalloc(&d0, maxg * 64 * 48) != hipSuccess || hipMalloc(&d1, maxg * 64 * 48) != hipSuccess) return 1;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const uint32_t iters = 2048;
  static uint32_t h0[4096 * 64 * 12], h1[4096 * 64 * 12];
  for (int grid : {1024, 4096}) {
    float t[3];
    size_t bad[3] = {0, 0, 0};
    for (int v = 0; v < 3; ++v) {
      auto k = v == 0 ? k_chain<0> : v == 1 ? k_chain<1> : k_chain<2>;
      uint32_t* d = v == 0 ? d0 : d1;
      hipLaunchKernelGGL(k, dim3(grid), dim3(64), 0, 0, iters, d);
      (void)hipDeviceSynchronize();
      (void)hipEventRecord(a);
      hipLaunchKernelGGL(k, dim3(grid), dim3(64), 0, 0, iters, d);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      (void)hipEventElapsedTime(&t[v], a, b);
      (void)hipMemcpy(v == 0 ? h0 : h1, d, grid * 64 * 48, hipMemcpyDeviceToHost);
      if (v)
        for (size_t i = 0; i < (size_t)grid * 64 * 12; ++i) bad[v] += h0[i] != h1[i];
    }
    printf("{\"waves\": %d, \"ns_per_mul_32x12\": %.1f, \"ns_per_mul_28x14_1acc\": %.1f, \"ns_per_mul_28x14_2acc\": "
           "%.1f, \"speedup_1acc\": %.3f, \"speedup_2acc\": %.3f, \"mismatched_words\": [%zu, %zu]}\n",
           grid, t[0] * 1e6 / iters, t[1] * 1e6 / iters, t[2] * 1e6 / iters, t[0] / t[1], t[0] / t[2], bad[1], bad[2]);
  }
  return 0;
}
