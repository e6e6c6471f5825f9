// fp_mul_gfx950 (one accumulator chain) vs fp_mul2_gfx950 (two interleaved chains): dependent
// product chains at 1 and 4 waves per SIMD, and a bit-exact comparison of the two on the same
// chain. hipcc -O3 --offload-arch=gfx950 -o tools/ubench/fpmul_variants tools/ubench/fpmul_variants.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../../consensus_overlord_amd/csrc/bls/fp.hpp"
#include "fp_mul2_gfx950.hpp"

using namespace ovh;

template <int V>
__global__ __launch_bounds__(64) void k_chain(uint32_t iters, uint32_t* out) {
  Fp x, y;
  for (int k = 0; k < 12; ++k) {
    x.v[k] = (k < 11) ? 0x9abcdefu * (threadIdx.x + k + 1 + blockIdx.x) : 0;
    y.v[k] = (k < 11) ? 0x1234567u * (threadIdx.x + k + 7) : 0;
  }
  for (uint32_t i = 0; i < iters; ++i) {
    if (V == 0) fp_mul(x, x, y);
    else fp_mul2_gfx950(x.v, x.v, y.v);
  }
  for (int k = 0; k < 12; ++k) out[(blockIdx.x * 64 + threadIdx.x) * 12 + k] = x.v[k];
}

int main() {
  uint32_t *d0, *d1;
  const int maxg = 4096;
  if (hipMalloc(&d0, maxg * 64 * 48) != hipSuccess || hipMalloc(&d1, maxg * 64 * 48) != hipSuccess) return 1;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const uint32_t iters = 2048;
  for (int grid : {1024, 4096}) {
    for (int v = 0; v < 2; ++v) {
      auto k = v == 0 ? k_chain<0> : k_chain<1>;
      hipLaunchKernelGGL(k, dim3(grid), dim3(64), 0, 0, iters, v == 0 ? d0 : d1);
      (void)hipDeviceSynchronize();
      (void)hipEventRecord(a);
      hipLaunchKernelGGL(k, dim3(grid), dim3(64), 0, 0, iters, v == 0 ? d0 : d1);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      printf("{\"variant\": %d, \"waves\": %d, \"ns_per_mul\": %.1f}\n", v, grid, ms * 1e6 / iters);
    }
    static uint32_t h0[4096 * 64 * 12], h1[4096 * 64 * 12];
    (void)hipMemcpy(h0, d0, grid * 64 * 48, hipMemcpyDeviceToHost);
    (void)hipMemcpy(h1, d1, grid * 64 * 48, hipMemcpyDeviceToHost);
    size_t bad = 0;
    for (size_t i = 0; i < (size_t)grid * 64 * 12; ++i) bad += h0[i] != h1[i];
    printf("{\"waves\": %d, \"mismatched_words\": %zu}\n", grid, bad);
  }
  return 0;
}
