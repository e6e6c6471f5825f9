// Integer-VALU issue-rate microbenchmark for gfx950 (roofline denominator for
// the BLS12-381 Montgomery arithmetic). Each lane runs 8 independent chains of
// one instruction so the measurement is issue-bound, not latency-bound.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 4096

__global__ void k_mad_u64_u32(uint64_t* out, uint32_t a, uint32_t b) {
  uint64_t acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = threadIdx.x + i;
  uint32_t x = a + threadIdx.x, y = b ^ threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      uint64_t cc;
      asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[i]), "=s"(cc) : "v"(x), "v"(y));
    }
  }
  uint64_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mul_lo_u32(uint64_t* out, uint32_t a, uint32_t b) {
  uint32_t acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = threadIdx.x + i;
  uint32_t y = b ^ threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(acc[i]) : "v"(y));
  }
  uint64_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mul_hi_u32(uint64_t* out, uint32_t a, uint32_t b) {
  uint32_t acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = threadIdx.x + i;
  uint32_t y = b ^ threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(acc[i]) : "v"(y));
  }
  uint64_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mad_u32_u24(uint64_t* out, uint32_t a, uint32_t b) {
  uint32_t acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = threadIdx.x + i;
  uint32_t x = a + threadIdx.x, y = b ^ threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(acc[i]) : "v"(x), "v"(y));
  }
  uint64_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mul_hi_u32_u24(uint64_t* out, uint32_t a, uint32_t b) {
  uint32_t acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = threadIdx.x + i;
  uint32_t y = b ^ threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(acc[i]) : "v"(y));
  }
  uint64_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_add_co_u32(uint64_t* out, uint32_t a, uint32_t b) {
  uint32_t acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = threadIdx.x + i;
  uint32_t y = b ^ threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      uint64_t cc;
      asm volatile("v_add_co_u32 %0, %1, %0, %2" : "+v"(acc[i]), "=s"(cc) : "v"(y));
    }
  }
  uint64_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_addc_co_u32(uint64_t* out, uint32_t a, uint32_t b) {
  uint32_t acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = threadIdx.x + i;
  uint32_t y = b ^ threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(acc[i]) : "v"(y) : "vcc");
    }
  }
  uint64_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_lshl_add_u64(uint64_t* out, uint32_t a, uint32_t b) {
  uint64_t acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = threadIdx.x + i;
  uint64_t y = ((uint64_t)a << 32) | (b ^ threadIdx.x);
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[i]) : "v"(y));
  }
  uint64_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef void (*kfn)(uint64_t*, uint32_t, uint32_t);

static void run(const char* name, kfn k, int insts_per_inner, uint64_t* d) {
  int blocks = 256 * 8, threads = 256;  // 8 waves/SIMD worth of work
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, 0x12345u, 0x9876543u);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  const int reps = 5;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, 0x12345u, 0x9876543u);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double lane_ops = (double)reps * blocks * threads * ITERS * 8.0 * insts_per_inner;
  double rate = lane_ops / (ms * 1e-3);
  // full-rate VALU: 256 CU * 4 SIMD * 32 lanes/clk * 2.4e9
  double full = 256.0 * 4 * 32 * 2.4e9;
  printf("{\"inst\": \"%s\", \"lane_ops_per_s\": %.4e, \"frac_of_fullrate_2p4GHz\": %.4f, \"ms\": %.3f}\n", name, rate, rate / full, ms / reps);
}

int main() {
  uint64_t* d;
  hipMalloc(&d, 256 * 8 * 256 * sizeof(uint64_t));
  run("v_mad_u64_u32", k_mad_u64_u32, 1, d);
  run("v_mul_lo_u32", k_mul_lo_u32, 1, d);
  run("v_mul_hi_u32", k_mul_hi_u32, 1, d);
  run("v_mad_u32_u24", k_mad_u32_u24, 1, d);
  run("v_mul_hi_u32_u24", k_mul_hi_u32_u24, 1, d);
  run("v_add_co_u32", k_add_co_u32, 1, d);
  run("v_add_co+v_addc_co pair", k_addc_co_u32, 2, d);
  run("v_lshl_add_u64", k_lshl_add_u64, 1, d);
  hipFree(d);
  return 0;
}
