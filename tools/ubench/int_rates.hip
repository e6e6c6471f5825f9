// Integer-VALU issue-rate microbenchmark for gfx950: the roofline denominators of the
// BLS12-381 Montgomery arithmetic (bench.py `roofline`).
//
// For each instruction and 1 / 2 / 4 / 8 waves per SIMD (1,024 x w single-wave workgroups on
// 256 CUs x 4 SIMDs, every one resident at once): each lane runs 8 independent chains of the
// instruction, so the loop is issue-bound, not latency-bound. Every launch lasts ~20 ms; 40
// launches run back to back (~0.8 s, the clock settles under load: MI355X_MICROARCH.md DVFS
// give-back) and then 10 timed launches (HIP events). Diagnostic stamps: lane 0 of every wave of
// the last timed launch records s_memtime (shader cycles) and s_memrealtime (100 MHz) around
// its loop, into a buffer of their own that nothing else reads; the held clock is the median
// over waves of delta(memtime) / delta(memrealtime) x 100 MHz.
//
// Output, one JSON object per (instruction, waves per SIMD):
//   lane_ops_per_s            measured rate (lane operations per second, whole chip)
//   clock_ghz                 held shader clock during the last launch (median over waves)
//   cycles_per_inst_per_simd  = 1,024 SIMDs x clock / (rate / 64): the issue cost of one wave
//                             instruction on one SIMD (4 = full rate, 16 lanes per clock)
//   frac_fullrate_2p4         rate / 3.93e13 (256 CU x 64 lanes/clk x 2.4 GHz)
//   frac_fullrate_held        rate / (256 x 64 x held clock)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define NCHAIN 8

// One asm statement per loop iteration: 4 rounds over the 8 independent chains (32 instructions),
// so the compiler inserts no hazard NOPs between them and the loop's SALU overhead is 3 per 32.
// The carry-outs of v_mad_u64_u32 / v_add_co_u32 go to vcc, as in the production Montgomery
// product (csrc/bls/fp_mul28_gfx950.hpp). (r04b measured the compiler's per-instruction form,
// `"=s"` carry-outs with an s_nop 0 between consecutive mads: 11 cycles per instruction at one
// wave per SIMD -- the hazard padding, not the VALU.)
#define R4(S) S S S S
#define MAD8                                                                                         \
  "v_mad_u64_u32 %[a0], vcc, %[x], %[y], %[a0]\n\tv_mad_u64_u32 %[a1], vcc, %[x], %[y], %[a1]\n\t"   \
  "v_mad_u64_u32 %[a2], vcc, %[x], %[y], %[a2]\n\tv_mad_u64_u32 %[a3], vcc, %[x], %[y], %[a3]\n\t"   \
  "v_mad_u64_u32 %[a4], vcc, %[x], %[y], %[a4]\n\tv_mad_u64_u32 %[a5], vcc, %[x], %[y], %[a5]\n\t"   \
  "v_mad_u64_u32 %[a6], vcc, %[x], %[y], %[a6]\n\tv_mad_u64_u32 %[a7], vcc, %[x], %[y], %[a7]\n\t"
#define ADD8                                                                                         \
  "v_add_co_u32 %[a0], vcc, %[a0], %[y]\n\tv_add_co_u32 %[a1], vcc, %[a1], %[y]\n\t"                 \
  "v_add_co_u32 %[a2], vcc, %[a2], %[y]\n\tv_add_co_u32 %[a3], vcc, %[a3], %[y]\n\t"                 \
  "v_add_co_u32 %[a4], vcc, %[a4], %[y]\n\tv_add_co_u32 %[a5], vcc, %[a5], %[y]\n\t"                 \
  "v_add_co_u32 %[a6], vcc, %[a6], %[y]\n\tv_add_co_u32 %[a7], vcc, %[a7], %[y]\n\t"
#define MUL8                                                                                         \
  "v_mul_lo_u32 %[a0], %[a0], %[y]\n\tv_mul_lo_u32 %[a1], %[a1], %[y]\n\t"                           \
  "v_mul_lo_u32 %[a2], %[a2], %[y]\n\tv_mul_lo_u32 %[a3], %[a3], %[y]\n\t"                           \
  "v_mul_lo_u32 %[a4], %[a4], %[y]\n\tv_mul_lo_u32 %[a5], %[a5], %[y]\n\t"                           \
  "v_mul_lo_u32 %[a6], %[a6], %[y]\n\tv_mul_lo_u32 %[a7], %[a7], %[y]\n\t"
#define ACC8 [a0] "+v"(acc[0]), [a1] "+v"(acc[1]), [a2] "+v"(acc[2]), [a3] "+v"(acc[3]), [a4] "+v"(acc[4]), \
             [a5] "+v"(acc[5]), [a6] "+v"(acc[6]), [a7] "+v"(acc[7])

struct Stamp {  // lane 0's s_memtime / s_memrealtime around the loop (diagnostic buffer only)
  uint64_t t0 = 0, r0 = 0;
  __device__ void begin(const uint64_t* st) {
    if (st && threadIdx.x == 0) {
      t0 = __builtin_amdgcn_s_memtime();
      r0 = __builtin_amdgcn_s_memrealtime();
    }
  }
  __device__ void end(uint64_t* st) {
    if (st && threadIdx.x == 0) {
      const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
      st[2 * blockIdx.x] = t1 - t0;
      st[2 * blockIdx.x + 1] = r1 - r0;
    }
  }
};

__global__ __launch_bounds__(64) void k_mad_u64_u32(uint64_t* out, uint64_t* stamps, uint32_t iters, uint32_t a,
                                                    uint32_t b) {
  uint64_t acc[NCHAIN];
  const uint32_t x = a + threadIdx.x, y = b ^ threadIdx.x;
  for (int i = 0; i < NCHAIN; ++i) acc[i] = threadIdx.x + i;
  Stamp sp;
  sp.begin(stamps);
  for (uint32_t it = 0; it < iters; ++it) asm volatile(R4(MAD8) : ACC8 : [x] "v"(x), [y] "v"(y) : "vcc");
  sp.end(stamps);
  uint64_t s = 0;
  for (int i = 0; i < NCHAIN; ++i) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(64) void k_add_co_u32(uint64_t* out, uint64_t* stamps, uint32_t iters, uint32_t a,
                                                   uint32_t b) {
  uint32_t acc[NCHAIN];
  const uint32_t y = b ^ threadIdx.x;
  for (int i = 0; i < NCHAIN; ++i) acc[i] = threadIdx.x + i + a;
  Stamp sp;
  sp.begin(stamps);
  for (uint32_t it = 0; it < iters; ++it) asm volatile(R4(ADD8) : ACC8 : [y] "v"(y) : "vcc");
  sp.end(stamps);
  uint64_t s = 0;
  for (int i = 0; i < NCHAIN; ++i) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(64) void k_mul_lo_u32(uint64_t* out, uint64_t* stamps, uint32_t iters, uint32_t a,
                                                   uint32_t b) {
  uint32_t acc[NCHAIN];
  const uint32_t y = b ^ threadIdx.x;
  for (int i = 0; i < NCHAIN; ++i) acc[i] = threadIdx.x + i + a;
  Stamp sp;
  sp.begin(stamps);
  for (uint32_t it = 0; it < iters; ++it) asm volatile(R4(MUL8) : ACC8 : [y] "v"(y));
  sp.end(stamps);
  uint64_t s = 0;
  for (int i = 0; i < NCHAIN; ++i) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// a single dependent chain (the production product's one-accumulator order): latency-bound at
// one wave per SIMD
__global__ __launch_bounds__(64) void k_mad_chain(uint64_t* out, uint64_t* stamps, uint32_t iters, uint32_t a,
                                                  uint32_t b) {
  uint64_t acc[NCHAIN];
  const uint32_t x = a + threadIdx.x, y = b ^ threadIdx.x;
  for (int i = 0; i < NCHAIN; ++i) acc[i] = threadIdx.x + i;
  Stamp sp;
  sp.begin(stamps);
  for (uint32_t it = 0; it < iters; ++it)
    asm volatile(R4(R4("v_mad_u64_u32 %[a0], vcc, %[x], %[y], %[a0]\n\tv_mad_u64_u32 %[a0], vcc, %[x], %[y], %[a0]\n\t"))
                 : [a0] "+v"(acc[0])
                 : [x] "v"(x), [y] "v"(y)
                 : "vcc");
  sp.end(stamps);
  uint64_t s = 0;
  for (int i = 0; i < NCHAIN; ++i) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef void (*kfn)(uint64_t*, uint64_t*, uint32_t, uint32_t, uint32_t);

static int run(const char* name, kfn k, int insts_per_step, int waves_per_simd, uint64_t* d, uint64_t* dst) {
  int ncu = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess || ncu <= 0) return 1;
  const int blocks = ncu * 4 * waves_per_simd, threads = 64;
  // ~20 ms per launch at ~5 cycles per instruction and ~2 GHz: 8 x iters x 5 cycles x w waves
  const uint32_t iters = (uint32_t)((1u << 18) / (uint32_t)(waves_per_simd * insts_per_step));
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return 1;
  for (int r = 0; r < 40; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, nullptr, iters, 0x12345u, 0x9876543u);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  const int reps = 10;
  hipEventRecord(e0);
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, r == reps - 1 ? dst : nullptr, iters, 0x12345u,
                       0x9876543u);
  hipEventRecord(e1);
  if (hipEventSynchronize(e1) != hipSuccess) return 1;
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<uint64_t> st((size_t)2 * blocks);
  if (hipMemcpy(st.data(), dst, st.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  std::vector<double> ghz;
  for (int b = 0; b < blocks; ++b)
    if (st[2 * b + 1]) ghz.push_back((double)st[2 * b] / (double)st[2 * b + 1] * 0.1);
  std::sort(ghz.begin(), ghz.end());
  const double clk = ghz.empty() ? 0.0 : ghz[ghz.size() / 2];
  // one loop iteration = one asm statement: 4 rounds x NCHAIN chains x insts_per_step instructions
  const double lane_ops = (double)reps * blocks * threads * (double)iters * 4 * NCHAIN * insts_per_step;
  const double rate = lane_ops / (ms * 1e-3);
  const double full24 = (double)ncu * 64 * 2.4e9, full_held = (double)ncu * 64 * clk * 1e9;
  const double cyc = clk > 0 ? ((double)ncu * 4 * clk * 1e9) / (rate / 64.0) : 0.0;
  printf("{\"inst\": \"%s\", \"waves_per_simd\": %d, \"lane_ops_per_s\": %.4e, \"clock_ghz\": %.3f, "
         "\"clock_ghz_p10_p90\": [%.3f, %.3f], \"cycles_per_inst_per_simd\": %.3f, \"frac_fullrate_2p4\": %.4f, "
         "\"frac_fullrate_held\": %.4f, \"ms_per_launch\": %.3f}\n",
         name, waves_per_simd, rate, clk, ghz.empty() ? 0.0 : ghz[ghz.size() / 10],
         ghz.empty() ? 0.0 : ghz[ghz.size() * 9 / 10], cyc, rate / full24, clk > 0 ? rate / full_held : 0.0, ms / reps);
  fflush(stdout);
  return 0;
}

int main() {
  uint64_t *d = nullptr, *dst = nullptr;
  if (hipMalloc(&d, (size_t)256 * 4 * 8 * 64 * sizeof(uint64_t)) != hipSuccess ||
      hipMalloc(&dst, (size_t)2 * 256 * 4 * 8 * sizeof(uint64_t)) != hipSuccess)
    return 1;
  for (int w : {1, 2, 4, 8}) {
    if (run("v_mad_u64_u32", k_mad_u64_u32, 1, w, d, dst)) return 1;
    if (run("v_add_co_u32", k_add_co_u32, 1, w, d, dst)) return 1;
  }
  for (int w : {1, 4}) {
    if (run("v_mul_lo_u32", k_mul_lo_u32, 1, w, d, dst)) return 1;
    if (run("v_mad_u64_u32 one dependent chain", k_mad_chain, 1, w, d, dst)) return 1;
  }
  (void)hipFree(d);
  (void)hipFree(dst);
  return 0;
}
