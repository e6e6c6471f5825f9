// Microbenchmark of the Fp-VM interpreter on gfx950 (consensus_overlord_amd/csrc/fpvm.hpp):
// cost of a NOP / LIN / MULS phase at several occupancies, and the latency of a dependent
// Montgomery product chain without LDS or barriers. Prints one JSON line per case.
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/vm_phase tools/ubench/vm_phase.hip && /tmp/vm_phase
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#include "../../consensus_overlord_amd/csrc/fpvm.hpp"
#include "../../consensus_overlord_amd/csrc/vm_progs.inc"

namespace ovh { namespace vm { constexpr uint32_t ABSENT = CONST_BASE + KZERO; } }

using namespace ovh;

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));     \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

constexpr int NSLOT = 64;

__global__ __launch_bounds__(64) void k_vm(const uint4* code, uint32_t nph, uint32_t W, const uint32_t* cst_g,
                                           uint32_t* out) {
  __shared__ uint32_t lds[VM_NCONST * 12 + 4 * NSLOT * 12];
  uint32_t* cst = lds;
  for (uint32_t k = threadIdx.x; k < VM_NCONST * 12; k += 64) cst[k] = cst_g[k];
  const uint32_t slice = threadIdx.x / W, lane = threadIdx.x % W;
  uint32_t* slots = lds + VM_NCONST * 12 + slice * NSLOT * 12;
  for (int k = 0; k < 12; ++k) slots[lane * 12 + k] = (k == 0) ? (lane + 3) : (k < 11 ? 0x1234567u * (lane + k) : 0);
  __syncthreads();
  vm::run(code, nph, W, lane, true, slots, cst, 0x5555aaaa5555aaaaull, vm::Out{nullptr, 0, 0});
  if (lane == 0) out[blockIdx.x * 64 + threadIdx.x] = slots[0];
}

// run() with every phase fetching the SAME code block (period 1): the instruction stream always
// hits in cache; compared with k_vm it prices the code-fetch latency the 1-phase prefetch exposes
__global__ __launch_bounds__(64) void k_vm_samecode(const uint4* code, uint32_t nph, uint32_t W, const uint32_t* cst_g,
                                                    uint32_t* out) {
  __shared__ uint32_t lds[VM_NCONST * 12 + 4 * NSLOT * 12];
  uint32_t* cst = lds;
  for (uint32_t k = threadIdx.x; k < VM_NCONST * 12; k += 64) cst[k] = cst_g[k];
  const uint32_t slice = threadIdx.x / W, lane = threadIdx.x % W;
  uint32_t* slots = lds + VM_NCONST * 12 + slice * NSLOT * 12;
  for (int k = 0; k < 12; ++k) slots[lane * 12 + k] = (k == 0) ? (lane + 3) : (k < 11 ? 0x1234567u * (lane + k) : 0);
  __syncthreads();
  uint4 q = code[lane];
#pragma unroll 1
  for (uint32_t ph = 0; ph < nph; ++ph) {
    const uint4 cur = q;
    q = code[lane + (ph & 1) * 0];
    vm::exec(cur, true, slots, cst, 0x5555aaaa5555aaaaull, vm::Out{nullptr, 0, 0});
  }
  __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (lane == 0) out[blockIdx.x * 64 + threadIdx.x] = slots[0];
}

__global__ __launch_bounds__(64) void k_chain(uint32_t iters, uint32_t* out) {
  Fp x, y;
  for (int k = 0; k < 12; ++k) {
    x.v[k] = (k < 11) ? 0x9abcdefu * (threadIdx.x + k + 1) : 0;
    y.v[k] = (k < 11) ? 0x1234567u * (threadIdx.x + k + 7) : 0;
  }
  for (uint32_t i = 0; i < iters; ++i) fp_mul(x, x, y);
  out[blockIdx.x * 64 + threadIdx.x] = x.v[0];
}

static uint32_t w0(uint32_t op, uint32_t dst) { return op | dst << 5; }

static int s5(uint32_t x) { return (x & 16) ? (int)x - 32 : (int)x; }

// phase header bits of one lane (tools/fpvm/sched.py phase_bits)
static uint32_t phase_bits(const uint32_t* w) {
  using namespace vm;
  const uint32_t opc = w[0] & 31;
  if (opc == OP_NOP) return 0;
  const int ca = s5(w[3] & 31), cb = s5((w[3] >> 5) & 31), cc = s5((w[3] >> 10) & 31), cd = s5((w[3] >> 15) & 31);
  if (opc == OP_MULS || opc == OP_SGN0 || opc == OP_LEX || opc == OP_EQ)
    return H_MUL | ((cb < 0 || cd < 0) ? H_MULNEG : 0) | (opc == OP_MULS ? 0 : H_FLAG);
  if (opc == OP_SELB) return H_LIN | H_SELB;
  if (opc == OP_LIN) {
    const bool unit = ca == 1 && cb >= -1 && cb <= 1 && cc >= -1 && cc <= 1 && cd >= -1 && cd <= 1;
    return unit ? (H_LIN | ((cb < 0 || cc < 0 || cd < 0) ? H_LINNEG : 0)) : H_ACC;
  }
  return H_RARE;
}

int main(int argc, char** argv) {
  // optional: vm_phase KIND W GRID -> that one case only (for PMC passes)
  const int only_kind = argc > 3 ? atoi(argv[1]) : -1;
  const uint32_t only_w = argc > 3 ? (uint32_t)atoi(argv[2]) : 0, only_grid = argc > 3 ? (uint32_t)atoi(argv[3]) : 0;
  const uint32_t NPH = 2048;
  uint32_t *d_cst, *d_out;
  CHECK(hipMalloc(&d_cst, sizeof(VM_CONST_WORDS)));
  CHECK(hipMemcpy(d_cst, VM_CONST_WORDS, sizeof(VM_CONST_WORDS), hipMemcpyHostToDevice));
  CHECK(hipMalloc(&d_out, 64 * 8192 * 4));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  const char* names[] = {"nop", "lin", "muls", "muls_half_lanes", "lin_coef", "muls_preadd", "lin4_neg", "selb",
                         "muls+lin4"};
  for (uint32_t W : {16u, 64u}) {
    if (only_kind >= 0 && W != only_w) continue;
    for (int kind = 0; kind < 9; ++kind) {
      if (only_kind >= 0 && kind != only_kind) continue;
      std::vector<uint32_t> code((size_t)(NPH + vm::PREFETCH) * W * 4, 0);
      for (uint32_t ph = 0; ph < NPH; ++ph)
        for (uint32_t l = 0; l < W; ++l) {
          uint32_t* c = &code[((size_t)ph * W + l) * 4];
          const uint32_t src = (l + 1) % W;
          if (kind == 1) {
            c[0] = w0(vm::OP_LIN, l);
            c[1] = l | src << 16;
            c[2] = vm::ABSENT | vm::ABSENT << 16;
            c[3] = 1 | 1 << 5;
          } else if (kind == 4) {
            c[0] = w0(vm::OP_LIN, l);
            c[1] = l | src << 16;
            c[2] = ((l + 2) % W) | ((l + 3) % W) << 16;
            c[3] = 3 | (32 - 2) << 5 | 6 << 10 | (32 - 1) << 15;  // 3a - 2b + 6c - d
          } else if (kind == 5) {
            c[0] = w0(vm::OP_MULS, l);
            c[1] = l | src << 16;
            c[2] = ((l + 2) % W) | ((l + 3) % W) << 16;
            c[3] = 1 | 1 << 5 | 1 << 10 | (32 - 1) << 15;  // (a + b)(c - d)
          } else if (kind == 6 || (kind == 8 && l % 2 == 1)) {
            c[0] = w0(vm::OP_LIN, l);
            c[1] = l | src << 16;
            c[2] = ((l + 2) % W) | ((l + 3) % W) << 16;
            c[3] = 1 | (32 - 1) << 5 | 1 << 10 | (32 - 1) << 15;  // a - b + c - d
          } else if (kind == 7) {
            c[0] = w0(vm::OP_SELB, l) | (l % 64) << 16;
            c[1] = vm::ABSENT | src << 16;
            c[2] = ((l + 2) % W) | vm::ABSENT << 16;
            c[3] = 0;
          } else if ((kind >= 2 && kind <= 3 && (kind == 2 || l % 2 == 0)) || kind == 8) {
            c[0] = w0(vm::OP_MULS, l);
            c[1] = l | vm::ABSENT << 16;
            c[2] = src | vm::ABSENT << 16;
            c[3] = 1 | 1 << 10;
          }
        }
      for (uint32_t ph = 0; ph < NPH; ++ph) {
        uint32_t h = 0;
        for (uint32_t l = 0; l < W; ++l) h |= phase_bits(&code[((size_t)ph * W + l) * 4]);
        for (uint32_t l = 0; l < W; ++l) code[((size_t)ph * W + l) * 4] |= h;
      }
      uint4* d_code;
      CHECK(hipMalloc(&d_code, code.size() * 4));
      CHECK(hipMemcpy(d_code, code.data(), code.size() * 4, hipMemcpyHostToDevice));
      for (uint32_t grid : {256u, 1024u, 2048u}) {
        if (only_kind >= 0 && grid != only_grid) continue;
        hipLaunchKernelGGL(k_vm, dim3(grid), dim3(64), 0, 0, d_code, NPH, W, d_cst, d_out);
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL(k_vm, dim3(grid), dim3(64), 0, 0, d_code, NPH, W, d_cst, d_out);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        printf("{\"case\": \"vm_%s\", \"W\": %u, \"waves\": %u, \"ms\": %.3f, \"ns_per_phase\": %.1f}\n", names[kind], W,
               grid, ms, ms * 1e6 / NPH);
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL(k_vm_samecode, dim3(grid), dim3(64), 0, 0, d_code, NPH, W, d_cst, d_out);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        CHECK(hipEventElapsedTime(&ms, a, b));
        printf("{\"case\": \"vm_%s_samecode\", \"W\": %u, \"waves\": %u, \"ms\": %.3f, \"ns_per_phase\": %.1f}\n",
               names[kind], W, grid, ms, ms * 1e6 / NPH);
      }
      CHECK(hipFree(d_code));
    }
  }
  if (only_kind >= 0) return 0;
  for (uint32_t grid : {256u, 1024u, 2048u, 4096u, 8192u}) {
    const uint32_t iters = 4096;
    hipLaunchKernelGGL(k_chain, dim3(grid), dim3(64), 0, 0, iters, d_out);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL(k_chain, dim3(grid), dim3(64), 0, 0, iters, d_out);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    printf("{\"case\": \"fp_mul_chain\", \"waves\": %u, \"ms\": %.3f, \"ns_per_mul\": %.1f, \"Mmul_per_s\": %.0f}\n",
           grid, ms, ms * 1e6 / iters, (double)grid * 64 * iters / (ms * 1e-3) / 1e6);
  }
  return 0;
}
