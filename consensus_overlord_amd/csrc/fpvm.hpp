// Fp-VM interpreter for gfx950: executes the phase-major programs produced by
// tools/fpvm/gen.py (vm_progs.inc) on one W-lane slice of a wave per unit of work (a vote,
// a fold of partials, a final check).
//
// LDS holds each slice's register file: `nslots` Fp slots of 12 x u32 (48 B, read and written
// as three ds_*_b128), plus the shared constant table. In every phase each lane runs at most
// one op (the generator's schedule) and the workgroup barrier makes its result visible to the
// next phase. Opcodes and operand encoding: tools/fpvm/sched.py.
#pragma once
#include "bls/fp.hpp"

namespace ovh {
namespace vm {

enum : uint32_t {
  OP_NOP = 0, OP_MULS = 1, OP_SGN0 = 2, OP_LEX = 3, OP_LIN = 4, OP_SEL = 5, OP_EQ = 6,
  OP_AND = 7, OP_OR = 8, OP_XOR = 9, OP_RBIT = 10, OP_ST = 11, OP_SELB = 12,
};

// Where `st` ops write: plane `imm` of unit `unit` in a structure-of-arrays slab (limb k of
// plane j at base[(j * 12 + k) * cap + unit]).
struct Out {
  uint32_t* base;
  uint32_t cap;
  uint32_t unit;
};
constexpr uint32_t CONST_BASE = 0x800;
constexpr uint32_t ABSENT = 0xFFFF;

__device__ __forceinline__ void ld_slot(Fp& r, const uint32_t* __restrict__ slots, const uint32_t* __restrict__ cst,
                                        uint32_t ref) {
  const uint32_t* src = ref >= CONST_BASE ? cst + (ref - CONST_BASE) * 12 : slots + ref * 12;
  const uint4* s4 = reinterpret_cast<const uint4*>(src);
  const uint4 a = s4[0], b = s4[1], c = s4[2];
  r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
  r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
  r.v[8] = c.x; r.v[9] = c.y; r.v[10] = c.z; r.v[11] = c.w;
}

__device__ __forceinline__ void st_slot(uint32_t* __restrict__ slots, uint32_t dst, const Fp& z) {
  uint4* d4 = reinterpret_cast<uint4*>(slots + dst * 12);
  d4[0] = make_uint4(z.v[0], z.v[1], z.v[2], z.v[3]);
  d4[1] = make_uint4(z.v[4], z.v[5], z.v[6], z.v[7]);
  d4[2] = make_uint4(z.v[8], z.v[9], z.v[10], z.v[11]);
}

__device__ __forceinline__ void set_flag(Fp& z, uint32_t f) {
  fp_zero(z);
  z.v[0] = f;
}

// x = A (+|-) B, B absent -> x = A
__device__ __forceinline__ void combine(Fp& x, const uint32_t* slots, const uint32_t* cst, uint32_t ra, uint32_t rb,
                                        uint32_t neg) {
  if (ra == ABSENT) fp_zero(x);
  else ld_slot(x, slots, cst, ra);
  if (rb != ABSENT) {
    Fp b;
    ld_slot(b, slots, cst, rb);
    if (neg) fp_sub(x, x, b);
    else fp_add(x, x, b);
  }
}

// One op of one lane. `in` = (w0, A|B<<16, C|D<<16, 0).
__device__ __forceinline__ void exec(const uint4 in, uint32_t* __restrict__ slots, const uint32_t* __restrict__ cst,
                                     uint64_t scalar, const Out& out) {
  const uint32_t op = in.x & 31;
  if (op == OP_NOP) return;
  const uint32_t dst = (in.x >> 8) & 0x7FF;
  const uint32_t ra = in.y & 0xFFFF, rb = in.y >> 16, rc = in.z & 0xFFFF, rd = in.z >> 16;
  Fp z;
  if (op == OP_ST) {
    ld_slot(z, slots, cst, ra);
    uint32_t* b = out.base + (size_t)((in.x >> 20) & 63) * 12 * out.cap + out.unit;
#pragma unroll
    for (int k = 0; k < 12; ++k) b[(size_t)k * out.cap] = z.v[k];
    return;
  }
  if (op == OP_SELB) {
    ld_slot(z, slots, cst, ((scalar >> ((in.x >> 20) & 63)) & 1) ? rc : rb);
  } else if (op == OP_RBIT) {
    set_flag(z, (uint32_t)(scalar >> ((in.x >> 20) & 63)) & 1u);
  } else if (op == OP_SEL) {
    Fp f;
    ld_slot(f, slots, cst, ra);
    ld_slot(z, slots, cst, f.v[0] ? rc : rb);
  } else if (op >= OP_AND) {
    Fp a, c;
    ld_slot(a, slots, cst, ra);
    ld_slot(c, slots, cst, rc);
    set_flag(z, op == OP_AND ? (a.v[0] & c.v[0]) : op == OP_OR ? (a.v[0] | c.v[0]) : (a.v[0] ^ c.v[0]));
  } else {
    Fp x, y;
    combine(x, slots, cst, ra, rb, (in.x >> 5) & 1);
    combine(y, slots, cst, rc, rd, (in.x >> 7) & 1);
    if (op <= OP_LEX) {
      fp_mul(z, x, y);
      if (op == OP_SGN0) set_flag(z, z.v[0] & 1u);
      else if (op == OP_LEX) set_flag(z, limbs_gt(z.v, HALF_P) ? 1u : 0u);
    } else if (op == OP_LIN) {
      if ((in.x >> 6) & 1) fp_sub(z, x, y);
      else fp_add(z, x, y);
    } else {  // OP_EQ
      set_flag(z, fp_eq(x, y) ? 1u : 0u);
    }
  }
  st_slot(slots, dst, z);
}

// Run `nphases` phases of a W-lane program. Every lane of the workgroup must call this (the
// phase barrier is a workgroup barrier); lanes of inactive slices pass active = false.
__device__ __forceinline__ void run(const uint4* __restrict__ code, uint32_t nphases, uint32_t W, uint32_t lane,
                                    bool active, uint32_t* __restrict__ slots, const uint32_t* __restrict__ cst,
                                    uint64_t scalar, const Out& out) {
  uint4 nxt = code[lane];
#pragma unroll 1
  for (uint32_t ph = 0; ph < nphases; ++ph) {
    const uint4 cur = nxt;
    nxt = code[(size_t)(ph + 1) * W + lane];  // code carries one trailing NOP phase
    if (active) exec(cur, slots, cst, scalar, out);
    __syncthreads();
  }
}

}  // namespace vm
}  // namespace ovh
