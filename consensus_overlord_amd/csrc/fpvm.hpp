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

// The interpreter also builds on the host (g++, tests/host/harness.cpp) so the CPU test suite
// runs the generated programs through this exact code; run() is device-only.
#if defined(__HIPCC__)
#define VM_FN __device__ __forceinline__
#else
#define VM_FN inline
struct uint4 {
  uint32_t x, y, z, w;
};
inline uint4 make_uint4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) { return uint4{a, b, c, d}; }
#endif

namespace ovh {
namespace vm {

enum : uint32_t {
  OP_NOP = 0, OP_MULS = 1, OP_SGN0 = 2, OP_LEX = 3, OP_INV = 4, OP_LIN = 5, OP_SEL = 6, OP_EQ = 7,
  OP_AND = 8, OP_OR = 9, OP_XOR = 10, OP_ST = 11, OP_SELB = 12,
};

// Where `st` ops write: plane `imm` of unit `unit` in a structure-of-arrays slab (limb k of
// plane j at base[(j * 12 + k) * cap + unit]).
struct Out {
  uint32_t* base;
  uint32_t cap;
  uint32_t unit;
};
constexpr uint32_t CONST_BASE = 0x800;

VM_FN void ld_slot(Fp& r, const uint32_t* __restrict__ slots, const uint32_t* __restrict__ cst,
                                        uint32_t ref) {
  const uint32_t* src = ref >= CONST_BASE ? cst + (ref - CONST_BASE) * 12 : slots + ref * 12;
  const uint4* s4 = reinterpret_cast<const uint4*>(src);
  const uint4 a = s4[0], b = s4[1], c = s4[2];
  r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
  r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
  r.v[8] = c.x; r.v[9] = c.y; r.v[10] = c.z; r.v[11] = c.w;
}

VM_FN void st_slot(uint32_t* __restrict__ slots, uint32_t dst, const Fp& z) {
  uint4* d4 = reinterpret_cast<uint4*>(slots + dst * 12);
  d4[0] = make_uint4(z.v[0], z.v[1], z.v[2], z.v[3]);
  d4[1] = make_uint4(z.v[4], z.v[5], z.v[6], z.v[7]);
  d4[2] = make_uint4(z.v[8], z.v[9], z.v[10], z.v[11]);
}

VM_FN void set_flag(Fp& z, uint32_t f) {
  fp_zero(z);
  z.v[0] = f;
}

// acc (13 limbs) += c * X for |c| <= 15, branch-free on the coefficient's value and sign.
VM_FN void acc_term(uint32_t* acc, const Fp& X, int c) {
  const uint32_t k = c < 0 ? (uint32_t)(-c) : (uint32_t)c;
  const uint32_t mask = c < 0 ? 0xFFFFFFFFu : 0u;
  uint64_t pr = 0;
  uint32_t cy = c < 0 ? 1u : 0u;  // two's complement: acc + ~prod + 1
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    pr = (uint64_t)X.v[j] * k + (pr >> 32);
    acc[j] = addc32(acc[j], (uint32_t)pr ^ mask, cy, &cy);
  }
  acc[12] = acc[12] + ((uint32_t)(pr >> 32) ^ mask) + cy;
}

// acc = 2^k p (k = 5: 32 p, k = 6: 64 p), 13 limbs: the bias that keeps a signed sum >= 0
VM_FN void acc_bias(uint32_t* acc, int k) {
  uint32_t prev = 0;
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    acc[j] = (P_LIMBS[j] << k) | (prev >> (32 - k));
    prev = P_LIMBS[j];
  }
  acc[12] = prev >> (32 - k);
}

// acc in [0, 128 p) -> acc mod p. With top = acc >> 352 and p_top = p >> 352, the ratio
// r = top / (p_top + 1) has floor(r) = floor(acc / p) or one less. The f32 quotient f below
// carries a relative error < 3 * 2^-24 and is shrunk by 2^-20, so f <= r and
// floor(f) >= floor(r) - 1: q = floor(f) is at most floor(acc / p) and at most 2 short of it.
// Subtract q p, then two conditional subtractions.
// 2p as 12 limbs + a top limb
constexpr uint32_t P2_LIMBS[12] = {
    P_LIMBS[0] << 1, (P_LIMBS[1] << 1) | (P_LIMBS[0] >> 31), (P_LIMBS[2] << 1) | (P_LIMBS[1] >> 31),
    (P_LIMBS[3] << 1) | (P_LIMBS[2] >> 31), (P_LIMBS[4] << 1) | (P_LIMBS[3] >> 31),
    (P_LIMBS[5] << 1) | (P_LIMBS[4] >> 31), (P_LIMBS[6] << 1) | (P_LIMBS[5] >> 31),
    (P_LIMBS[7] << 1) | (P_LIMBS[6] >> 31), (P_LIMBS[8] << 1) | (P_LIMBS[7] >> 31),
    (P_LIMBS[9] << 1) | (P_LIMBS[8] >> 31), (P_LIMBS[10] << 1) | (P_LIMBS[9] >> 31),
    (P_LIMBS[11] << 1) | (P_LIMBS[10] >> 31)};
constexpr uint32_t P2_TOP = P_LIMBS[11] >> 31;

VM_FN void acc_reduce(Fp& r, uint32_t* acc) {
  const uint64_t top = ((uint64_t)acc[12] << 32) | acc[11];  // acc >> 352
  constexpr float QS = (float)((1.0 - 0x1p-20) / ((double)P_LIMBS[11] + 1.0));
  const uint32_t q = (uint32_t)((float)top * QS);
  uint64_t pr = 0;
  uint32_t br = 0;
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    pr = (uint64_t)P_LIMBS[j] * q + (pr >> 32);
    acc[j] = subc32(acc[j], (uint32_t)pr, br, &br);
  }
  acc[12] = acc[12] - (uint32_t)(pr >> 32) - br;
  // acc is now below 3p: acc - p and acc - 2p as two interleaved borrow chains, keep the
  // smallest non-negative of acc, acc - p, acc - 2p
  uint32_t d1[13], d2[13], b1 = 0, b2 = 0;
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    d1[j] = subc32(acc[j], P_LIMBS[j], b1, &b1);
    d2[j] = subc32(acc[j], P2_LIMBS[j], b2, &b2);
  }
  d1[12] = subc32(acc[12], 0u, b1, &b1);
  d2[12] = subc32(acc[12], P2_TOP, b2, &b2);
#pragma unroll
  for (int j = 0; j < 13; ++j) acc[j] = !b2 ? d2[j] : (!b1 ? d1[j] : acc[j]);
#pragma unroll
  for (int j = 0; j < 12; ++j) r.v[j] = acc[j];
}

// Modular inverse of a Montgomery value by the binary extended Euclidean algorithm on the
// raw representation (the inputs are public batch data: variable time is fine), then back to
// Montgomery form with one product by raw R^3 (r3). 0 -> 0.
VM_FN bool limbs_is_one(const Fp& w) {
  uint32_t acc = w.v[0] ^ 1u;
#pragma unroll
  for (int i = 1; i < 12; ++i) acc |= w.v[i];
  return acc == 0;
}

// w /= 2; x = x / 2 mod p
VM_FN void halve2(Fp& w, Fp& x) {
#pragma unroll
  for (int i = 0; i < 11; ++i) w.v[i] = (w.v[i] >> 1) | (w.v[i + 1] << 31);
  w.v[11] >>= 1;
  uint32_t c = 0;
  const uint32_t m = 0u - (x.v[0] & 1u);
#pragma unroll
  for (int i = 0; i < 12; ++i) x.v[i] = addc32(x.v[i], P_LIMBS[i] & m, c, &c);
#pragma unroll
  for (int i = 0; i < 11; ++i) x.v[i] = (x.v[i] >> 1) | (x.v[i + 1] << 31);
  x.v[11] = (x.v[11] >> 1) | (c << 31);
}

VM_FN void fp_inv_binary(Fp& r, const Fp& a, const Fp& r3) {
  Fp u = a, v, x1, x2;
  fp_load(v, P_LIMBS);
  fp_zero(x1);
  x1.v[0] = 1;
  fp_zero(x2);
  if (fp_is_zero(a)) {
    fp_zero(r);
    return;
  }
#pragma unroll 1
  while (!limbs_is_one(u) && !limbs_is_one(v)) {
#pragma unroll 1
    while (!(u.v[0] & 1)) halve2(u, x1);
#pragma unroll 1
    while (!(v.v[0] & 1)) halve2(v, x2);
    uint32_t br = 0;
    Fp d;
#pragma unroll
    for (int i = 0; i < 12; ++i) d.v[i] = subc32(u.v[i], v.v[i], br, &br);
    if (!br) {
      u = d;
      fp_sub(x1, x1, x2);
    } else {
      br = 0;
#pragma unroll
      for (int i = 0; i < 12; ++i) v.v[i] = subc32(v.v[i], u.v[i], br, &br);
      fp_sub(x2, x2, x1);
    }
  }
  fp_mul(r, limbs_is_one(u) ? x1 : x2, r3);
}

// r = A + s B mod p for s in {-1, 0, +1} (A, B < p; the encoder points B at the zero
// constant when s = 0), branch-free: d = A + (s < 0 ? p - B : B) < 2p, then one conditional
// subtraction of p.
VM_FN void addsub(Fp& r, const Fp& A, const Fp& B, int s) {
  // the three carry chains (p - B, A + B', d - p) run skewed by one limb each and interleave, so
  // no chain's carry read directly follows its own carry write (gfx950 wait states)
  uint32_t nb[12], d[12], t[12], b0 = 0, c1 = 0, b2 = 0;
  const bool ng = s < 0;
#pragma unroll
  for (int j = 0; j < 14; ++j) {
    if (j < 12) nb[j] = subc32(P_LIMBS[j], B.v[j], b0, &b0);
    if (j >= 1 && j <= 12) d[j - 1] = addc32(A.v[j - 1], ng ? nb[j - 1] : B.v[j - 1], c1, &c1);
    if (j >= 2) t[j - 2] = subc32(d[j - 2], P_LIMBS[j - 2], b2, &b2);
  }
#pragma unroll
  for (int j = 0; j < 12; ++j) r.v[j] = b2 ? d[j] : t[j];
}

// Two independent addsubs with their carry chains interleaved limb by limb: on gfx950 a VALU
// carry read right after the VALU carry write costs wait states (s_nop), which the other
// chain's instruction fills.
VM_FN void addsub2(Fp& r1, const Fp& A1, const Fp& B1, int s1, Fp& r2, const Fp& A2, const Fp& B2, int s2) {
  uint32_t n1[12], n2[12], d1[12], d2[12], t1[12], t2[12], b1 = 0, b2 = 0, c1 = 0, c2 = 0;
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    n1[j] = subc32(P_LIMBS[j], B1.v[j], b1, &b1);
    n2[j] = subc32(P_LIMBS[j], B2.v[j], b2, &b2);
  }
  const bool g1 = s1 < 0, g2 = s2 < 0;
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    d1[j] = addc32(A1.v[j], g1 ? n1[j] : B1.v[j], c1, &c1);
    d2[j] = addc32(A2.v[j], g2 ? n2[j] : B2.v[j], c2, &c2);
  }
  b1 = b2 = 0;
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    t1[j] = subc32(d1[j], P_LIMBS[j], b1, &b1);
    t2[j] = subc32(d2[j], P_LIMBS[j], b2, &b2);
  }
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    r1.v[j] = b1 ? d1[j] : t1[j];
    r2.v[j] = b2 ? d2[j] : t2[j];
  }
}

#if defined(__HIPCC__)
VM_FN bool wave_any(bool p) { return __ballot(p) != 0; }
#else
// host emulation runs one lane at a time; with g_host_any set every wave-uniform block runs
// for every lane (the device behaviour when any other lane of the wave needs the block)
extern bool g_host_any;
inline bool wave_any(bool p) { return p || g_host_any; }
#endif

// One phase of one lane. `in` = (w0, A|B<<16, C|D<<16, coefficients). The common ops share one
// straight-line body: x = A + cb B, y = C + cc cd D (unit coefficients, tools/fpvm/ir.lin_form),
// then fp_mul(x, y) (muls / sgn0 / lex), x == y (eq) or k (x + cc y) (lin). Each block runs
// when any lane of the wave needs it (a wave-uniform branch) and every lane keeps the result
// of its own op. Rare ops (sel, selb, logic, st, inv, lin with general coefficients) take
// per-lane branches after that.
VM_FN void exec(const uint4 in, bool active, uint32_t* __restrict__ slots,
                                     const uint32_t* __restrict__ cst, uint64_t scalar, const Out& out) {
  const uint32_t op = active ? (in.x & 31) : (uint32_t)OP_NOP;
  if (!wave_any(op != OP_NOP)) return;
  const uint32_t dst = (in.x >> 5) & 0x7FF;
  const uint32_t imm = (in.x >> 16) & 63;
  // four operands, always valid references (a missing one is the zero constant)
  Fp A, B, C, D;
  ld_slot(A, slots, cst, in.y & 0xFFFF);
  ld_slot(B, slots, cst, in.y >> 16);
  ld_slot(C, slots, cst, in.z & 0xFFFF);
  ld_slot(D, slots, cst, in.z >> 16);
  const int ca = ((int)(in.w << 27)) >> 27, cb = ((int)(in.w << 22)) >> 27;
  const int cc = ((int)(in.w << 17)) >> 27, cd = ((int)(in.w << 12)) >> 27;
  const bool is_mul = op == OP_MULS || op == OP_SGN0 || op == OP_LEX || op == OP_EQ;
  const bool lin_unit = ca == 1 && cb >= -1 && cb <= 1 && cc >= -1 && cc <= 1 && cd >= -1 && cd <= 1;
  const bool is_lin = op == OP_LIN && lin_unit;
  Fp z = A;
  if (wave_any(is_mul || is_lin)) {
    Fp x, y;
    addsub2(x, A, B, cb, y, C, D, cc * cd);
    if (wave_any(is_mul)) {
      Fp m;
      fp_mul(m, x, y);
      const bool flag = is_mul && op != OP_MULS;
      if (wave_any(flag)) {
        uint32_t f = 0;
        if (op == OP_SGN0) f = m.v[0] & 1u;
        if (op == OP_LEX) f = limbs_gt(m.v, HALF_P) ? 1u : 0u;
        if (op == OP_EQ) f = fp_eq(x, y) ? 1u : 0u;
#pragma unroll
        for (int j = 0; j < 12; ++j) m.v[j] = flag ? (j == 0 ? f : 0u) : m.v[j];
      }
      if (is_mul) z = m;
    }
    if (wave_any(is_lin)) {
      Fp l;
      addsub(l, x, y, cc);
      const uint32_t k = (in.w >> 20) & 15;
      if (wave_any(is_lin && k > 1)) {  // "scaled" form: k * (unit sum), k < 16 (k <= 1: unchanged)
        uint32_t acc[13];
        uint64_t pr = 0;
        const uint32_t kk = k > 1 ? k : 1u;
#pragma unroll
        for (int j = 0; j < 12; ++j) {
          pr = (uint64_t)l.v[j] * kk + (pr >> 32);
          acc[j] = (uint32_t)pr;
        }
        acc[12] = (uint32_t)(pr >> 32);
        acc_reduce(l, acc);
      }
      if (is_lin) z = l;
    }
  }
  const bool rare = op != OP_NOP && !is_mul && !is_lin;
  if (wave_any(rare)) {
    if (op == OP_ST) {
      uint32_t* b = out.base + (size_t)imm * 12 * out.cap + out.unit;
#pragma unroll
      for (int k = 0; k < 12; ++k) b[(size_t)k * out.cap] = A.v[k];
    } else if (op == OP_SELB) {
      z = ((scalar >> imm) & 1) ? C : B;
    } else if (op == OP_SEL) {
      z = A.v[0] ? C : B;
    } else if (op >= OP_AND && op <= OP_XOR) {
      set_flag(z, op == OP_AND ? (A.v[0] & C.v[0]) : op == OP_OR ? (A.v[0] | C.v[0]) : (A.v[0] ^ C.v[0]));
    } else if (op == OP_INV) {
#ifndef OVH_VM_NO_INV
      fp_inv_binary(z, A, C);
#endif
    } else if (op == OP_LIN && !lin_unit) {  // general coefficients
      uint32_t acc[13];
      acc_bias(acc, 6);
      acc_term(acc, A, ca);
      acc_term(acc, B, cb);
      acc_term(acc, C, cc);
      acc_term(acc, D, cd);
      acc_reduce(z, acc);
    }
  }
  if (op != OP_NOP && op != OP_ST) st_slot(slots, dst, z);
}

// Run `nphases` phases of a W-lane program. Every lane of the workgroup must call this (the
// phase barrier is a workgroup barrier); lanes of inactive slices pass active = false.
#if defined(__HIPCC__)
__device__ __forceinline__ void run(const uint4* __restrict__ code, uint32_t nphases, uint32_t W, uint32_t lane,
                                    bool active, uint32_t* __restrict__ slots, const uint32_t* __restrict__ cst,
                                    uint64_t scalar, const Out& out, uint64_t* __restrict__ trace = nullptr) {
  // trace (diagnostics, OVH_FLAG_VM_TRACE): wall clock after every phase barrier
  if (trace && threadIdx.x == 0) trace[0] = wall_clock64();
  // instructions are prefetched two phases ahead (an HBM/L2 round trip outlasts a light phase)
  uint4 nxt = code[lane], nxt2 = code[(size_t)W + lane];
#pragma unroll 1
  for (uint32_t ph = 0; ph < nphases; ++ph) {
    const uint4 cur = nxt;
    nxt = nxt2;
    nxt2 = code[(size_t)(ph + 2) * W + lane];  // code carries two trailing NOP phases
    exec(cur, active, slots, cst, scalar, out);
    // The VM kernels are single-wave workgroups: the phase's slot writes are visible to the
    // next phase's reads once this wave's LDS operations completed (lgkmcnt(0)); the barrier
    // is kept for ordering but no longer waits for the instruction prefetch / HBM stores.
    __asm__ volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (trace && threadIdx.x == 0) trace[ph + 1] = wall_clock64();
  }
}

#endif  // __HIPCC__

}  // namespace vm
}  // namespace ovh
