// Fp-VM interpreter for gfx950: executes the phase-major programs produced by
// tools/fpvm/gen.py (vm_progs.inc) on one W-lane slice of a wave per unit of work (a vote,
// a fold of partials, a final check).
//
// LDS holds each slice's register file: `nslots` Fp slots of 12 x u32 (48 B, read and written
// as three ds_*_b128), plus the shared constant table. In every phase each lane runs at most
// one op (the generator's schedule); a slot written in phase t is read from phase t + 1 on.
// Opcodes and operand encoding: tools/fpvm/sched.py.
//
// Lazy reduction. A slot holds a Montgomery representative in [0, 2p) (p < 2^381, so 2^384 >
// 9.8 p leaves room): products take operands in [0, 4p) -- a + b or a + (2p - b) of two slots,
// with no reduction -- and return [0, 1.625 p) after one conditional subtraction
// ((4p)^2 / 2^384 + p < 2.63 p); linear combinations sum their terms unreduced (< 8p, times
// k <= 15 < 120p) and reduce once by a float estimate of the quotient to [0, 2p). Only the ops
// whose result depends on the canonical value (sgn0, lex, the equality test, `st` outputs,
// inversion) canonicalise: a product by the plain 1 of a value below 4p is at most p.
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

// trailing NOP phases the uploaded code and side words carry (run's unrolled loops read past the
// end; r05's prefetch distance)
constexpr uint32_t PREFETCH = 6;

// Where `st` ops write: plane `imm` of unit `unit` in a structure-of-arrays slab (limb k of
// plane j at base[(j * 12 + k) * cap + unit]).
struct Out {
  uint32_t* base;
  uint32_t cap;
  uint32_t unit;
};
constexpr uint32_t CONST_BASE = 0x800;
// fixed constant-table entries (tools/fpvm/gen.py): 0 the plain 1, 1 the zero, KTAB + n
// (n = 0..4) n (2p + 1) as raw limbs, the offset of a unit lin with n negated terms
constexpr uint32_t KZERO = 1, KTAB = 2;

VM_FN void ld_slot(Fp& r, const uint32_t* __restrict__ slots, const uint32_t* __restrict__ cst,
                   uint32_t ref) {
  // bit 11 picks the table, the low 11 bits index it (one select + one multiply-add)
  const uint32_t* src = ((ref & CONST_BASE) ? cst : slots) + (ref & (CONST_BASE - 1)) * 12;
  const uint4* s4 = reinterpret_cast<const uint4*>(src);
  const uint4 a = s4[0], b = s4[1], c = s4[2];
  r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
  r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
  r.v[8] = c.x; r.v[9] = c.y; r.v[10] = c.z; r.v[11] = c.w;
}

VM_FN const uint4* slot_ptr(const uint32_t* __restrict__ slots, const uint32_t* __restrict__ cst, uint32_t ref) {
  return reinterpret_cast<const uint4*>(((ref & CONST_BASE) ? cst : slots) + (ref & (CONST_BASE - 1)) * 12);
}

// the four operands of a phase, loaded limb-quarter-major (B, D, A, C for limbs 0..3, then 4..7,
// then 8..11): the pre-add / lin chains start on the low limbs while the rest is in flight
#if defined(__HIPCC__)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(3))) uint32_t* lds_cptr;
VM_FN uint32_t lds_addr(const uint32_t* __restrict__ slots, const uint32_t* __restrict__ cst, uint32_t ref) {
  return (uint32_t)(uintptr_t)(lds_cptr)(((ref & CONST_BASE) ? cst : slots) + (ref & (CONST_BASE - 1)) * 12);
}
VM_FN void unpack4(Fp& r, int q, const u32x4 v) {
  r.v[4 * q] = v.x; r.v[4 * q + 1] = v.y; r.v[4 * q + 2] = v.z; r.v[4 * q + 3] = v.w;
}
#endif

VM_FN void ld_slots4(Fp& A, Fp& B, Fp& C, Fp& D, const uint32_t* __restrict__ slots,
                     const uint32_t* __restrict__ cst, uint32_t ra, uint32_t rb, uint32_t rc, uint32_t rd) {
#if defined(__HIPCC__) && defined(OVH_VM_ASM_LOADS)
  // (A/B build; the compiler-scheduled loads below measured 1.3% faster in the vote kernel,
  // profiles/r03g_ab_summary.txt.) The twelve reads are issued in one asm statement and waited for in three (one per limb
  // quarter), so the compiler's waitcnt pass sees no LDS loads here: left to it, the loop's back
  // edge merged these loads' pending state with the stores the phase ends with and it put an
  // lgkmcnt(0) before the next phase's reads -- a full LDS round trip for the stores, every phase.
  // LDS operations of a wave complete in order, so lgkmcnt(8 / 4 / 0) right after the reads
  // guarantee the first 4 / 8 / 12 of them (and everything older) are done.
  const uint32_t xa = lds_addr(slots, cst, ra), xb = lds_addr(slots, cst, rb), xc = lds_addr(slots, cst, rc),
                 xd = lds_addr(slots, cst, rd);
  u32x4 b0, d0, a0, c0, b1, d1, a1, c1, b2, d2, a2, c2;
  asm volatile(
      "ds_read_b128 %0, %12\n\tds_read_b128 %1, %13\n\tds_read_b128 %2, %14\n\tds_read_b128 %3, %15\n\t"
      "ds_read_b128 %4, %12 offset:16\n\tds_read_b128 %5, %13 offset:16\n\t"
      "ds_read_b128 %6, %14 offset:16\n\tds_read_b128 %7, %15 offset:16\n\t"
      "ds_read_b128 %8, %12 offset:32\n\tds_read_b128 %9, %13 offset:32\n\t"
      "ds_read_b128 %10, %14 offset:32\n\tds_read_b128 %11, %15 offset:32"
      : "=&v"(b0), "=&v"(d0), "=&v"(a0), "=&v"(c0), "=&v"(b1), "=&v"(d1), "=&v"(a1), "=&v"(c1), "=&v"(b2),
        "=&v"(d2), "=&v"(a2), "=&v"(c2)
      : "v"(xb), "v"(xd), "v"(xa), "v"(xc)
      : "memory");
  asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(b0), "+v"(d0), "+v"(a0), "+v"(c0));
  unpack4(B, 0, b0); unpack4(D, 0, d0); unpack4(A, 0, a0); unpack4(C, 0, c0);
  asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(b1), "+v"(d1), "+v"(a1), "+v"(c1));
  unpack4(B, 1, b1); unpack4(D, 1, d1); unpack4(A, 1, a1); unpack4(C, 1, c1);
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(b2), "+v"(d2), "+v"(a2), "+v"(c2));
  unpack4(B, 2, b2); unpack4(D, 2, d2); unpack4(A, 2, a2); unpack4(C, 2, c2);
  return;
#endif
#if defined(__HIP_DEVICE_COMPILE__)
  // LDS byte addresses (r06): bit 11 of a reference selects the constant table through a
  // sign-extended bit-field extract used as a bit-select mask (v_bfe_i32 + v_bfi_b32, where r05's
  // pointer select took and / compare / cndmask), the low 11 bits index 48-byte entries
  // (v_bfe_u32 + v_mad_u32_u24)
  // (the select is written as v_bfi_b32 in asm: as C the compiler turns it back into the VCC
  // compare + cndmask, whose VCC write-then-read also costs wait states)
  typedef const __attribute__((address_space(3))) u32x4* lds_q;
  const uint32_t sb = (uint32_t)(uintptr_t)(lds_cptr)slots, cb = (uint32_t)(uintptr_t)(lds_cptr)cst;
  auto addr = [&](uint32_t ref) -> lds_q {
    const uint32_t m = (uint32_t)__builtin_amdgcn_sbfe((int32_t)ref, 11, 1);
    uint32_t base;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(base) : "v"(m), "v"(cb), "v"(sb));
    return (lds_q)(uintptr_t)(__builtin_amdgcn_ubfe(ref, 0, 11) * 48u + base);
  };
  const lds_q pa = addr(ra), pb = addr(rb), pc = addr(rc), pd = addr(rd);
#else
  const uint4 *pa = slot_ptr(slots, cst, ra), *pb = slot_ptr(slots, cst, rb), *pc = slot_ptr(slots, cst, rc),
              *pd = slot_ptr(slots, cst, rd);
#endif
#pragma unroll
  for (int q = 0; q < 3; ++q) {
#if defined(__HIP_DEVICE_COMPILE__)
    const u32x4 b = pb[q], d = pd[q], a = pa[q], c = pc[q];
#else
    const uint4 b = pb[q], d = pd[q], a = pa[q], c = pc[q];
#endif
    B.v[4 * q] = b.x; B.v[4 * q + 1] = b.y; B.v[4 * q + 2] = b.z; B.v[4 * q + 3] = b.w;
    D.v[4 * q] = d.x; D.v[4 * q + 1] = d.y; D.v[4 * q + 2] = d.z; D.v[4 * q + 3] = d.w;
    A.v[4 * q] = a.x; A.v[4 * q + 1] = a.y; A.v[4 * q + 2] = a.z; A.v[4 * q + 3] = a.w;
    C.v[4 * q] = c.x; C.v[4 * q + 1] = c.y; C.v[4 * q + 2] = c.z; C.v[4 * q + 3] = c.w;
#if defined(__HIPCC__)
    __builtin_amdgcn_sched_barrier(0);  // keep the quarter order (the scheduler clusters by address)
#endif
  }
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

// 2p as 12 limbs (2p < 2^382)
constexpr uint32_t P2_LIMBS[12] = {
    P_LIMBS[0] << 1, (P_LIMBS[1] << 1) | (P_LIMBS[0] >> 31), (P_LIMBS[2] << 1) | (P_LIMBS[1] >> 31),
    (P_LIMBS[3] << 1) | (P_LIMBS[2] >> 31), (P_LIMBS[4] << 1) | (P_LIMBS[3] >> 31),
    (P_LIMBS[5] << 1) | (P_LIMBS[4] >> 31), (P_LIMBS[6] << 1) | (P_LIMBS[5] >> 31),
    (P_LIMBS[7] << 1) | (P_LIMBS[6] >> 31), (P_LIMBS[8] << 1) | (P_LIMBS[7] >> 31),
    (P_LIMBS[9] << 1) | (P_LIMBS[8] >> 31), (P_LIMBS[10] << 1) | (P_LIMBS[9] >> 31),
    (P_LIMBS[11] << 1) | (P_LIMBS[10] >> 31)};

// [0, 2p) -> [0, p): one conditional subtraction
VM_FN void canon(Fp& r, const Fp& a) {
  uint32_t d[12], br = 0;
#pragma unroll
  for (int j = 0; j < 12; ++j) d[j] = subc32(a.v[j], P_LIMBS[j], br, &br);
#pragma unroll
  for (int j = 0; j < 12; ++j) r.v[j] = br ? a.v[j] : d[j];
}

// NP = 2^384 - p: adding q NP is subtracting q p modulo 2^384 with a carry chain through
// 64-bit products (no borrow flags)
constexpr uint32_t NP_LIMBS[12] = {
    0u - P_LIMBS[0], ~P_LIMBS[1], ~P_LIMBS[2], ~P_LIMBS[3], ~P_LIMBS[4], ~P_LIMBS[5],
    ~P_LIMBS[6], ~P_LIMBS[7], ~P_LIMBS[8], ~P_LIMBS[9], ~P_LIMBS[10], ~P_LIMBS[11]};
static_assert(P_LIMBS[0] != 0, "NP_LIMBS: no borrow out of limb 0");

// f32 quotient estimate floor(x / p) for x = t 2^359 + (lower bits), t = x >> 359 < 2^30: with
// Pt = p >> 359, t / (Pt + 1) <= x / p < (t + 1) / Pt and x / p - t / (Pt + 1) < 1e-4 for
// x < 250 p; the quotient is shrunk by 2^-20 (the f32 roundings stay below it), so the result
// is floor(x / p) or one less.
VM_FN uint32_t quot_est(uint32_t t) {
  constexpr float QS = (float)((1.0 - 0x1p-20) / (double)((P_LIMBS[11] >> 7) + 1));
  return (uint32_t)((float)t * QS);
}

// r = k s - q p in [0, 2p) for s < 16p (13 limbs), 1 <= k <= 15: q = quot_est of k s, and
// k s + q NP modulo 2^384 as one carry chain of 64-bit products.
VM_FN void scale_reduce(Fp& r, const uint32_t* s, uint32_t k) {
  const uint32_t q = quot_est(k * (uint32_t)((((uint64_t)s[12] << 32) | s[11]) >> 7));
  uint64_t acc = 0;
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    acc = (uint64_t)k * s[j] + (acc >> 32);
    acc = (uint64_t)q * NP_LIMBS[j] + acc;
    r.v[j] = (uint32_t)acc;
  }
}

// 2p + 1 as 12 limbs (2p is even: no carry)
constexpr uint32_t P2P1_LIMBS[12] = {
    P2_LIMBS[0] + 1, P2_LIMBS[1], P2_LIMBS[2], P2_LIMBS[3], P2_LIMBS[4], P2_LIMBS[5],
    P2_LIMBS[6], P2_LIMBS[7], P2_LIMBS[8], P2_LIMBS[9], P2_LIMBS[10], P2_LIMBS[11]};

// r = sum_t c_t X_t mod p in [0, 2p) for four X_t < 2p and general |c_t| <= 15 (the final's
// Granger-Scott combinations 3t +- 2z) in one borrow-free pass of 64-bit products. (Unit sums
// take lin_sum: v_mad_u64_u32 issues slower than the add chains, measured r02l.)
// A negative term enters as |c| ~X (xor mask); the offset nw (2p + 1), nw = sum of the negative
// |c|, turns those into |c| (2p - X) plus nw 2^384, which the final reduction modulo 2^384
// drops: the true sum s' = sum |c_t| Y_t (Y_t = X_t or 2p - X_t) lies in [0, 120p). Each limb
// accumulates its column in 64 bits (< 2^38: no carries between terms); q = floor(s'/p) or one
// less from the top column (the carries into it from below are at most 2^10 units of 2^352,
// far inside quot_est's margin), then r = s' + q (2^384 - p) modulo 2^384 in one carry pass.
VM_FN void lin_mad(Fp& r, const Fp& A, const Fp& B, const Fp& C, const Fp& D, int ca, int cb, int cc, int cd) {
  const Fp* X[4] = {&A, &B, &C, &D};
  const int cf[4] = {ca, cb, cc, cd};
  uint64_t acc[12];
#pragma unroll
  for (int j = 0; j < 12; ++j) acc[j] = 0;
  uint32_t nw = 0;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const uint32_t a = cf[t] < 0 ? (uint32_t)(-cf[t]) : (uint32_t)cf[t];
    const uint32_t m = cf[t] < 0 ? ~0u : 0u;
    nw += a & m;
#pragma unroll
    for (int j = 0; j < 12; ++j) acc[j] = (uint64_t)a * (X[t]->v[j] ^ m) + acc[j];
  }
#pragma unroll
  for (int j = 0; j < 12; ++j) acc[j] = (uint64_t)nw * P2P1_LIMBS[j] + acc[j];
  const int64_t top = (int64_t)(acc[11] >> 7) - ((int64_t)nw << 25);  // s' >> 359, short by <= 8
  const uint32_t q = top > 0 ? quot_est((uint32_t)top) : 0u;
  uint64_t cy = 0;
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    const uint64_t v = (uint64_t)q * NP_LIMBS[j] + (acc[j] + cy);
    r.v[j] = (uint32_t)v;
    cy = v >> 32;
  }
}

// Product operands x = A + B, y = C + (ny ? 2p - D : D) in [0, 4p), no reduction. Only y is
// ever negated: the encoder puts a product's negated operand on y (tools/fpvm/sched.py
// lane_operands; no program negates both), so the negation's borrow chain runs once, and only
// when some lane of the wave has one (`any_neg`, r06: 77 -> 53 VALU in the 1,062 of the vote
// program's 1,375 product phases that have one). Both paths write x, y in full (no register
// copies at the join). The carry chains are skewed by one limb so no chain reads its carry
// right after writing it (gfx950 wait states).
VM_FN void pre_add2(Fp& x, const Fp& A, const Fp& B, Fp& y, const Fp& C, const Fp& D, bool ny, bool any_neg) {
  uint32_t c1 = 0, c2 = 0;
  if (any_neg) {
    uint32_t nd[12], b2 = 0;
#pragma unroll
    for (int j = 0; j < 13; ++j) {
      if (j < 12) {
        nd[j] = subc32(P2_LIMBS[j], D.v[j], b2, &b2);
        x.v[j] = addc32(A.v[j], B.v[j], c1, &c1);
      }
      if (j >= 1) y.v[j - 1] = addc32(C.v[j - 1], ny ? nd[j - 1] : D.v[j - 1], c2, &c2);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      x.v[j] = addc32(A.v[j], B.v[j], c1, &c1);
      y.v[j] = addc32(C.v[j], D.v[j], c2, &c2);
    }
  }
}

// phase header bits (w0 bits 22..31, tools/fpvm/sched.py H_*)
constexpr uint32_t H_MUL = 1u << 22, H_MULNEG = 1u << 23, H_FLAG = 1u << 24, H_LIN = 1u << 25,
                   H_LINNEG = 1u << 26, H_ACC = 1u << 27, H_RARE = 1u << 28, H_SELB = 1u << 29,
                   H_LINNEG2 = 1u << 30, H_LINNEG3 = 1u << 31;
constexpr uint32_t H_ANY = H_MUL | H_LIN | H_ACC | H_RARE;

// The negated-sum chain of lin_sum: XB / XC XOR B / C with their masks (D always): a unit sum's
// negated terms sit in the last positions (tools/fpvm/sched.py lane_operands), so the phase
// header (H_LINNEG2: some lane negates C, H_LINNEG3: B) skips the XORs no lane needs.
template <bool XB, bool XC>
VM_FN void lin_chain_neg(uint32_t* s, const Fp& A, const Fp& B, const Fp& C, const Fp& D, uint32_t mb, uint32_t mc,
                         uint32_t md, const Fp& K) {
  uint32_t u[12], v[12], w[12], c1 = 0, c2 = 0, c3 = 0, c4 = 0;
#pragma unroll
  for (int j = 0; j < 14; ++j) {
    if (j < 12) {
      u[j] = addc32(A.v[j], XB ? B.v[j] ^ mb : B.v[j], c1, &c1);
      v[j] = addc32(XC ? C.v[j] ^ mc : C.v[j], D.v[j] ^ md, c2, &c2);
    }
    if (j >= 1 && j <= 12) w[j - 1] = addc32(u[j - 1], v[j - 1], c3, &c3);
    if (j >= 2) s[j - 2] = addc32(w[j - 2], K.v[j - 2], c4, &c4);
  }
}

// s = A + sb B + sc C + sd D with unit signs (a zero coefficient points its operand at the zero
// constant), s < 8p in 12 limbs: a negated term enters as ~X (mb, mc, md: all-ones masks of the
// negated terms; a unit sum's first term is never negated, ir._expand_unit) and the offset
// K = n (2p + 1) (n negated terms, constant-table entry KTAB + n) turns each ~X into 2p - X
// modulo 2^384. Four carry chains (A + B', C' + D', their sum, + K) skewed by one limb each.
VM_FN void lin_sum(uint32_t* s, const Fp& A, const Fp& B, const Fp& C, const Fp& D, uint32_t mb, uint32_t mc,
                   uint32_t md, uint32_t hdr, const uint32_t* __restrict__ cst) {
  if (hdr & H_LINNEG) {
    const uint32_t n = (mb & 1u) + (mc & 1u) + (md & 1u);
    Fp K;
    ld_slot(K, nullptr, cst, CONST_BASE + KTAB + n);
    if (hdr & H_LINNEG3) {
      lin_chain_neg<true, true>(s, A, B, C, D, mb, mc, md, K);
    } else if (hdr & H_LINNEG2) {
#if defined(__HIP_DEVICE_COMPILE__)
      __asm__ volatile("");  // (kept branches: three chains, never selects between them)
#endif
      lin_chain_neg<false, true>(s, A, B, C, D, mb, mc, md, K);
    } else {
#if defined(__HIP_DEVICE_COMPILE__)
      __asm__ volatile("");
#endif
      lin_chain_neg<false, false>(s, A, B, C, D, mb, mc, md, K);
    }
  } else {
    uint32_t u[12], v[12], c1 = 0, c2 = 0, c3 = 0;
#pragma unroll
    for (int j = 0; j < 13; ++j) {
      if (j < 12) {
        u[j] = addc32(A.v[j], B.v[j], c1, &c1);
        v[j] = addc32(C.v[j], D.v[j], c2, &c2);
      }
      if (j >= 1) s[j - 1] = addc32(u[j - 1], v[j - 1], c3, &c3);
    }
  }
  s[12] = 0;
}

// Modular inverse of a Montgomery value (op inv, final program only): bls/fp.hpp fp_inv_divsteps
// (Bernstein-Yang divsteps), then back to Montgomery form with one product by raw R^3 (r3, a
// constant-table entry). 0 -> 0. `a` must be canonical.
VM_FN void fp_inv(Fp& r, const Fp& a, const Fp& r3) { fp_inv_divsteps(r, a, r3); }

#if defined(__HIPCC__)
// the header is the same in every lane: read it once into an SGPR
VM_FN uint32_t uniform(uint32_t w0) { return __builtin_amdgcn_readfirstlane(w0); }
#else
// host emulation runs one lane at a time with the phase's header: a block runs for every lane
// when any lane of the phase needs it, as on the device
inline uint32_t uniform(uint32_t w0) { return w0; }
#endif

// One phase of one lane. `in` = (w0, A|B<<16, C|D<<16, coefficients). The common ops run behind
// wave-uniform branches (a block runs when any lane of the wave needs it) and each lane stores
// the result of its own op:
//   products  x = A + cb B, y = C + cd D (unit signs), m = x y: muls; sgn0 / lex / eq take the
//             from-Montgomery product (y = plain 1; eq: x = A - B) and flag its canonical value;
//   linear    lin_mad: k (A + cb B + cc C + cd D) with unit signs, or general coefficients
//             |c| <= 15, and selb (bit imm of the vote's scalar ? C : B);
//   rare      sel, logic, st, inv (per-lane branches).
// The sign of the 5-bit two's-complement coefficient field whose top bit is `bit` of w3, as a
// mask (a bit-field extract on the device)
VM_FN uint32_t sign_mask(uint32_t w, int bit) { return (uint32_t)((int32_t)(w << (31 - bit)) >> 31); }
VM_FN int coef5(uint32_t w, int lo) { return ((int)(w << (27 - lo))) >> 27; }

// r06: only what every phase needs is decoded up front (the header, the opcode, the four operand
// addresses); each block extracts its own fields (dst, coefficient signs, scale, imm), so a
// product phase no longer pays for the linear blocks' decoding (r05: 10 VALU per phase).
VM_FN void exec(const uint4 in, bool active, uint32_t* __restrict__ slots, const uint32_t* __restrict__ cst,
                uint64_t scalar, const Out& out) {
  // the phase header (bits 22.. of w0, equal in every lane; tools/fpvm/sched.py phase_bits) names
  // the blocks some lane of the phase needs: scalar branches, no ballots
  const uint32_t hdr = uniform(in.x);
  if (!(hdr & H_ANY)) return;
  const uint32_t op = active ? (in.x & 31) : (uint32_t)OP_NOP;
  // four operands, always valid references (a missing one is the zero constant); selb (bit imm
  // of the vote's scalar ? C : B) is a one-term unit lin: A := the picked operand, B = C = 0
  // (its encoded coefficients and scale are 0: tools/fpvm/sched.py lane_operands)
  uint32_t ra = in.y & 0xFFFF, rb = in.y >> 16, rc = in.z & 0xFFFF;
  bool selb = false;
  if (hdr & H_SELB) {
#if defined(__HIP_DEVICE_COMPILE__)
    // (kept a branch: if-converted, these selects ran in every phase, r06 ISA)
    __asm__ volatile("");
#endif
    selb = op == OP_SELB;
    const bool bit = ((scalar >> ((in.x >> 16) & 63)) & 1) != 0;
    ra = selb ? (bit ? rc : rb) : ra;
    rb = selb ? CONST_BASE + KZERO : rb;
    rc = selb ? CONST_BASE + KZERO : rc;
  }
  Fp A, B, C, D;
  ld_slots4(A, B, C, D, slots, cst, ra, rb, rc, in.z >> 16);
  const uint32_t dst = (in.x >> 5) & 0x7FF;
  // A phase's lin ops all run in one block (tools/fpvm/sched.py encode, PHASE_UNIT, asserted):
  // the unit-sum block, or every lin op in the general block with FORCE_ACC (w3 bit 24) set. So
  // a lane's block is that bit (r05 re-derived it from the coefficients in every phase); selb
  // ops run in the unit block
  const bool force_acc = (in.w & (1u << 24)) != 0;
  if (hdr & H_MUL) {
    const bool is_mul = op == OP_MULS || op == OP_SGN0 || op == OP_LEX || op == OP_EQ;
    Fp x, y, m;
    pre_add2(x, A, B, y, C, D, sign_mask(in.w, 19) != 0, (hdr & H_MULNEG) != 0);
    fp_mul(m, x, y);
    if (hdr & H_FLAG) {  // m is canonical here: the product of a value below 4p and the plain 1
      const bool flag = is_mul && op != OP_MULS;
      uint32_t f = 0;
      if (op == OP_SGN0) f = m.v[0] & 1u;
      if (op == OP_LEX) f = limbs_gt(m.v, HALF_P) ? 1u : 0u;
      if (op == OP_EQ) f = fp_is_zero(m) ? 1u : 0u;
#pragma unroll
      for (int j = 0; j < 12; ++j) m.v[j] = flag ? (j == 0 ? f : 0u) : m.v[j];
    }
    if (is_mul) st_slot(slots, dst, m);
  }
  if (hdr & H_LIN) {
    uint32_t s[13];
    lin_sum(s, A, B, C, D, sign_mask(in.w, 9), sign_mask(in.w, 14), sign_mask(in.w, 19), hdr, cst);
    // "scaled" form k * (unit sum), k < 16 (k <= 1: unchanged; selb: 0)
    const uint32_t k = (in.w >> 20) & 15;
    Fp l;
    scale_reduce(l, s, k > 1 ? k : 1u);
    if ((op == OP_LIN && !force_acc) || selb) st_slot(slots, dst, l);
  }
  if (hdr & H_ACC) {  // general coefficients
    Fp l;
    lin_mad(l, A, B, C, D, coef5(in.w, 0), coef5(in.w, 5), coef5(in.w, 10), coef5(in.w, 15));
    if (op == OP_LIN && force_acc) st_slot(slots, dst, l);
  }
  if (hdr & H_RARE) {
    const bool rare = op != OP_NOP && op != OP_LIN && !selb && op != OP_MULS && op != OP_SGN0 && op != OP_LEX &&
                      op != OP_EQ;
    const uint32_t imm = (in.x >> 16) & 63;
    Fp z = A;
    if (op == OP_ST) {
      canon(z, A);
      uint32_t* b = out.base + (size_t)imm * 12 * out.cap + out.unit;
#pragma unroll
      for (int k = 0; k < 12; ++k) b[(size_t)k * out.cap] = z.v[k];
    } else if (op == OP_SEL) {
      z = A.v[0] ? C : B;
    } else if (op >= OP_AND && op <= OP_XOR) {
      set_flag(z, op == OP_AND ? (A.v[0] & C.v[0]) : op == OP_OR ? (A.v[0] | C.v[0]) : (A.v[0] ^ C.v[0]));
    } else if (op == OP_INV) {
#ifndef OVH_VM_NO_INV
      Fp a;
      canon(a, A);
      fp_inv(z, a, C);
#endif
    }
    if (rare && op != OP_ST) st_slot(slots, dst, z);
  }
#if defined(__HIP_DEVICE_COMPILE__)
  // Every path of the phase retires its operand reads here (free on the paths that consumed
  // them). Left pending on some path, they merged into the loop head's wait-count state, and
  // the next phase's first write of a register one of them had loaded (an operand address) got
  // an lgkmcnt(0): a wait for this phase's result stores before the next phase could issue its
  // reads (r06 ISA). LDS operations complete in order, so the last quarter of each operand
  // covers all twelve reads.
  __asm__ volatile("" ::"v"(A.v[11]), "v"(B.v[11]), "v"(C.v[11]), "v"(D.v[11]));
#endif
}

// Run `nphases` phases of a W-lane program (the code is phase-major: lane l of phase t at
// index t W + l). Every lane of the workgroup must call this; lanes of inactive slices pass
// active = false. The VM kernels are single-wave workgroups, so no phase barrier is needed: a
// wave's LDS operations are performed in issue order, and a slot a phase writes is read from the
// next phase on (tools/fpvm/sched.py), so the next phase's loads may issue while this phase's
// stores are still in flight.
#if defined(__HIPCC__)
// Side words (programs scheduled with spills, tools/fpvm/sched.py spill_pass): one uint32 per
// lane per phase, bit 31 valid, bit 30 fill (else spill), bits 0..10 the slot, bits 11..22 the
// scratch entry (12 words at scr + 12 entry, the unit's own scratch). A spill stores its slot
// after the phase's op; a fill's load is issued at the start of the phase before its own (the
// previous iteration reads the next phase's side word) and written to its slot after that
// phase's op and spills -- so the slot is valid from its phase on, and one phase hides the
// load. Fills
// read through `nt` loads (L2-served, never a stale L1 line); a spill's store precedes any fill
// of its entry by >= 2 phases (spill_pass gap).
constexpr uint32_t SIDE_VALID = 1u << 31, SIDE_FILL = 1u << 30;

__device__ __forceinline__ void side_spill(uint32_t sw, uint32_t* __restrict__ slots, uint32_t* __restrict__ scr) {
  if ((sw & (SIDE_VALID | SIDE_FILL)) == SIDE_VALID) {
    const u32x4* s = reinterpret_cast<const u32x4*>(slots + (sw & 0x7FF) * 12);
    const u32x4 a = s[0], b = s[1], c = s[2];
    u32x4* d = reinterpret_cast<u32x4*>(scr + ((sw >> 11) & 0xFFF) * 12);
    d[0] = a;
    d[1] = b;
    d[2] = c;
  }
}

template <bool SIDE = false>
__device__ __forceinline__ void run(const uint4* __restrict__ code, uint32_t nphases, uint32_t W, uint32_t lane,
                                    bool active, uint32_t* __restrict__ slots, const uint32_t* __restrict__ cst,
                                    uint64_t scalar, const Out& out, uint64_t* __restrict__ trace = nullptr,
                                    const uint32_t* __restrict__ side = nullptr, uint32_t* __restrict__ scr = nullptr) {
  static_assert(PREFETCH >= 5, "the unrolled loops below read up to 4 phases past the end");
  if constexpr (SIDE) {
    // r06: the loop is unrolled three times over three-register rings. At the start of phase ph
    // the words of phase ph + 2 load into the registers that held phase ph - 1's (no register
    // copies: r05's four-deep rings rotated 12 VALU per phase, and the copy of the newest load
    // waited for it inside the same phase). The loads of a phase are issued at its start (the
    // next phase's fill first), so whatever the compiler waits for at the next phase's start has
    // had a whole phase. A partial last round runs up to two of the code's trailing NOP phases
    // (no ops, zero side words).
    uint4 qa = code[lane], qb = code[W + lane], qc;
    uint32_t sa = side[lane], sb = side[W + lane], sc;
    // inactive lanes (a slice past the batch's end) run no side op: their unit has no scratch
    if (!active) sa = sb = 0;
    // the first words complete before the loop: the compiler loads them straight into the loop's
    // registers, and its wait-count state merged at the loop head then made every phase wait for
    // its own fresh prefetch (r06 ISA)
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    // phase ph: instruction q, side word s, the next phase's side word sn (its fill is issued
    // now); q2 / s2 take phase ph + 2's words
    auto step = [&](const uint4& q, uint4& q2, const uint32_t s, const uint32_t sn, uint32_t& s2,
                    const uint32_t ph) __attribute__((always_inline)) {
      const bool fill = (sn & (SIDE_VALID | SIDE_FILL)) == (SIDE_VALID | SIDE_FILL);
      u32x4 f0, f1, f2;
      if (fill) {
        const u32x4* src = reinterpret_cast<const u32x4*>(scr + ((sn >> 11) & 0xFFF) * 12);
        f0 = __builtin_nontemporal_load(src);
        f1 = __builtin_nontemporal_load(src + 1);
        f2 = __builtin_nontemporal_load(src + 2);
      }
      q2 = code[(size_t)(ph + 2) * W + lane];
      s2 = active ? side[(size_t)(ph + 2) * W + lane] : 0u;
      exec(q, active, slots, cst, scalar, out);
      // this phase's spill reads its slot before the fill lands: a fill may take the slot of a
      // value whose last read is this spill
      side_spill(s, slots, scr);
      if (fill) {
        u32x4* d = reinterpret_cast<u32x4*>(slots + (sn & 0x7FF) * 12);
        d[0] = f0;
        d[1] = f1;
        d[2] = f2;
      }
    };
#pragma unroll 1
    for (uint32_t ph = 0; ph < nphases; ph += 3) {
      step(qa, qc, sa, sb, sc, ph);
      step(qb, qa, sb, sc, sa, ph + 1);
      step(qc, qb, sc, sa, sb, ph + 2);
    }
    __asm__ volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    return;
  }
  // trace (diagnostics, OVH_FLAG_VM_TRACE): wall clock after every phase
  if (trace && threadIdx.x == 0) trace[0] = wall_clock64();
  // unrolled three times over a three-register ring, phase ph + 2's words loaded at the start of
  // phase ph (as the side-word loop above); a partial last round runs trailing NOP phases
  uint4 qa = code[lane], qb = code[W + lane], qc;
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), as above
  auto step = [&](const uint4& q, uint4& q2, const uint32_t ph) __attribute__((always_inline)) {
    q2 = code[(size_t)(ph + 2) * W + lane];
    exec(q, active, slots, cst, scalar, out);
    if (trace && ph < nphases) {
      __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (threadIdx.x == 0) trace[ph + 1] = wall_clock64();
    }
  };
#pragma unroll 1
  for (uint32_t ph = 0; ph < nphases; ph += 3) {
    step(qa, qc, ph);
    step(qb, qa, ph + 1);
    step(qc, qb, ph + 2);
  }
  // the caller reads results through LDS (other lanes' slots) and may reuse it
  __asm__ volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

#endif  // __HIPCC__

}  // namespace vm
}  // namespace ovh
