// libovhip: HIP (gfx950) implementation of the C ABI in include/ovhip.h.
//
// Batch verification (ovh_verify_batch_device), DESIGN.md section 4:
//   k_h2f         lane per vote: expand_message_xmd (SHA-256) + hash_to_field -> u0, u1
//   k_vm_vote     16-lane slice per vote, 4 votes per wave: the Fp-VM "vote" program --
//                 pk / sig decompression + subgroup checks, hash_to_G2, r pk, r sigma,
//                 f = Miller(r pk, H); the epilogue writes the vote's code with the reference
//                 precedence and its (f, r sigma) contribution (identity if the vote failed)
//   k_vm_fold     16-lane slice per 4 partials: (prod f, sum S), repeated down to <= 4
//   k_vm_final    one wave: prod f * Miller(-G1, sum S) -> final exponentiation == 1 ?
//   k_vm_pairchk  16-lane slice per surviving vote when the combined check fails
// Per-vote state lives in HBM as structure-of-arrays by limb: limb k of element i of an Fp
// plane j at slab[(j * 12 + k) * cap + i].
#include <hip/hip_runtime.h>

#include <mutex>
#include <new>
#include <string.h>
#include <vector>

#include "../../include/ovhip.h"
#include "bls/verify.hpp"
#include "fpvm.hpp"
#include "sm3.hpp"
#include "vm_progs.inc"

using namespace ovh;

#define WG 64  // one wave per workgroup: spreads lane-per-vote work over all CUs

// ------------------------------------------------------------------------ SoA helpers
struct Slab {
  uint32_t* p;
  uint32_t cap;
  __device__ __forceinline__ void ld(Fp& a, uint32_t j, uint32_t i) const {
    const uint32_t* b = p + (size_t)j * 12 * cap + i;
#pragma unroll
    for (int k = 0; k < 12; ++k) a.v[k] = b[(size_t)k * cap];
  }
  __device__ __forceinline__ void st(const Fp& a, uint32_t j, uint32_t i) const {
    uint32_t* b = p + (size_t)j * 12 * cap + i;
#pragma unroll
    for (int k = 0; k < 12; ++k) b[(size_t)k * cap] = a.v[k];
  }
  __device__ void ld2(Fp2& a, uint32_t j, uint32_t i) const {
    ld(a.c0, j, i);
    ld(a.c1, j + 1, i);
  }
  __device__ void st2(const Fp2& a, uint32_t j, uint32_t i) const {
    st(a.c0, j, i);
    st(a.c1, j + 1, i);
  }
  __device__ void ld_g2j(G2J& a, uint32_t i) const {
    ld2(a.X, 0, i);
    ld2(a.Y, 2, i);
    ld2(a.Z, 4, i);
  }
  __device__ void st_g2j(const G2J& a, uint32_t i) const {
    st2(a.X, 0, i);
    st2(a.Y, 2, i);
    st2(a.Z, 4, i);
  }
  __device__ void ld_g2a(G2A& a, uint32_t i) const {
    ld2(a.x, 0, i);
    ld2(a.y, 2, i);
  }
  __device__ void st_g2a(const G2A& a, uint32_t i) const {
    st2(a.x, 0, i);
    st2(a.y, 2, i);
  }
  __device__ void ld_g1a(G1A& a, uint32_t i) const {
    ld(a.x, 0, i);
    ld(a.y, 1, i);
  }
  __device__ void st_g1a(const G1A& a, uint32_t i) const {
    st(a.x, 0, i);
    st(a.y, 1, i);
  }
  __device__ void ld_f12(Fp12& f, uint32_t i) const {
    Fp* c = &f.c0.c0.c0;
    for (int j = 0; j < 12; ++j) ld(c[j], j, i);
  }
  __device__ void st_f12(const Fp12& f, uint32_t i) const {
    const Fp* c = &f.c0.c0.c0;
    for (int j = 0; j < 12; ++j) st(c[j], j, i);
  }
};

// Fp planes of the per-vote state slab.
enum : uint32_t {
  S_U = VM_S_U,       // 4 planes: u0, u1 (hash_to_field, Montgomery)
  S_FB = VM_S_FB,     // 12 planes: pk affine (2), sig affine (4), H projective (6) -- fallback inputs
  S_RS = VM_S_RS,     // 6 planes: r * sig (projective)
  S_F = VM_S_F,       // 12 planes: f = Miller(r pk, H)
  S_TOTAL = VM_S_TOTAL,
};
// partial = (F: 12 planes, S: 6 planes)
constexpr uint32_t PART_PLANES = 18;
// words per fin region: 16 unpacked + 4 folded partials as planes
constexpr size_t FIN_STRIDE = (size_t)PART_PLANES * 12 * 20;

enum : int { ST_H2F = 0, ST_VOTE, ST_FOLD, ST_FINAL, ST_FALLBACK };
static_assert(ST_FALLBACK + 1 == OVH_NSTAGES, "stage table");

__device__ __forceinline__ uint64_t rlc_scalar(uint64_t seed, uint32_t i) {
  // SplitMix64 on (seed, i): the 64-bit RLC coefficient of vote i (never 0).
  uint64_t z = seed + 0x9e3779b97f4a7c15ull * ((uint64_t)i + 1);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  z = z ^ (z >> 31);
  return z ? z : 1;
}

// ------------------------------------------------------------------------ kernels
__global__ __launch_bounds__(WG) void k_h2f(uint32_t n, const uint8_t* __restrict__ hashes, XmdTemplates t, Slab s) {
  const uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  uint32_t msg[8], uni[64];
  be_words_from_bytes(msg, hashes + (size_t)i * 32, 8);
  expand_message_xmd_256(uni, msg, t);
  Fp2 u0, u1;
  hash_to_field_fp2x2(u0, u1, uni);
  s.st2(u0, S_U, i);
  s.st2(u1, S_U + 2, i);
}

// ZCash header of a compressed point without decompression (the VM program decompresses):
// bad = BAD_ENCODING, inf = valid infinity encoding, x = masked plain limbs (x1 for G2).
__device__ void parse_hdr(const uint8_t* b, uint32_t nbytes, uint32_t* x_hi, uint32_t* x_lo, uint32_t& bad,
                          uint32_t& inf, uint32_t& sort, uint32_t& xzero) {
  const uint8_t b0 = b[0];
  bad = 0;
  inf = 0;
  sort = (b0 >> 5) & 1u;
  xzero = 0;
  uint8_t t[48];
  for (int i = 0; i < 48; ++i) t[i] = b[i];
  t[0] &= 0x1f;
  limbs_from_be48(x_hi, t);
  if (nbytes == 96) limbs_from_be48(x_lo, b + 48);
  if (!(b0 & 0x80)) {
    bad = 1;
    return;
  }
  if (b0 & 0x40) {
    uint32_t acc = b0 & 0x3f;
    for (uint32_t i = 1; i < nbytes; ++i) acc |= b[i];
    if (acc) bad = 1;
    else inf = 1;
    return;
  }
  if (!limbs_lt_p(x_hi)) bad = 1;
  if (nbytes == 96 && !limbs_lt_p(x_lo)) bad = 1;
  uint32_t z = 0;
  for (int k = 0; k < 12; ++k) z |= x_hi[k] | (nbytes == 96 ? x_lo[k] : 0u);
  xzero = z == 0;
}

struct VmDev {  // a program in device memory
  const uint4* code;
  uint32_t nphases;
  const uint16_t* in;   // device copies of the slot maps
  const uint16_t* out;
  uint64_t* trace;  // OVH_FLAG_VM_TRACE: nphases + 1 timestamps of workgroup 0, else null
};

#define VM_SLICES 4  // 16-lane slices per 64-lane workgroup (vote, pairchk)
#define VM_FOLD_UNITS (64 / VM_FOLD_W)  // fold units per 64-lane workgroup

__device__ __forceinline__ void load_consts(uint32_t* cst, const uint32_t* __restrict__ g, uint32_t n) {
  for (uint32_t k = threadIdx.x; k < n * 12; k += blockDim.x) cst[k] = g[k];
}

__device__ __forceinline__ void slot_flag(uint32_t* slots, uint32_t s, uint32_t f) {
  uint4* d = reinterpret_cast<uint4*>(slots + s * 12);
  d[0] = make_uint4(f, 0, 0, 0);
  d[1] = make_uint4(0, 0, 0, 0);
  d[2] = make_uint4(0, 0, 0, 0);
}

__device__ __forceinline__ void slot_put(uint32_t* slots, uint32_t s, const uint32_t* v) {
  for (int k = 0; k < 12; ++k) slots[s * 12 + k] = v[k];
}

__device__ __forceinline__ uint32_t slot_flag_get(const uint32_t* slots, uint32_t s) { return slots[s * 12]; }

// One fold unit on a 16-lane slice: out[t] = (prod F, sum S) over in[4t .. 4t+3] (missing ->
// identity); with codes (level 0) every vote whose code is not 0 contributes the identity.
// All 64 threads of the workgroup call it (the phase barrier); `active` marks the working slice.
__device__ __forceinline__ void fold_unit(uint32_t t, uint32_t m, const VmDev& prog, const uint32_t* cst,
                                          uint32_t* slots, uint32_t lane, bool active, Slab inF, Slab inS,
                                          Slab out, const int32_t* __restrict__ codes) {
  if (active) {
    for (uint32_t k = lane; k < 4 * PART_PLANES; k += VM_FOLD_W) {
      const uint32_t q = k / PART_PLANES, j = k % PART_PLANES, e = 4 * t + q;
      Fp v;
      if (e < m && (!codes || codes[e] == 0)) {
        if (j < 12) inF.ld(v, j, e);
        else inS.ld(v, j - 12, e);
      } else if (j == 0 || j == 12 + 2) {
        fp_one(v);
      } else {
        fp_zero(v);
      }
      slot_put(slots, VM_FOLD_IN[k], v.v);
    }
  }
  __syncthreads();
  vm::run(prog.code, VM_FOLD_NPHASES, VM_FOLD_W, lane, active, slots, cst, 0, vm::Out{nullptr, 0, 0});
  if (active) {
    for (uint32_t k = lane; k < PART_PLANES; k += VM_FOLD_W) {
      Fp v;
      const uint32_t src = VM_FOLD_OUT[k];
      for (int q = 0; q < 12; ++q) v.v[q] = slots[src * 12 + q];
      out.st(v, k, t);
    }
  }
}

// Per vote: VM "vote" program + reference-precedence code + the vote's (f, r sigma)
// contribution. LDS: constants, then VM_SLICES x (VM_VOTE_NSLOTS slots).
__global__ __launch_bounds__(64) void k_vm_vote(uint32_t n, VmDev prog, VmDev fold, const uint32_t* __restrict__ cst_g,
                                                const uint8_t* __restrict__ pks, const uint8_t* __restrict__ sigs,
                                                Slab s, uint64_t seed, int32_t* __restrict__ codes, Slab part0) {
  __builtin_amdgcn_s_setprio(2);  // per-vote stages outrank a co-resident final-stream wave
  extern __shared__ uint4 lds4[];
  uint32_t* lds = reinterpret_cast<uint32_t*>(lds4);
  uint32_t* cst = lds;
  const uint32_t slice = threadIdx.x / VM_VOTE_W, lane = threadIdx.x % VM_VOTE_W;
  uint32_t* slots = lds + VM_NCONST * 12 + slice * (VM_VOTE_NSLOTS * 12 + 4);
  uint32_t* hdr = slots + VM_VOTE_NSLOTS * 12;  // [pflags, code]
  const uint32_t i = blockIdx.x * VM_SLICES + slice;
  const bool active = i < n;
  load_consts(cst, cst_g, VM_NCONST);
  if (active) {
    if (lane == 0) {
      uint32_t x[12], bad, inf, sort, xz;
      parse_hdr(pks + (size_t)i * 48, 48, x, x, bad, inf, sort, xz);
      slot_put(slots, VM_VOTE_IN[VM_VOTE_IN_PK_X], x);
      slot_flag(slots, VM_VOTE_IN[VM_VOTE_IN_PK_SORT], sort);
      hdr[0] = bad | inf << 1 | xz << 2;
    }
  }
  __syncthreads();
  if (active) {
    if (lane == 1) {
      uint32_t x1[12], x0[12], bad, inf, sort, xz;
      parse_hdr(sigs + (size_t)i * 96, 96, x1, x0, bad, inf, sort, xz);
      slot_put(slots, VM_VOTE_IN[VM_VOTE_IN_SIG_X1], x1);
      slot_put(slots, VM_VOTE_IN[VM_VOTE_IN_SIG_X0], x0);
      slot_flag(slots, VM_VOTE_IN[VM_VOTE_IN_SIG_SORT], sort);
      hdr[0] |= (bad | inf << 1 | xz << 2) << 8;
    } else if (lane >= 2 && lane < 6) {
      Fp u;
      s.ld(u, S_U + (lane - 2), i);
      slot_put(slots, VM_VOTE_IN[VM_VOTE_IN_U00 + (lane - 2)], u.v);
    }
  }
  __syncthreads();
  vm::run(prog.code, VM_VOTE_NPHASES, VM_VOTE_W, lane, active, slots, cst, rlc_scalar(seed, i),
          vm::Out{s.p, s.cap, i},
          blockIdx.x == 0 ? prog.trace : nullptr);
  if (active && lane == 0) {
    const uint32_t pf = hdr[0];
    const uint32_t pk_bad = pf & 1, pk_inf = (pf >> 1) & 1, pk_xz = (pf >> 2) & 1;
    const uint32_t sg_bad = (pf >> 8) & 1, sg_inf = (pf >> 9) & 1, sg_xz = (pf >> 10) & 1;
    const uint32_t pk_ok = slot_flag_get(slots, VM_VOTE_OUT[VM_VOTE_OUT_PK_OK]);
    const uint32_t pk_grp = slot_flag_get(slots, VM_VOTE_OUT[VM_VOTE_OUT_PK_GRP]);
    const uint32_t sg_ok = slot_flag_get(slots, VM_VOTE_OUT[VM_VOTE_OUT_SIG_OK]);
    const uint32_t sg_grp = slot_flag_get(slots, VM_VOTE_OUT[VM_VOTE_OUT_SIG_GRP]);
    const uint32_t h_inf = slot_flag_get(slots, VM_VOTE_OUT[VM_VOTE_OUT_H_INF]);
    // consensus.rs:397-416: pk parse (102) > sig parse (1..3) > [core_verify] sig group (3) >
    // pk infinity (6) > pk group (3) > H(m) = O or sig = O (5) > pairing (batch)
    int32_t c;
    if (pk_bad || (!pk_inf && (!pk_ok || pk_xz))) c = OVH_ERR_PUBKEY;
    else if (sg_bad) c = BLST_BAD_ENCODING;
    else if (!sg_inf && !sg_ok) c = BLST_POINT_NOT_ON_CURVE;
    else if (!sg_inf && (sg_xz || !sg_grp)) c = BLST_POINT_NOT_IN_GROUP;
    else if (pk_inf) c = BLST_PK_IS_INFINITY;
    else if (!pk_grp) c = BLST_POINT_NOT_IN_GROUP;
    else if (h_inf || sg_inf) c = BLST_VERIFY_FAIL;
    else c = 0;
    codes[i] = c;
  }
  // fold level 0, fused: this workgroup's 4 votes -> partial blockIdx.x of part0 (F planes
  // 0..11, S planes 12..17), the identity for failed votes. The slices' `st` outputs (HBM)
  // and codes are made visible to the workgroup first; the fold reuses the vote slots' LDS.
  __threadfence();
  __syncthreads();
  fold_unit(blockIdx.x, n, fold, cst, lds + VM_NCONST * 12, threadIdx.x % VM_FOLD_W,
            threadIdx.x < VM_FOLD_W && 4 * blockIdx.x < n,
            Slab{s.p + (size_t)S_F * 12 * s.cap, s.cap}, Slab{s.p + (size_t)S_RS * 12 * s.cap, s.cap}, part0,
            codes);
}

// Fold level: SLICES units per 64-thread workgroup (4 on the main stream; 1 on the final
// stream, whose 10.8 KB of LDS fits beside a CU's four vote workgroups).
template <int SLICES>
__global__ __launch_bounds__(64) void k_vm_fold(uint32_t m, VmDev prog, const uint32_t* __restrict__ cst_g, Slab inF,
                                                Slab inS, Slab out, const int32_t* __restrict__ codes) {
  __builtin_amdgcn_s_setprio(2);  // short: run ahead of a co-resident final wave
  extern __shared__ uint4 lds4[];
  uint32_t* lds = reinterpret_cast<uint32_t*>(lds4);
  uint32_t* cst = lds;
  const uint32_t slice = threadIdx.x / VM_FOLD_W, lane = threadIdx.x % VM_FOLD_W;
  const uint32_t sl = slice < SLICES ? slice : 0;  // idle slices address slice 0 (never write)
  uint32_t* slots = lds + VM_NCONST * 12 + sl * VM_FOLD_NSLOTS * 12;
  const uint32_t t = blockIdx.x * SLICES + slice;
  const bool active = slice < SLICES && 4 * t < m;
  load_consts(cst, cst_g, VM_NCONST);
  fold_unit(t, m, prog, cst, slots, lane, active, inF, inS, out, codes);
}

// Final: prod F * Miller(-G1, sum S) over in[0..m-1] (m <= 4) -> FE == 1 -> *result.
__global__ __launch_bounds__(64) void k_vm_final(uint32_t m, VmDev prog, const uint32_t* __restrict__ cst_g, Slab inF,
                                                 Slab inS, int32_t* __restrict__ result) {
  extern __shared__ uint4 lds4[];
  uint32_t* lds = reinterpret_cast<uint32_t*>(lds4);
  uint32_t* cst = lds;
  uint32_t* slots = lds + VM_NCONST * 12;
  const uint32_t lane = threadIdx.x;
  load_consts(cst, cst_g, VM_NCONST);
  for (uint32_t k = lane; k < 4 * PART_PLANES; k += 64) {
    const uint32_t q = k / PART_PLANES, j = k % PART_PLANES;
    Fp v;
    if (q < m) {
      if (j < 12) inF.ld(v, j, q);
      else inS.ld(v, j - 12, q);
    } else if (j == 0 || j == 12 + 2) {
      fp_one(v);
    } else {
      fp_zero(v);
    }
    slot_put(slots, VM_FINAL_IN[k], v.v);
  }
  __syncthreads();
  vm::run(prog.code, VM_FINAL_NPHASES, VM_FINAL_W, lane, true, slots, cst, 0, vm::Out{nullptr, 0, 0},
          blockIdx.x == 0 ? prog.trace : nullptr);
  if (lane == 0) *result = slot_flag_get(slots, VM_FINAL_OUT[0]) ? 1 : 0;
}

// Per-vote fallback: codes[i] (still 0) := e(pk, H) == e(G1, sigma) ? 0 : VERIFY_FAIL.
__global__ __launch_bounds__(64) void k_vm_pairchk(uint32_t n, VmDev prog, const uint32_t* __restrict__ cst_g, Slab s,
                                                   int32_t* __restrict__ codes, const int32_t* __restrict__ verdict) {
  if (verdict && *verdict == 1) return;  // pipelined path: the combined check passed
  extern __shared__ uint4 lds4[];
  uint32_t* lds = reinterpret_cast<uint32_t*>(lds4);
  uint32_t* cst = lds;
  const uint32_t slice = threadIdx.x / VM_PAIRCHK_W, lane = threadIdx.x % VM_PAIRCHK_W;
  uint32_t* slots = lds + VM_NCONST * 12 + slice * VM_PAIRCHK_NSLOTS * 12;
  const uint32_t i = blockIdx.x * VM_SLICES + slice;
  const bool active = i < n && codes[i] == 0;
  load_consts(cst, cst_g, VM_NCONST);
  if (active)
    for (uint32_t k = lane; k < 12; k += VM_PAIRCHK_W) {
      Fp v;
      s.ld(v, S_FB + k, i);
      slot_put(slots, VM_PAIRCHK_IN[k], v.v);
    }
  __syncthreads();
  vm::run(prog.code, VM_PAIRCHK_NPHASES, VM_PAIRCHK_W, lane, active, slots, cst, 0, vm::Out{nullptr, 0, 0},
          blockIdx.x == 0 ? prog.trace : nullptr);
  if (active && lane == 0) codes[i] = slot_flag_get(slots, VM_PAIRCHK_OUT[0]) ? 0 : BLST_VERIFY_FAIL;
}

// AoS partials (216 words: F 144, S 72) -> planes
__global__ __launch_bounds__(64) void k_unpack_partials(uint32_t k, const uint32_t* __restrict__ parts, Slab F, Slab S) {
  const uint32_t t = blockIdx.x * 64 + threadIdx.x;
  if (t >= k * PART_PLANES) return;
  const uint32_t q = t / PART_PLANES, j = t % PART_PLANES;
  Fp v;
  for (int l = 0; l < 12; ++l) v.v[l] = parts[(size_t)q * 216 + j * 12 + l];
  if (j < 12) F.st(v, j, q);
  else S.st(v, j - 12, q);
}

// planes element 0 -> AoS partial
__global__ __launch_bounds__(64) void k_pack_partial2(Slab F, Slab S, uint32_t* __restrict__ out) {
  const uint32_t t = threadIdx.x;
  if (t >= PART_PLANES) return;
  Fp v;
  if (t < 12) F.ld(v, t, 0);
  else S.ld(v, t - 12, 0);
  for (int l = 0; l < 12; ++l) out[t * 12 + l] = v.v[l];
}

// ---- single-call kernels (one lane) ----
__global__ __launch_bounds__(WG) void k_verify_one(const uint8_t* sig, uint32_t sl, const uint8_t* hash, uint32_t hl, const uint8_t* pk,
                             uint32_t pl, XmdTemplates t, int32_t* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *out = verify_one(sig, sl, hash, hl, pk, pl, t);
}

#define GROUPCHECK_FAIL (0x100 | BLST_POINT_NOT_IN_GROUP)
// Parse list items: code_sig[i] (blst code, group-checked if gc) and the Jacobian point.
__global__ __launch_bounds__(WG) void k_parse_sig_list(uint32_t n, const uint8_t* __restrict__ data,
                                                       const uint64_t* __restrict__ off, const uint64_t* __restrict__ len,
                                                       int gc, int32_t* __restrict__ codes, Slab pts) {
  const uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  G2A a;
  bool inf;
  int e = g2_from_bytes(a, inf, data + off[i], (uint32_t)len[i]);
  G2J j;
  if (e == BLST_SUCCESS) {
    if (inf) {
      jac_set_inf(j);
    } else {
      jac_from_aff(j, a);
      if (gc && !g2_in_subgroup(j)) e = GROUPCHECK_FAIL;  // reported after all parses
    }
  }
  if (e != BLST_SUCCESS) jac_set_inf(j);
  pts.st_g2j(j, i);
  codes[i] = e;
}

__global__ __launch_bounds__(WG) void k_parse_pk_list(uint32_t n, const uint8_t* __restrict__ data,
                                                      const uint64_t* __restrict__ off, const uint64_t* __restrict__ len,
                                                      int32_t* __restrict__ codes, Slab pts) {
  const uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  G1A a;
  bool inf;
  int e = g1_from_bytes(a, inf, data + off[i], (uint32_t)len[i]);
  Fp X, Y, Z;
  if (e == BLST_SUCCESS && !inf) {
    X = a.x;
    Y = a.y;
    fp_one(Z);
  } else {
    fp_one(X);
    fp_one(Y);
    fp_zero(Z);
  }
  pts.st(X, 0, i);
  pts.st(Y, 1, i);
  pts.st(Z, 2, i);
  codes[i] = e;
}

__global__ __launch_bounds__(WG) void k_sum_g2_compress(uint32_t n, Slab pts, uint8_t* out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  G2J acc, x;
  jac_set_inf(acc);
  for (uint32_t i = 0; i < n; ++i) {
    pts.ld_g2j(x, i);
    jac_add(acc, acc, x);
  }
  g2_compress(out, acc);
}

__global__ __launch_bounds__(WG) void k_sum_g1(uint32_t n, Slab pts, uint32_t* out_jac /*36 words*/, uint8_t* out48) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  G1J acc, x;
  jac_set_inf(acc);
  for (uint32_t i = 0; i < n; ++i) {
    pts.ld(x.X, 0, i);
    pts.ld(x.Y, 1, i);
    pts.ld(x.Z, 2, i);
    jac_add(acc, acc, x);
  }
  for (int k = 0; k < 12; ++k) {
    out_jac[k] = acc.X.v[k];
    out_jac[12 + k] = acc.Y.v[k];
    out_jac[24 + k] = acc.Z.v[k];
  }
  if (out48) g1_compress(out48, acc);
}

// inner_verify_aggregated_signature (consensus.rs:365-382) after BlsPublicKey::aggregate.
__global__ __launch_bounds__(WG) void k_verify_agg(const uint32_t* agg_pk_jac, const uint8_t* sig, uint32_t sl, const uint8_t* hash,
                             uint32_t hl, XmdTemplates t, int32_t* out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  G2A s;
  bool sinf;
  int e = g2_from_bytes(s, sinf, sig, sl);
  if (e != BLST_SUCCESS) {
    *out = e;
    return;
  }
  if (hl != 32) {
    *out = OVH_ERR_HASH_LEN;
    return;
  }
  G1J pj;
  for (int k = 0; k < 12; ++k) {
    pj.X.v[k] = agg_pk_jac[k];
    pj.Y.v[k] = agg_pk_jac[12 + k];
    pj.Z.v[k] = agg_pk_jac[24 + k];
  }
  G1A pa;
  bool pinf = !jac_to_aff(pa, pj);
  uint32_t msg[8];
  be_words_from_bytes(msg, hash, 8);
  *out = core_verify(pa, pinf, s, sinf, msg, t);
}

__device__ void sk_words(uint32_t k[8], const uint8_t* sk) {
  for (int i = 0; i < 8; ++i) {
    const uint8_t* p = sk + 28 - 4 * i;
    k[i] = ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
  }
}

__global__ __launch_bounds__(WG) void k_sign(uint32_t n, const uint8_t* __restrict__ sks,
                                             const uint8_t* __restrict__ hashes, XmdTemplates t,
                                             uint8_t* __restrict__ sigs) {
  const uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  uint32_t k[8], msg[8];
  sk_words(k, sks + (size_t)i * 32);
  be_words_from_bytes(msg, hashes + (size_t)i * 32, 8);
  G2J h, s;
  hash_to_g2(h, msg, t);
  jac_mul_words(s, h, k, 8);
  g2_compress(sigs + (size_t)i * 96, s);
}

__global__ __launch_bounds__(WG) void k_sk_to_pk(uint32_t n, const uint8_t* __restrict__ sks, uint8_t* __restrict__ pks) {
  const uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  uint32_t k[8];
  sk_words(k, sks + (size_t)i * 32);
  G1J g, p;
  fp_load(g.X, G1X_M);
  fp_load(g.Y, G1Y_M);
  fp_one(g.Z);
  jac_mul_words(p, g, k, 8);
  g1_compress(pks + (size_t)i * 48, p);
}

// ------------------------------------------------------------------------ host side
struct ovh_ctx {
  int device = 0;
  uint32_t flags = 0;
  hipStream_t stream = nullptr;
  // pipelined batches (ovh_verify_batch_device_async): the final check + fallback of batch k run
  // on fstream while batch k + 1's per-vote stages run on stream; OVH_BATCH_SLOTS slots of batch
  // state rotate (a slot is reused only after its final-stream work finished).
  hipStream_t fstream = nullptr;
  hipStream_t hstream = nullptr;  // hash_to_field of the next batch, beside the current vote
  hipEvent_t ev_h[OVH_BATCH_SLOTS] = {};
  hipEvent_t ev_front[OVH_BATCH_SLOTS] = {}, ev_back[OVH_BATCH_SLOTS] = {};
  uint32_t* state_slot[OVH_BATCH_SLOTS] = {};
  uint32_t* red_slot[OVH_BATCH_SLOTS] = {};
  uint32_t* fin = nullptr;       // OVH_BATCH_SLOTS x FIN_STRIDE words: per-slot combine scratch
  uint32_t pipe_k = 0;
  int last_slot = 0;
  XmdTemplates xmd;
  std::mutex mu;  // Crypto is Send + Sync: serialise device use per context
  // batch buffers
  uint32_t cap = 0;
  uint32_t* state = nullptr;     // S_TOTAL Fp slabs, cap each
  uint32_t* red = nullptr;       // reduction scratch: 2 x (12 + 6) Fp slabs of cap/8
  uint32_t red_cap = 0;
  int32_t* st_pk = nullptr;
  int32_t* st_sig = nullptr;
  int32_t* codes = nullptr;      // internal codes for host-pointer API
  uint8_t* in_buf = nullptr;     // staging for host inputs
  size_t in_cap = 0;
  uint32_t* partial = nullptr;   // 216 words
  int32_t* result = nullptr;     // device scalar
  uint32_t last_n = 0;
  // Fp-VM programs + constant table in device memory
  VmDev vm_vote{}, vm_fold{}, vm_final{}, vm_pairchk{};
  uint32_t* vm_consts = nullptr;
  std::vector<void*> vm_bufs;
  // OVH_FLAG_PROFILE: start/stop events per stage of the last batch call
  hipEvent_t ev0[OVH_NSTAGES] = {}, ev1[OVH_NSTAGES] = {};
  uint32_t ev_mask = 0;
};

#define HIPCHK(x)                                  \
  do {                                             \
    if ((x) != hipSuccess) return OVH_ERR_DEVICE;  \
  } while (0)

static const char* const STAGE_NAMES[OVH_NSTAGES] = {"hash_to_field", "vote", "fold", "final", "fallback"};

// LDS bytes of the VM kernels: constants + slices x slots (+ a 16-byte slice header for vote)
static constexpr size_t LDS_VOTE = (size_t)VM_NCONST * 48 + VM_SLICES * ((size_t)VM_VOTE_NSLOTS * 48 + 16);
static constexpr size_t LDS_FOLD = (size_t)VM_NCONST * 48 + VM_FOLD_UNITS * (size_t)VM_FOLD_NSLOTS * 48;
static constexpr size_t LDS_FINAL = (size_t)VM_NCONST * 48 + (size_t)VM_FINAL_NSLOTS * 48;
static constexpr size_t LDS_PAIRCHK = (size_t)VM_NCONST * 48 + VM_SLICES * (size_t)VM_PAIRCHK_NSLOTS * 48;
static_assert(VM_VOTE_W * VM_SLICES == 64 && VM_FOLD_W * VM_FOLD_UNITS == 64 && VM_PAIRCHK_W * VM_SLICES == 64 &&
                  VM_FINAL_W == 64, "VM slice widths");
static constexpr size_t LDS_FOLD1 = (size_t)VM_NCONST * 48 + (size_t)VM_FOLD_NSLOTS * 48;
static_assert(LDS_VOTE <= 160 * 1024 && LDS_FINAL <= 160 * 1024, "VM LDS budget");
static_assert(VM_FOLD_NSLOTS * 12 <= VM_SLICES * (VM_VOTE_NSLOTS * 12 + 4), "fused fold reuses the vote slots");

static int vm_upload(ovh_ctx* c, VmDev& d, const uint32_t* code, uint32_t nphases, uint32_t W, const uint16_t* in,
                     uint32_t nin, const uint16_t* out, uint32_t nout) {
  const size_t words = (size_t)nphases * W * 4, pad = (size_t)2 * W * 4;  // + two NOP phases (prefetch)
  void *dc = nullptr, *di = nullptr, *dout = nullptr;
  HIPCHK(hipMalloc(&dc, (words + pad) * 4));
  c->vm_bufs.push_back(dc);
  HIPCHK(hipMemcpy(dc, code, words * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemset((uint32_t*)dc + words, 0, pad * 4));
  HIPCHK(hipMalloc(&di, nin * 2 + 2));
  c->vm_bufs.push_back(di);
  HIPCHK(hipMemcpy(di, in, nin * 2, hipMemcpyHostToDevice));
  HIPCHK(hipMalloc(&dout, nout * 2 + 2));
  c->vm_bufs.push_back(dout);
  HIPCHK(hipMemcpy(dout, out, nout * 2, hipMemcpyHostToDevice));
  d.code = (const uint4*)dc;
  d.nphases = nphases;
  d.in = (const uint16_t*)di;
  d.out = (const uint16_t*)dout;
  d.trace = nullptr;
  if (c->flags & OVH_FLAG_VM_TRACE) {
    void* dt = nullptr;
    HIPCHK(hipMalloc(&dt, ((size_t)nphases + 1) * 8));
    c->vm_bufs.push_back(dt);
    HIPCHK(hipMemset(dt, 0, ((size_t)nphases + 1) * 8));
    d.trace = (uint64_t*)dt;
  }
  return 0;
}

static int vm_init(ovh_ctx* c) {
  HIPCHK(hipMalloc(&c->vm_consts, sizeof(VM_CONST_WORDS)));
  HIPCHK(hipMemcpy(c->vm_consts, VM_CONST_WORDS, sizeof(VM_CONST_WORDS), hipMemcpyHostToDevice));
  if (vm_upload(c, c->vm_vote, VM_VOTE_CODE, VM_VOTE_NPHASES, VM_VOTE_W, VM_VOTE_IN, VM_VOTE_NIN, VM_VOTE_OUT,
                VM_VOTE_NOUT) ||
      vm_upload(c, c->vm_fold, VM_FOLD_CODE, VM_FOLD_NPHASES, VM_FOLD_W, VM_FOLD_IN, VM_FOLD_NIN, VM_FOLD_OUT,
                VM_FOLD_NOUT) ||
      vm_upload(c, c->vm_final, VM_FINAL_CODE, VM_FINAL_NPHASES, VM_FINAL_W, VM_FINAL_IN, VM_FINAL_NIN,
                VM_FINAL_OUT, VM_FINAL_NOUT) ||
      vm_upload(c, c->vm_pairchk, VM_PAIRCHK_CODE, VM_PAIRCHK_NPHASES, VM_PAIRCHK_W, VM_PAIRCHK_IN,
                VM_PAIRCHK_NIN, VM_PAIRCHK_OUT, VM_PAIRCHK_NOUT))
    return OVH_ERR_DEVICE;
  HIPCHK(hipFuncSetAttribute((const void*)k_vm_vote, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_VOTE));
  HIPCHK(hipFuncSetAttribute((const void*)k_vm_fold<VM_FOLD_UNITS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)LDS_FOLD));
  HIPCHK(hipFuncSetAttribute((const void*)k_vm_fold<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_FOLD1));
  HIPCHK(hipFuncSetAttribute((const void*)k_vm_final, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_FINAL));
  HIPCHK(hipFuncSetAttribute((const void*)k_vm_pairchk, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)LDS_PAIRCHK));
  return 0;
}

// Stage bracket: events on the context's stream around the stage's kernels.
struct StageScope {
  ovh_ctx* c;
  int k;
  hipStream_t st;
  StageScope(ovh_ctx* c_, int k_, hipStream_t st_ = nullptr) : c(c_), k(k_), st(st_ ? st_ : c_->stream) {
    if (c->flags & OVH_FLAG_PROFILE) (void)hipEventRecord(c->ev0[k], st);
  }
  ~StageScope() {
    if (c->flags & OVH_FLAG_PROFILE) {
      (void)hipEventRecord(c->ev1[k], st);
      c->ev_mask |= 1u << k;
    }
  }
};


static const uint8_t DEFAULT_DST[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_";

static uint32_t nblk(size_t n) { return (uint32_t)((n + WG - 1) / WG); }

static int ensure_cap(ovh_ctx* c, size_t n) {
  if (n > (1u << 24)) return OVH_ERR_ARG;
  if (n <= c->cap && c->state) return 0;
  uint32_t cap = 256;
  while (cap < n) cap <<= 1;
  HIPCHK(hipStreamSynchronize(c->stream));
  if (c->fstream) HIPCHK(hipStreamSynchronize(c->fstream));
  if (c->hstream) HIPCHK(hipStreamSynchronize(c->hstream));
  for (int k = 0; k < OVH_BATCH_SLOTS; ++k) {
    if (c->state_slot[k]) (void)hipFree(c->state_slot[k]);
    if (c->red_slot[k]) (void)hipFree(c->red_slot[k]);
    c->state_slot[k] = c->red_slot[k] = nullptr;
  }
  if (c->st_pk) (void)hipFree(c->st_pk);
  if (c->st_sig) (void)hipFree(c->st_sig);
  if (c->codes) (void)hipFree(c->codes);
  c->state = nullptr;
  c->red = nullptr;
  c->red_cap = cap / 4 > 64 ? cap / 4 : 64;
  for (int k = 0; k < OVH_BATCH_SLOTS; ++k) {
    HIPCHK(hipMalloc(&c->state_slot[k], (size_t)S_TOTAL * 12 * cap * 4));
    HIPCHK(hipMalloc(&c->red_slot[k], (size_t)2 * PART_PLANES * 12 * c->red_cap * 4));
  }
  c->state = c->state_slot[0];
  c->red = c->red_slot[0];
  HIPCHK(hipMalloc(&c->st_pk, (size_t)cap * 4));
  HIPCHK(hipMalloc(&c->st_sig, (size_t)cap * 4));
  HIPCHK(hipMalloc(&c->codes, (size_t)cap * 4));
  c->cap = cap;
  return 0;
}

// Wait for pipelined batch work on the final stream (APIs that reuse the batch state as
// scratch call this first).
static int drain(ovh_ctx* c) {
  if (c->fstream) HIPCHK(hipStreamSynchronize(c->fstream));
  return 0;
}

// Batch state slot k for the next batch on the main stream: the stream first waits until the
// final stream has finished with the slot's previous batch (its fallback reads that state).
static int take_slot(ovh_ctx* c, int k) {
  HIPCHK(hipStreamWaitEvent(c->stream, c->ev_back[k], 0));
  c->state = c->state_slot[k];
  c->red = c->red_slot[k];
  c->last_slot = k;
  return 0;
}

static int ensure_in(ovh_ctx* c, size_t bytes) {
  if (bytes <= c->in_cap && c->in_buf) return 0;
  size_t cap = 4096;
  while (cap < bytes) cap <<= 1;
  if (c->in_buf) (void)hipFree(c->in_buf);
  c->in_buf = nullptr;
  HIPCHK(hipMalloc(&c->in_buf, cap));
  c->in_cap = cap;
  return 0;
}

extern "C" {

ovh_ctx* ovh_create(int device, const uint8_t* dst, size_t dst_len, uint32_t flags) {
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  ovh_ctx* c = new (std::nothrow) ovh_ctx();
  if (!c) return nullptr;
  c->device = device;
  c->flags = flags;
  if (!dst) {
    dst = DEFAULT_DST;
    dst_len = 43;
  }
  if (!xmd_build_templates(c->xmd, dst, (uint32_t)dst_len) ||
      hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(&c->partial, 216 * 4) != hipSuccess || hipMalloc(&c->result, 64) != hipSuccess) {
    delete c;
    return nullptr;
  }
  if (vm_init(c)) {
    ovh_destroy(c);
    return nullptr;
  }
  {
    int lo = 0, hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo, &hi);  // lo = numerically largest = lowest priority
    if (hipStreamCreateWithPriority(&c->fstream, hipStreamNonBlocking, lo) != hipSuccess ||
        hipStreamCreateWithFlags(&c->hstream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&c->fin, (size_t)OVH_BATCH_SLOTS * FIN_STRIDE * 4) != hipSuccess) {
      ovh_destroy(c);
      return nullptr;
    }
    for (int k = 0; k < OVH_BATCH_SLOTS; ++k)
      if (hipEventCreateWithFlags(&c->ev_front[k], hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&c->ev_h[k], hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&c->ev_back[k], hipEventDisableTiming) != hipSuccess) {
        ovh_destroy(c);
        return nullptr;
      }
  }
  if (flags & OVH_FLAG_PROFILE)
    for (int k = 0; k < OVH_NSTAGES; ++k)
      if (hipEventCreate(&c->ev0[k]) != hipSuccess || hipEventCreate(&c->ev1[k]) != hipSuccess) {
        ovh_destroy(c);
        return nullptr;
      }
  return c;
}

void ovh_destroy(ovh_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->fstream) (void)hipStreamSynchronize(c->fstream);
  if (c->hstream) (void)hipStreamSynchronize(c->hstream);
  for (int k = 0; k < OVH_BATCH_SLOTS; ++k)
    for (void* p : {(void*)c->state_slot[k], (void*)c->red_slot[k]})
      if (p) (void)hipFree(p);
  for (void* p : {(void*)c->st_pk, (void*)c->st_sig, (void*)c->codes, (void*)c->in_buf, (void*)c->partial,
                  (void*)c->result, (void*)c->vm_consts, (void*)c->fin})
    if (p) (void)hipFree(p);
  if (c->fstream) (void)hipStreamDestroy(c->fstream);
  if (c->hstream) (void)hipStreamDestroy(c->hstream);
  for (int k = 0; k < OVH_BATCH_SLOTS; ++k) {
    if (c->ev_front[k]) (void)hipEventDestroy(c->ev_front[k]);
    if (c->ev_h[k]) (void)hipEventDestroy(c->ev_h[k]);
    if (c->ev_back[k]) (void)hipEventDestroy(c->ev_back[k]);
  }
  for (void* p : c->vm_bufs) (void)hipFree(p);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  for (int k = 0; k < OVH_NSTAGES; ++k) {
    if (c->ev0[k]) (void)hipEventDestroy(c->ev0[k]);
    if (c->ev1[k]) (void)hipEventDestroy(c->ev1[k]);
  }
  delete c;
}

int ovh_vm_trace(ovh_ctx* c, int prog, uint64_t* stamps, size_t max) {
  if (!c || prog < 0 || prog > 3 || (max && !stamps)) return -OVH_ERR_ARG;
  if (!(c->flags & OVH_FLAG_VM_TRACE)) return 0;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return -OVH_ERR_DEVICE;
  const VmDev* d = prog == 0 ? &c->vm_vote : prog == 1 ? &c->vm_fold : prog == 2 ? &c->vm_final : &c->vm_pairchk;
  const size_t n = (size_t)d->nphases + 1, k = max < n ? max : n;
  if (hipStreamSynchronize(c->stream) != hipSuccess ||
      (k && hipMemcpy(stamps, d->trace, k * 8, hipMemcpyDeviceToHost) != hipSuccess))
    return -OVH_ERR_DEVICE;
  return (int)n;
}

int ovh_stage_times(ovh_ctx* c, float* ms, size_t max) {
  if (!c || (!ms && max)) return -OVH_ERR_ARG;
  if (!(c->flags & OVH_FLAG_PROFILE)) return 0;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess || hipStreamSynchronize(c->stream) != hipSuccess) return -OVH_ERR_DEVICE;
  const size_t n = max < OVH_NSTAGES ? max : OVH_NSTAGES;
  for (size_t k = 0; k < n; ++k) {
    ms[k] = 0.f;
    if (c->ev_mask & (1u << k))
      if (hipEventElapsedTime(&ms[k], c->ev0[k], c->ev1[k]) != hipSuccess) return -OVH_ERR_DEVICE;
  }
  return (int)n;
}

const char* ovh_stage_name(int k) { return (k >= 0 && k < OVH_NSTAGES) ? STAGE_NAMES[k] : nullptr; }

void* ovh_stream(ovh_ctx* c) { return c ? (void*)c->stream : nullptr; }

int ovh_sm3(const uint8_t* msg, size_t len, uint8_t out[32]) {
  if ((!msg && len) || !out) return OVH_ERR_ARG;
  sm3_digest(msg, len, out);
  return 0;
}

// 0 < sk < r, 32 bytes big-endian (blst SecretKey::from_bytes)
static bool sk_valid(const uint8_t* sk, size_t len) {
  static const uint8_t R_BE[32] = {0x73, 0xed, 0xa7, 0x53, 0x29, 0x9d, 0x7d, 0x48, 0x33, 0x39, 0xd8,
                                   0x08, 0x09, 0xa1, 0xd8, 0x05, 0x53, 0xbd, 0xa4, 0x02, 0xff, 0xfe,
                                   0x5b, 0xfe, 0xff, 0xff, 0xff, 0xff, 0x00, 0x00, 0x00, 0x01};
  if (!sk || len != 32) return false;
  bool nz = false;
  for (int i = 0; i < 32; ++i) nz |= sk[i] != 0;
  if (!nz) return false;
  return memcmp(sk, R_BE, 32) < 0;
}

int ovh_sign(ovh_ctx* c, const uint8_t* sk, size_t sk_len, const uint8_t* hash, size_t hash_len, uint8_t out[96]) {
  if (!c || !out) return OVH_ERR_ARG;
  if (hash_len != 32 || !hash) return OVH_ERR_HASH_LEN;
  if (!sk_valid(sk, sk_len)) return BLST_BAD_ENCODING;
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  if (ensure_in(c, 256)) return OVH_ERR_DEVICE;
  HIPCHK(hipMemcpyAsync(c->in_buf, sk, 32, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->in_buf + 32, hash, 32, hipMemcpyHostToDevice, c->stream));
  k_sign<<<1, WG, 0, c->stream>>>(1, c->in_buf, c->in_buf + 32, c->xmd, c->in_buf + 64);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out, c->in_buf + 64, 96, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int ovh_sk_to_pk(ovh_ctx* c, const uint8_t* sk, size_t sk_len, uint8_t out[48]) {
  if (!c || !out) return OVH_ERR_ARG;
  if (!sk_valid(sk, sk_len)) return BLST_BAD_ENCODING;
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  if (ensure_in(c, 128)) return OVH_ERR_DEVICE;
  HIPCHK(hipMemcpyAsync(c->in_buf, sk, 32, hipMemcpyHostToDevice, c->stream));
  k_sk_to_pk<<<1, WG, 0, c->stream>>>(1, c->in_buf, c->in_buf + 32);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out, c->in_buf + 32, 48, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int ovh_verify(ovh_ctx* c, const uint8_t* sig, size_t sig_len, const uint8_t* hash, size_t hash_len, const uint8_t* pk,
               size_t pk_len) {
  if (!c) return OVH_ERR_ARG;
  if (hash_len != 32 || !hash) return OVH_ERR_HASH_LEN;
  if (sig_len > 4096 || pk_len > 4096 || (sig_len && !sig) || (pk_len && !pk)) return OVH_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  if (ensure_in(c, 32 + sig_len + pk_len + 64)) return OVH_ERR_DEVICE;
  uint8_t* d = c->in_buf;
  HIPCHK(hipMemcpyAsync(d, hash, 32, hipMemcpyHostToDevice, c->stream));
  if (sig_len) HIPCHK(hipMemcpyAsync(d + 32, sig, sig_len, hipMemcpyHostToDevice, c->stream));
  if (pk_len) HIPCHK(hipMemcpyAsync(d + 32 + sig_len, pk, pk_len, hipMemcpyHostToDevice, c->stream));
  k_verify_one<<<1, WG, 0, c->stream>>>(d + 32, (uint32_t)sig_len, d, 32, d + 32 + sig_len, (uint32_t)pk_len, c->xmd,
                                         c->result);
  HIPCHK(hipGetLastError());
  int32_t r = -1;
  HIPCHK(hipMemcpyAsync(&r, c->result, 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return r;
}

// Stage a (data, lens, n) list on the device: bytes at d, offsets/lengths (u64) after it.
static int stage_list(ovh_ctx* c, const uint8_t* data, const size_t* lens, size_t n, size_t base, uint8_t** d_data,
                      uint64_t** d_off, uint64_t** d_len, size_t* used) {
  size_t total = 0;
  for (size_t i = 0; i < n; ++i) total += lens[i];
  std::vector<uint64_t> meta(2 * n + 1);
  size_t o = 0;
  for (size_t i = 0; i < n; ++i) {
    meta[i] = o;
    meta[n + i] = lens[i];
    o += lens[i];
  }
  const size_t data_bytes = (total + 15) & ~(size_t)15;
  const size_t need = base + data_bytes + 16 * (n + 1);
  if (ensure_in(c, need)) return OVH_ERR_DEVICE;
  uint8_t* d = c->in_buf + base;
  if (total) HIPCHK(hipMemcpyAsync(d, data, total, hipMemcpyHostToDevice, c->stream));
  uint64_t* m = (uint64_t*)(d + data_bytes);
  if (n) HIPCHK(hipMemcpyAsync(m, meta.data(), 16 * n, hipMemcpyHostToDevice, c->stream));
  *d_data = d;
  *d_off = m;
  *d_len = m + n;
  *used = need;
  return 0;
}

int ovh_aggregate_sigs(ovh_ctx* c, const uint8_t* sigs, const size_t* sig_lens, size_t n_sigs, const uint8_t* pks,
                       const size_t* pk_lens, size_t n_pks, uint8_t out[96]) {
  if (!c || !out) return OVH_ERR_ARG;
  if (n_sigs != n_pks) return OVH_ERR_LEN_MISMATCH;
  const size_t n = n_sigs;
  if (n && (!sig_lens || !pk_lens)) return OVH_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  if (drain(c) || ensure_cap(c, n > 0 ? n : 1)) return OVH_ERR_DEVICE;
  // the staging buffer may be reallocated by the second stage_list: stage both first, then launch
  uint8_t *ds, *dp;
  uint64_t *so, *sl, *po, *pl;
  size_t used1 = 0, used2 = 0;
  {
    // size the staging buffer for both lists up front
    size_t t1 = 0, t2 = 0;
    for (size_t i = 0; i < n; ++i) {
      t1 += sig_lens[i];
      t2 += pk_lens[i];
    }
    if (ensure_in(c, t1 + t2 + 512 + 32 * (n + 1))) return OVH_ERR_DEVICE;
  }
  if (stage_list(c, sigs, sig_lens, n, 0, &ds, &so, &sl, &used1)) return OVH_ERR_DEVICE;
  if (stage_list(c, pks, pk_lens, n, used1, &dp, &po, &pl, &used2)) return OVH_ERR_DEVICE;
  Slab pts{c->state, c->cap};
  Slab ppts{c->state + (size_t)6 * 12 * c->cap, c->cap};
  if (n) {
    k_parse_sig_list<<<nblk(n), WG, 0, c->stream>>>((uint32_t)n, ds, so, sl, (c->flags & OVH_FLAG_AGG_NO_GROUPCHECK) ? 0 : 1,
                                                   c->st_sig, pts);
    k_parse_pk_list<<<nblk(n), WG, 0, c->stream>>>((uint32_t)n, dp, po, pl, c->st_pk, ppts);
    HIPCHK(hipGetLastError());
  }
  std::vector<int32_t> cs(n), cp(n);
  if (n) {
    HIPCHK(hipMemcpyAsync(cs.data(), c->st_sig, 4 * n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(cp.data(), c->st_pk, 4 * n, hipMemcpyDeviceToHost, c->stream));
  }
  HIPCHK(hipStreamSynchronize(c->stream));
  // consensus.rs:431-439: per pair, signature first, then the public key.
  for (size_t i = 0; i < n; ++i) {
    if (cs[i] != BLST_SUCCESS && cs[i] != GROUPCHECK_FAIL) return cs[i];
    if (cp[i] != BLST_SUCCESS) return OVH_ERR_PUBKEY;
  }
  // BlsSignature::combine (consensus.rs:441): empty -> AGGR_TYPE_MISMATCH, then group checks
  if (n == 0) return BLST_AGGR_TYPE_MISMATCH;
  for (size_t i = 0; i < n; ++i)
    if (cs[i] == GROUPCHECK_FAIL) return BLST_POINT_NOT_IN_GROUP;
  k_sum_g2_compress<<<1, WG, 0, c->stream>>>((uint32_t)n, pts, c->in_buf + used2);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out, c->in_buf + used2, 96, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

// Parses + sums a pk list on the device; the Jacobian sum (36 words) stays at *d_sum.
static int sum_pks(ovh_ctx* c, const uint8_t* pks, const size_t* pk_lens, size_t n, uint8_t* out48, uint32_t** d_sum) {
  if (n && !pk_lens) return OVH_ERR_ARG;
  if (drain(c) || ensure_cap(c, n > 0 ? n : 1)) return OVH_ERR_DEVICE;
  size_t t = 0;
  for (size_t i = 0; i < n; ++i) t += pk_lens[i];
  if (ensure_in(c, t + 16 * (n + 1) + 256)) return OVH_ERR_DEVICE;
  uint8_t* dp;
  uint64_t *po, *pl;
  size_t used = 0;
  if (stage_list(c, pks, pk_lens, n, 0, &dp, &po, &pl, &used)) return OVH_ERR_DEVICE;
  Slab ppts{c->state, c->cap};
  if (n) {
    k_parse_pk_list<<<nblk(n), WG, 0, c->stream>>>((uint32_t)n, dp, po, pl, c->st_pk, ppts);
    HIPCHK(hipGetLastError());
  }
  std::vector<int32_t> cp(n);
  if (n) HIPCHK(hipMemcpyAsync(cp.data(), c->st_pk, 4 * n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  for (size_t i = 0; i < n; ++i)
    if (cp[i] != BLST_SUCCESS) return OVH_ERR_PUBKEY;
  if (n == 0) return BLST_AGGR_TYPE_MISMATCH;
  uint32_t* sum = (uint32_t*)(c->in_buf + ((used + 15) & ~(size_t)15));
  uint8_t* o48 = (uint8_t*)(sum + 36);
  k_sum_g1<<<1, WG, 0, c->stream>>>((uint32_t)n, ppts, sum, o48);
  HIPCHK(hipGetLastError());
  if (out48) HIPCHK(hipMemcpyAsync(out48, o48, 48, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  *d_sum = sum;
  return 0;
}

int ovh_aggregate_pks(ovh_ctx* c, const uint8_t* pks, const size_t* pk_lens, size_t n, uint8_t out[48]) {
  if (!c || !out) return OVH_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  uint32_t* sum = nullptr;
  return sum_pks(c, pks, pk_lens, n, out, &sum);
}

int ovh_verify_aggregated(ovh_ctx* c, const uint8_t* agg_sig, size_t agg_len, const uint8_t* hash, size_t hash_len,
                          const uint8_t* pks, const size_t* pk_lens, size_t n) {
  if (!c) return OVH_ERR_ARG;
  if (agg_len > 4096 || (agg_len && !agg_sig)) return OVH_ERR_ARG;
  if (n && !pk_lens) return OVH_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  {
    size_t t = 0;
    for (size_t i = 0; i < n; ++i) t += pk_lens[i];
    if (ensure_in(c, t + 16 * (n + 1) + 1024 + agg_len)) return OVH_ERR_DEVICE;  // no realloc below
  }
  uint32_t* sum = nullptr;
  int e = sum_pks(c, pks, pk_lens, n, nullptr, &sum);
  if (e) return e;
  // stage sig + hash behind the sum (sum occupies 36 words + 48 bytes)
  uint8_t* d = (uint8_t*)sum + 256;
  const size_t hl = (hash && hash_len <= 64) ? hash_len : 0;
  if (agg_len) HIPCHK(hipMemcpyAsync(d, agg_sig, agg_len, hipMemcpyHostToDevice, c->stream));
  if (hl) HIPCHK(hipMemcpyAsync(d + agg_len, hash, hl, hipMemcpyHostToDevice, c->stream));
  k_verify_agg<<<1, WG, 0, c->stream>>>(sum, d, (uint32_t)agg_len, d + agg_len, (uint32_t)(hash ? hash_len : 0), c->xmd,
                                       c->result);
  HIPCHK(hipGetLastError());
  int32_t r = -1;
  HIPCHK(hipMemcpyAsync(&r, c->result, 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return r;
}

// ---- batch ----
// Per-vote stages of a batch on the main stream: hash_to_field, then the vote kernel with fold
// level 0 fused in: *outF / *outS = ceil(n / 4) partials as planes in the slot's fold scratch
// (half 0), *out_m their count.
static int batch_front(ovh_ctx* c, uint32_t n, const uint8_t* d_sigs, const uint8_t* d_hashes, const uint8_t* d_pks,
                       uint64_t seed, int32_t* d_codes, Slab* outF, Slab* outS, uint32_t* out_m, int slot = -1) {
  Slab s{c->state, c->cap};
  hipStream_t st = c->stream;
  c->ev_mask = 0;
  const uint32_t nwg = (n + VM_SLICES - 1) / VM_SLICES;
  Slab p0{c->red, c->red_cap};
  if (slot >= 0) {
    // pipelined: hash_to_field on its own stream, as soon as the slot's previous batch has
    // finished its per-vote stages (the only reader of the S_U planes), so it runs beside the
    // current vote kernel; the vote waits for it
    HIPCHK(hipStreamWaitEvent(c->hstream, c->ev_front[slot], 0));
    {
      StageScope p(c, ST_H2F, c->hstream);
      k_h2f<<<nblk(n), WG, 0, c->hstream>>>(n, d_hashes, c->xmd, s);
    }
    HIPCHK(hipEventRecord(c->ev_h[slot], c->hstream));
    HIPCHK(hipStreamWaitEvent(st, c->ev_h[slot], 0));
  } else {
    StageScope p(c, ST_H2F);
    k_h2f<<<nblk(n), WG, 0, st>>>(n, d_hashes, c->xmd, s);
  }
  {
    StageScope p(c, ST_VOTE);
    k_vm_vote<<<nwg, 64, LDS_VOTE, st>>>(n, c->vm_vote, c->vm_fold, c->vm_consts, d_pks, d_sigs, s, seed, d_codes,
                                         p0);
  }
  HIPCHK(hipGetLastError());
  c->last_n = n;
  *outF = p0;
  *outS = Slab{c->red + (size_t)12 * 12 * c->red_cap, c->red_cap};
  *out_m = nwg;
  return 0;
}

// Fold levels down to <= `until` partials, on stream st, ping-ponging through the slot's fold
// scratch (the level-0 partials are in half 0; *flip_io carries the next output half across
// calls). slices = 4 (main stream) or 1 (the final stream, beside the next batch's vote
// workgroups).
static int fold_levels(ovh_ctx* c, hipStream_t st, int slices, Slab* F, Slab* S, uint32_t* m, uint32_t until = 4,
                       int* flip_io = nullptr) {
  StageScope p(c, ST_FOLD, st);
  int flip = flip_io ? *flip_io : 1;
  while (*m > until) {
    const uint32_t mo = (*m + 3) / 4;
    uint32_t* base = c->red + (size_t)flip * PART_PLANES * 12 * c->red_cap;
    Slab o{base, c->red_cap};
    if (slices == 1)
      k_vm_fold<1><<<mo, 64, LDS_FOLD1, st>>>(*m, c->vm_fold, c->vm_consts, *F, *S, o, nullptr);
    else
      k_vm_fold<VM_FOLD_UNITS><<<(mo + VM_FOLD_UNITS - 1) / VM_FOLD_UNITS, 64, LDS_FOLD, st>>>(*m, c->vm_fold, c->vm_consts, *F,
                                                                                 *S, o, nullptr);
    *F = o;
    *S = Slab{base + (size_t)12 * 12 * c->red_cap, c->red_cap};
    *m = mo;
    flip ^= 1;
  }
  if (flip_io) *flip_io = flip;
  return hipGetLastError() == hipSuccess ? 0 : OVH_ERR_DEVICE;
}

// Verdict words in c->result: [0] single-call APIs, then per batch slot the pipelined batch
// and pipelined combine verdicts, then the synchronous combine's.
enum { RES_BATCH = 4, RES_COMBINE = RES_BATCH + OVH_BATCH_SLOTS, RES_SYNC = RES_COMBINE + OVH_BATCH_SLOTS };
static_assert(RES_SYNC < 16, "verdict words fit c->result");

int ovh_batch_partial_device(ovh_ctx* c, size_t n, const uint8_t* d_sigs, const uint8_t* d_hashes, const uint8_t* d_pks,
                             uint64_t seed, int32_t* d_codes, uint8_t* d_partial) {
  if (!c || !d_codes || !d_partial || (n && (!d_sigs || !d_hashes || !d_pks))) return OVH_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  if (n == 0) {
    // neutral partial: F = 1, S = O = (0 : 1 : 0)
    std::vector<uint32_t> p(216, 0);
    for (int k = 0; k < 12; ++k) p[k] = ONE_M[k];
    for (int k = 0; k < 12; ++k) p[144 + 24 + k] = ONE_M[k];  // Y.c0 = 1
    HIPCHK(hipMemcpyAsync(d_partial, p.data(), 864, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->last_n = 0;
    return 0;
  }
  if (ensure_cap(c, n)) return OVH_ERR_DEVICE;
  if (take_slot(c, (int)(c->pipe_k++ % OVH_BATCH_SLOTS))) return OVH_ERR_DEVICE;
  Slab F, S;
  uint32_t m;
  int e = batch_front(c, (uint32_t)n, d_sigs, d_hashes, d_pks, seed, d_codes, &F, &S, &m);
  if (e || (e = fold_levels(c, c->stream, VM_SLICES, &F, &S, &m))) return e;
  if (m > 1) {  // fold the last <= 4 into one partial
    uint32_t* base = c->red + (size_t)(F.p == c->red ? 1 : 0) * PART_PLANES * 12 * c->red_cap;
    Slab o{base, c->red_cap};
    k_vm_fold<VM_FOLD_UNITS><<<1, 64, LDS_FOLD, c->stream>>>(m, c->vm_fold, c->vm_consts, F, S, o, nullptr);
    F = o;
  }
  // pack element 0 (F planes, S planes) into the AoS partial
  k_pack_partial2<<<1, 64, 0, c->stream>>>(F, m > 1 ? Slab{F.p + (size_t)12 * 12 * F.cap, F.cap} : S,
                                           (uint32_t*)d_partial);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

// Final check on <= 4 partials given as planes: k_vm_final on stream `st`, verdict to *d_res.
static void enqueue_final(ovh_ctx* c, hipStream_t st, Slab F, Slab S, uint32_t m, int32_t* d_res) {
  StageScope p(c, ST_FINAL, st);
  k_vm_final<<<1, 64, LDS_FINAL, st>>>(m, c->vm_final, c->vm_consts, F, S, d_res);
}

// Per-vote fallback of the batch in state slot `slot`, on stream `st`, skipped on the device
// when *d_verdict == 1 (d_verdict null: always runs).
static void enqueue_fallback(ovh_ctx* c, hipStream_t st, int slot, uint32_t n, int32_t* d_codes,
                             const int32_t* d_verdict) {
  StageScope p(c, ST_FALLBACK, st);
  k_vm_pairchk<<<(n + VM_SLICES - 1) / VM_SLICES, 64, LDS_PAIRCHK, st>>>(
      n, c->vm_pairchk, c->vm_consts, Slab{c->state_slot[slot], c->cap}, d_codes, d_verdict);
}

// AoS partials (k <= 16) -> <= 4 partials as planes in the fin area of `slot` (unpack, and one
// fold level when k > 4), on stream st. Scratch: fin slot area + the slot's upper half.
static int stage_partials(ovh_ctx* c, hipStream_t st, size_t k, const uint8_t* d_partials, uint32_t* scratch,
                          Slab* F, Slab* S, uint32_t* m) {
  Slab uF{scratch, 16}, uS{scratch + (size_t)12 * 12 * 16, 16};
  k_unpack_partials<<<(uint32_t)((k * PART_PLANES + 63) / 64), 64, 0, st>>>((uint32_t)k, (const uint32_t*)d_partials,
                                                                           uF, uS);
  if (k <= 4) {
    *F = uF;
    *S = uS;
    *m = (uint32_t)k;
  } else {
    uint32_t* o = scratch + (size_t)PART_PLANES * 12 * 16;
    Slab oF{o, 4};
    k_vm_fold<VM_FOLD_UNITS><<<1, 64, LDS_FOLD, st>>>((uint32_t)k, c->vm_fold, c->vm_consts, uF, uS, oF, nullptr);
    *F = oF;
    *S = Slab{o + (size_t)12 * 12 * 4, 4};
    *m = (uint32_t)((k + 3) / 4);
  }
  return hipGetLastError() == hipSuccess ? 0 : OVH_ERR_DEVICE;
}

int ovh_combine_partials_device(ovh_ctx* c, size_t k, const uint8_t* d_partials) {
  if (!c || !d_partials || k == 0 || k > 4096) return -OVH_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return -OVH_ERR_DEVICE;
  if (ensure_cap(c, k * 4 > 256 ? k * 4 : 256)) return -OVH_ERR_DEVICE;
  if (drain(c)) return -OVH_ERR_DEVICE;
  // AoS partials -> planes (F at S_F, S at S_RS of the current slot's state), fold to <= 4
  Slab F{c->state + (size_t)S_F * 12 * c->cap, c->cap}, S{c->state + (size_t)S_RS * 12 * c->cap, c->cap};
  k_unpack_partials<<<(uint32_t)((k * PART_PLANES + 63) / 64), 64, 0, c->stream>>>((uint32_t)k,
                                                                                   (const uint32_t*)d_partials, F, S);
  uint32_t m = (uint32_t)k;
  int flip = 0;
  while (m > 4) {
    const uint32_t mo = (m + 3) / 4;
    uint32_t* base = c->red + (size_t)flip * PART_PLANES * 12 * c->red_cap;
    Slab o{base, c->red_cap};
    k_vm_fold<VM_FOLD_UNITS><<<(mo + VM_FOLD_UNITS - 1) / VM_FOLD_UNITS, 64, LDS_FOLD, c->stream>>>(m, c->vm_fold, c->vm_consts,
                                                                                       F, S, o, nullptr);
    F = o;
    S = Slab{base + (size_t)12 * 12 * c->red_cap, c->red_cap};
    m = mo;
    flip ^= 1;
  }
  enqueue_final(c, c->stream, F, S, m, c->result + RES_SYNC);
  if (hipGetLastError() != hipSuccess) return -OVH_ERR_DEVICE;
  int32_t r = -1;
  if (hipMemcpyAsync(&r, c->result + RES_SYNC, 4, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
      hipStreamSynchronize(c->stream) != hipSuccess)
    return -OVH_ERR_DEVICE;
  return r;
}

int ovh_batch_fallback_device(ovh_ctx* c, size_t n, int32_t* d_codes) {
  if (!c || !d_codes) return OVH_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  if (n == 0) return 0;
  if (n != c->last_n) return OVH_ERR_ARG;
  enqueue_fallback(c, c->stream, c->last_slot, (uint32_t)n, d_codes, nullptr);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int ovh_combine_partials_device_async(ovh_ctx* c, size_t k, const uint8_t* d_partials, size_t n, int32_t* d_codes) {
  if (!c || !d_partials || k == 0 || k > 16 || (n && !d_codes)) return OVH_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  if (n != c->last_n) return OVH_ERR_ARG;
  const int slot = c->last_slot;
  // the partials were produced (and gathered) before this call returned to the host
  uint32_t* scratch = c->fin + (size_t)slot * FIN_STRIDE;
  Slab F, S;
  uint32_t m;
  if (stage_partials(c, c->fstream, k, d_partials, scratch, &F, &S, &m)) return OVH_ERR_DEVICE;
  int32_t* verdict = c->result + RES_COMBINE + slot;
  enqueue_final(c, c->fstream, F, S, m, verdict);
  if (n) enqueue_fallback(c, c->fstream, slot, (uint32_t)n, d_codes, verdict);
  HIPCHK(hipEventRecord(c->ev_back[slot], c->fstream));
  HIPCHK(hipGetLastError());
  return 0;
}

int ovh_verify_batch_device_async(ovh_ctx* c, size_t n, const uint8_t* d_sigs, const uint8_t* d_hashes,
                                  const uint8_t* d_pks, uint64_t seed, int32_t* d_codes) {
  if (!c || (n && (!d_sigs || !d_hashes || !d_pks || !d_codes))) return OVH_ERR_ARG;
  if (n == 0) return 0;
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  if (ensure_cap(c, n)) return OVH_ERR_DEVICE;
  const int slot = (int)(c->pipe_k++ % OVH_BATCH_SLOTS);
  if (take_slot(c, slot)) return OVH_ERR_DEVICE;
  Slab F, S;
  uint32_t m;
  int e = batch_front(c, (uint32_t)n, d_sigs, d_hashes, d_pks, seed, d_codes, &F, &S, &m, slot);
  if (e) return e;
  // fold levels: the wide ones on the main stream (short, high priority), the narrow ones and
  // the combined check + fallback on the final stream -- balancing the two streams' chains
  int flip = 1;
  if ((e = fold_levels(c, c->stream, VM_SLICES, &F, &S, &m, 64, &flip))) return e;
  HIPCHK(hipEventRecord(c->ev_front[slot], c->stream));
  HIPCHK(hipStreamWaitEvent(c->fstream, c->ev_front[slot], 0));
  if ((e = fold_levels(c, c->fstream, 1, &F, &S, &m, 4, &flip))) return e;
  int32_t* verdict = c->result + RES_BATCH + slot;
  enqueue_final(c, c->fstream, F, S, m, verdict);
  enqueue_fallback(c, c->fstream, slot, (uint32_t)n, d_codes, verdict);
  HIPCHK(hipEventRecord(c->ev_back[slot], c->fstream));
  HIPCHK(hipGetLastError());
  return 0;
}

int ovh_batch_wait(ovh_ctx* c) {
  if (!c) return OVH_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipStreamSynchronize(c->fstream));
  HIPCHK(hipStreamSynchronize(c->hstream));
  return 0;
}

int ovh_verify_batch_device(ovh_ctx* c, size_t n, const uint8_t* d_sigs, const uint8_t* d_hashes, const uint8_t* d_pks,
                            uint64_t seed, int32_t* d_codes) {
  int e = ovh_verify_batch_device_async(c, n, d_sigs, d_hashes, d_pks, seed, d_codes);
  return e ? e : ovh_batch_wait(c);
}

int ovh_verify_batch(ovh_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* hashes, const uint8_t* pks, uint64_t seed,
                     int32_t* codes) {
  if (!c || (n && (!sigs || !hashes || !pks || !codes))) return OVH_ERR_ARG;
  if (n == 0) return 0;
  if (n > (1u << 24)) return OVH_ERR_ARG;
  uint8_t* d = nullptr;
  {
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    if (ensure_in(c, n * (96 + 32 + 48 + 4))) return OVH_ERR_DEVICE;
    d = c->in_buf;
    HIPCHK(hipMemcpyAsync(d, sigs, n * 96, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(d + n * 96, hashes, n * 32, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(d + n * 128, pks, n * 48, hipMemcpyHostToDevice, c->stream));
  }
  int32_t* dc = (int32_t*)(d + n * 176);
  int e = ovh_verify_batch_device(c, n, d, d + n * 96, d + n * 128, seed, dc);
  if (e) return e;
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipMemcpyAsync(codes, dc, 4 * n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int ovh_sign_batch_device(ovh_ctx* c, size_t n, const uint8_t* d_sks, const uint8_t* d_hashes, uint8_t* d_sigs) {
  if (!c || (n && (!d_sks || !d_hashes || !d_sigs))) return OVH_ERR_ARG;
  if (n == 0) return 0;
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  k_sign<<<nblk(n), WG, 0, c->stream>>>((uint32_t)n, d_sks, d_hashes, c->xmd, d_sigs);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int ovh_sk_to_pk_batch_device(ovh_ctx* c, size_t n, const uint8_t* d_sks, uint8_t* d_pks) {
  if (!c || (n && (!d_sks || !d_pks))) return OVH_ERR_ARG;
  if (n == 0) return 0;
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  k_sk_to_pk<<<nblk(n), WG, 0, c->stream>>>((uint32_t)n, d_sks, d_pks);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

}  // extern "C"
