// libovhip: HIP (gfx950) implementation of the C ABI in include/ovhip.h.
//
// Batch verification (ovh_verify_batch_device), DESIGN.md section 4:
//   k_h2f         lane per vote: expand_message_xmd (SHA-256) + hash_to_field -> u0, u1
//   k_vm_vote     16-lane slice per vote, 4 votes per wave: the Fp-VM "vote" program --
//                 pk / sig decompression + subgroup checks, hash_to_G2, r pk,
//                 f = Miller(r pk, H), sigma and tau = -psi^2(sigma) stored for the MSM; the
//                 epilogue writes the vote's code with the reference precedence, then folds
//                 the workgroup's 4 votes' f into one partial (level 0; 1 if the vote failed)
//   k_vm_vote_t   the same with the public key from the device validator table (or a QC's
//                 aggregated key): no decompression / subgroup check of the key
//                 (both programs keep <= 90 values in LDS and spill the rest to a per-vote
//                 scratch through side words, so a CU holds eight vote workgroups: pipelined
//                 batches put their vote grids on two streams in turn and two co-reside)
//   k_vm_fold     fold levels: 4 partials -> (prod f, sum S); level 1 = groups of 16 votes
//   k_msm_*       Pippenger MSM of S = sum r_i sigma_i (msm.hpp), on the final stream
//   k_vm_final    one wave: prod f * Miller(-G1, S) -> final exponentiation == 1 ?
//   bisection, only when the combined check failed (device-gated):
//   k_vm_rs       per vote r_i sigma_i (the MSM's terms), then fold levels 0-1 of (f, r sigma)
//   k_vm_group    the same check per 16-vote group
//   k_vm_votechk  per vote of a failing group: f_i * Miller(-G1, r_i sigma_i) == 1
// Per-vote state lives in HBM as structure-of-arrays by limb: limb k of element i of an Fp
// plane j at slab[(j * 12 + k) * cap + i].
#include <hip/hip_runtime.h>

#include <errno.h>
#include <stdlib.h>
#include <sys/random.h>
#include <sys/types.h>

#include <algorithm>
#include <atomic>
#include <deque>
#include <mutex>
#include <new>
#include <string>
#include <string.h>
#include <unordered_map>
#include <vector>

#include "../../include/ovhip.h"
#include "bls/verify.hpp"
#include "fpvm.hpp"
#include "keygen.hpp"
#include "rlp.hpp"
#include "sm3.hpp"
#ifdef OVH_VM_PROGS
#include OVH_VM_PROGS  // A/B builds: another generation of the programs
#else
#include <vm_progs.inc>  // generated (tools/fpvm/gen.py): -Icsrc (Makefile) or -I OUT_DIR (overlord-hip/build.rs)
#endif
static_assert(VM_KZERO == ovh::vm::KZERO && VM_KTAB == ovh::vm::KTAB, "fixed constants (tools/fpvm/gen.py)");

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
  S_SIG = VM_S_SIG,   // 4 planes: sigma (affine)
  S_TAU = VM_S_TAU,   // 4 planes: tau = -psi^2(sigma) (affine)
  S_F = VM_S_F,       // 12 planes: f = Miller(r pk, H)
  S_RS = VM_S_RS,     // 6 planes: r * sig (projective; bisection only, k_vm_rs)
  S_TOTAL = VM_S_TOTAL,
};
// partial = (F: 12 planes, S: 6 planes)
constexpr uint32_t PART_PLANES = 18;
// words per fin region: 16 unpacked + 4 folded partials as planes
constexpr size_t FIN_STRIDE = (size_t)PART_PLANES * 12 * 20;

enum : int { ST_H2F = 0, ST_VOTE, ST_FOLD, ST_FINAL, ST_FALLBACK, ST_MSM };
static_assert(ST_MSM + 1 == OVH_NSTAGES, "stage table");

__device__ __forceinline__ uint64_t rlc_scalar(uint64_t seed, uint64_t i) {
  // SplitMix64 on (seed, i): the 64-bit RLC coefficient of vote i (never 0). The seed is a
  // fresh secret per batch (getrandom, host side), so the coefficients are unpredictable.
  uint64_t z = seed + 0x9e3779b97f4a7c15ull * (i + 1);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  z = z ^ (z >> 31);
  return z ? z : 1;
}

// A batch of one vote checks its own pairing equation, e(pk, H) e(-G1, sigma) = 1: no random
// coefficient is needed, so its scalar is 1 (base UNIT_BASE) and the "MSM" is sigma itself
// (k_sig_as_S), which saves the MSM's launches on the per-call path (ovh_verify).
#define UNIT_BASE 0xFFFFFFFFFFFFFFFFull
__device__ __forceinline__ uint64_t vote_scalar(uint64_t seed, uint64_t base, uint64_t i) {
  return base == UNIT_BASE ? 1ull : rlc_scalar(seed, base + i);
}

// ------------------------------------------------------------------------ kernels
// Vote digests (ovh_vote_digests*): lane per vote, rlp(Vote) + SM3 (rlp.hpp, sm3.hpp).
__global__ __launch_bounds__(WG) void k_vote_digest(uint32_t n, const uint64_t* __restrict__ heights,
                                                    const uint64_t* __restrict__ rounds,
                                                    const uint8_t* __restrict__ types, const uint8_t* __restrict__ bh,
                                                    const uint8_t* __restrict__ lens, uint8_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  uint8_t h[VOTE_HASH_MAX];
  const uint32_t len = lens[i];
  uint8_t d[32];
  if (len > VOTE_HASH_MAX) {
    // lengths live in device memory (ovh_vote_digests_device cannot reject them on the host):
    // an over-long block hash gets the all-zero digest, which no vote hash equals
    for (int k = 0; k < 32; ++k) out[(size_t)i * 32 + k] = 0;
    return;
  }
  for (uint32_t k = 0; k < len; ++k) h[k] = bh[(size_t)i * VOTE_HASH_MAX + k];
  vote_digest(d, heights[i], rounds[i], types[i], h, len);
  for (int k = 0; k < 32; ++k) out[(size_t)i * 32 + k] = d[k];
}

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
  uint64_t* clk;    // OVH_FLAG_VM_CLOCK (vote / vote_t): per workgroup (d memtime, d realtime), else null
  const uint32_t* side;  // spilled programs (vote / vote_t): per-lane side words (fpvm.hpp run), else null
};
// per-vote scratch of the spilled vote programs (tools/fpvm/gen.py SPILL_K): entries of 12 words
constexpr uint32_t VOTE_NSCR = VM_VOTE_NSCR > VM_VOTE_T_NSCR ? VM_VOTE_NSCR : VM_VOTE_T_NSCR;

// OVH_FLAG_VM_CLOCK: shader-cycle and 100 MHz stamps around a workgroup's program (diagnostic
// runs of the measurement only; a null pointer executes no stamp). Capacity: VM_CLOCK_WGS
// workgroups of one launch.
#define VM_CLOCK_WGS (1u << 16)
struct ClockStamp {
  uint64_t t0 = 0, r0 = 0;
  __device__ __forceinline__ void begin(const uint64_t* clk) {
    if (clk && threadIdx.x == 0) {
      t0 = __builtin_amdgcn_s_memtime();
      r0 = __builtin_amdgcn_s_memrealtime();
    }
  }
  __device__ __forceinline__ void end(uint64_t* clk) {
    if (clk && threadIdx.x == 0 && blockIdx.x < VM_CLOCK_WGS) {
      const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
      clk[2 * blockIdx.x] = t1 - t0;
      clk[2 * blockIdx.x + 1] = r1 - r0;
    }
  }
};

// Batches of at most SMALL_MAX votes (one vote per wave: 1,024 waves fill the chip's SIMDs)
// take the small-batch path: votew per vote, fold, one final exponentiation (verify_small_locked).
#ifndef SMALL_MAX
#define SMALL_MAX 1024u
#endif
#define VM_SLICES 4  // 16-lane slices per 64-lane workgroup (vote, vote_t)
// LDS layout of the VM kernels (words): the constant table, then slot regions that start on a
// 128-byte boundary and repeat at 128-byte strides, so slot s and constant c share LDS banks
// exactly when s = c (mod 8) -- the rule tools/fpvm/sched.py spreads operand reads by.
constexpr uint32_t align128w(uint32_t w) { return (w + 31) / 32 * 32; }
// 256-byte alignment (one LDS row of 64 banks): slot s of every slice and constant c then sit in
// bank groups (3 s) and (3 c) mod 16 -- the model tools/fpvm/sched.py allocates slots by. A
// ds_read_b128 lane group of a 16-lane program spans two slices ({0-3,12-15} of one and {4-11}
// of the next), which only share that model when the slice stride is a multiple of 256 B.
constexpr uint32_t align256w(uint32_t w) { return (w + 63) / 64 * 64; }
constexpr uint32_t SLOT_BASE_W = align256w(VM_NCONST * 12);
constexpr uint32_t VOTE_STRIDE_W = align256w(VM_VOTE_NSLOTS * 12 + 4);  // + 4 header words
constexpr uint32_t VOTE_T_STRIDE_W = align256w(VM_VOTE_T_NSLOTS * 12 + 4);
constexpr uint32_t FOLD_STRIDE_W = align128w(VM_FOLD_NSLOTS * 12);
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
// inS.p null: every S is the identity (the batch path's S is the MSM's, msm.hpp).
// All 64 threads of the workgroup call it (the phase barrier); `active` marks the working slice.
__device__ __forceinline__ void fold_unit(uint32_t t, uint32_t m, const VmDev& prog, const uint32_t* cst,
                                          uint32_t* slots, uint32_t lane, bool active, Slab inF, Slab inS,
                                          Slab out, const int32_t* __restrict__ codes) {
  if (active) {
    for (uint32_t k = lane; k < 4 * PART_PLANES; k += VM_FOLD_W) {
      const uint32_t q = k / PART_PLANES, j = k % PART_PLANES, e = 4 * t + q;
      Fp v;
      if (e < m && (!codes || codes[e] == 0) && (j < 12 || inS.p)) {
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
      vm::canon(v, v);  // slots hold [0, 2p) representatives (fpvm.hpp); planes are canonical
      out.st(v, k, t);
    }
  }
}

// The vote waves of a CU run the same program in near lockstep, so every phase's operand loads
// (12 KB per wave) reach the CU's LDS at the same moment. OVH_VOTE_STAGGER > 0 offsets the start
// of the wave on SIMD s by s x OVH_VOTE_STAGGER x 64 cycles (the offset persists: every wave's
// phases take equally long), spreading those bursts. r03k A/B: 6 / 12 / 24 each +0.8-1.2%
// verifs/s against 0 (profiles/r03k_stagger_ab.txt); 12 is the default.
#ifndef OVH_VOTE_STAGGER
#define OVH_VOTE_STAGGER 12
#endif
__device__ __forceinline__ void vote_stagger() {
#if OVH_VOTE_STAGGER > 0
  const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_REG_HW_ID, all 32 bits
  const uint32_t n = ((hw >> 4) & 3) * OVH_VOTE_STAGGER;          // SIMD_ID
#pragma unroll 1
  for (uint32_t k = 0; k < n; ++k) __builtin_amdgcn_s_sleep(1);
#endif
}

// Public keys given as points (ovh_set_validators table, or a QC's aggregated key): planes
// X, Y, Z (homogeneous projective, Montgomery) of `cap` entries, plus per-entry flags.
#define PKF_PARSE 1u  // the 48 bytes did not parse -> "lose public key" (102)
#define PKF_INF 2u    // the point at infinity      -> BLST_PK_IS_INFINITY (6) at verify
#define PKF_GRP 4u    // not in G1                  -> BLST_POINT_NOT_IN_GROUP (3) at verify
struct PkSrc {
  const uint32_t* planes;
  uint32_t cap;
  const uint32_t* flags;
  const int32_t* idx;  // vote i uses entry idx[i] (null: entry i)
};

// ------------------------------------------------------------------------ the vote pool
// The per-vote work of every batch ("Vote pool"). A batch is published to a
// device queue as a descriptor; the pool kernel's workgroups (one wave each, four 16-lane vote
// slices) claim 4-vote quads from the queue in publication order -- across batches -- and run
// the "vote" / "vote_t" program on each, so a workgroup that finishes batch k's quad takes batch
// k + 1's at once: no grid boundary, no per-grid tail, no stream-order wait between batches. One
// pool grid is launched (on the pool stream) after each publication, which guarantees that some
// grid runs after the batch appeared; a workgroup exits when the queue is empty, so the grid
// launched for batch k + 1 usually finds batch k's grid still working and its own workgroups do
// nothing. A batch's final stream waits for its quads with k_pool_wait (done counter).
//
// Queue words (uint64, each on its own 128-byte line): cur = the oldest batch that may still have
// unclaimed quads; npub = batches published; slot_of[seq % POOL_SEQR] = the batch slot of batch
// seq; per slot, claim = (seq << 32) | quads claimed of the slot's batch and done = quads
// completed. A workgroup claims with ONE fetch-add on the claim word of batch cur's slot (no
// compare-and-swap window: r05a's CAS on a shared cursor handed out one quad per ~25 us). The
// claim word carries the batch it counts for, so a claim through a stale cur / slot_of is still
// exact: it is quad `count` of batch `seq` (processed iff count < that batch's nq, after its
// publication). Batches take batch slots (take_slot) and a slot is reused only after its batch
// completed; every quad a workgroup claimed below nq is processed, so a slot is never
// republished under a workgroup that holds one of its quads.
#define POOL_SEQR 16u
#define POOL_QW 16u  // uint64 words per 128-byte line
enum : uint32_t {
  PQ_CUR = 0,
  PQ_NPUB = POOL_QW,
  PQ_SLOTOF = 2 * POOL_QW,
  PQ_NANN = 3 * POOL_QW,
  PQ_DONE = 4 * POOL_QW,
  PQ_CLAIM = PQ_DONE + OVH_BATCH_SLOTS * POOL_QW,
  PQ_INFL = PQ_CLAIM + OVH_BATCH_SLOTS * POOL_QW,  // quads claimed and not yet done (all batches)
  PQ_OCC = PQ_INFL + POOL_QW,  // POOL_OCC_N uint32: pool quads running on each SIMD (simd_key)
};
constexpr uint32_t POOL_OCC_N = 4096;
constexpr uint32_t PQ_WORDS = PQ_OCC + POOL_OCC_N / 2;
static_assert(POOL_SEQR > OVH_BATCH_SLOTS && POOL_SEQR / 2 <= POOL_QW, "pool queue layout");
// A workgroup that finds the queue empty polls it for POOL_IDLE_TICKS (20 us) before it exits --
// or, while a batch is announced but not yet published (nann > npub: its staging and
// hash_to_field are on ovh_stream) or another workgroup still runs a quad (infl > 0: more batches
// are likely on their way), for up to POOL_WAIT_TICKS (20 ms). A grid whose spare workgroups left
// while the rest kept working holds its stream (the next batches' grids queue behind it), and the
// pool ran on the 1,024 workgroups that had found a quad: r05h without the announcement; r05x
// (pool log) with it, the host still enqueueing batch k's final stream 50 us after batch k's
// publication, before it announced batch k + 1.
#define POOL_IDLE_TICKS 2000ull
#define POOL_WAIT_TICKS 2000000ull

// The SIMD a wave runs on, as a 12-bit key: XCC (3 bits) | SE (2) | SA (1) | CU (4) | SIMD (2) from
// HW_REG_XCC_ID and HW_REG_HW_ID (amd_device_functions.h bit layout for gfx950); the pool log
// records it per quad (ovh_pool_log, tools/pool_timeline.py)
__device__ __forceinline__ uint32_t simd_key() {
  const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID, all 32 bits
  const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);  // HW_REG_XCC_ID bits 3:0
  return (xcc & 7u) << 9 | ((hw >> 13) & 3u) << 7 | ((hw >> 12) & 1u) << 6 | ((hw >> 8) & 15u) << 2 |
         ((hw >> 4) & 3u);
}
__device__ __forceinline__ uint32_t* pq_occ(uint64_t* q) { return reinterpret_cast<uint32_t*>(q + PQ_OCC); }
// SIMD spreading: while the current batch is the last published and its unclaimed quads fit the
// SIMDs that run no pool quad (estimate: SIMDs - quads in flight), a workgroup whose SIMD already
// runs a pool quad leaves the claim to one on an idle SIMD for up to POOL_SPREAD_TICKS (200 us):
// a lone batch's 1,024 quads then take 1,024 SIMDs (two quads on a SIMD take 4.6-5.6 ms, one
// 3.8, r05az) -- with the pool's grids dealt one wave per SIMD (pool_grid0)
#define POOL_SPREAD_TICKS 20000ull

struct PoolBatch {  // one published batch (written by k_pool_publish, read by the pool)
  uint64_t seq;          // its sequence number (written last: a claimer checks it, pool_claim)
  uint32_t n, nq;
  uint32_t table;        // 1: keys are points (program vote_t), 0: n x 48 compressed bytes (vote)
  uint32_t has_idx;      // vote_t: vote i uses table entry idx[i] (staged after the keys), else i
  uint64_t seed, base;   // RLC coefficients (vote_scalar)
  int32_t* codes;
  const uint32_t* planes;  // vote_t: key points (X, Y, Z planes of `pcap` entries) and flags
  const uint32_t* flags;
  uint32_t pcap, cap;    // cap: the state slab's
  uint32_t* state;       // the slot's state slab (u planes in; sigma, tau, f planes out)
  uint32_t* part0;       // fold region R0 (one partial per quad) of `part_cap` entries
  const uint8_t* stage;  // staged signatures | keys | table indices (k_pool_stage)
  uint64_t* clk;         // OVH_FLAG_VM_CLOCK: per-workgroup stamps, else null
  uint32_t part_cap, pad;
  uint64_t* plog;        // OVH_FLAG_VM_CLOCK: this batch's pool-log record (ovh_pool_log), else null
};

// Pool log (OVH_FLAG_VM_CLOCK diagnostics, ovh_pool_log): a ring of PLOG_RING batch records of
// PLOG_WORDS u64: [0..15] 100 MHz stamps of the batch's stream events (PLOG_EV_*) and its seq,
// then per quad (< PLOG_QUADS) its start (bits 0..47) with the SIMD it ran on (simd_key, bits 48..59), the
// claim flags (pool_claim, bits 60..63) and end.
#define PLOG_RING 64u
#define PLOG_QUADS 1024u
#define PLOG_WORDS (16u + 2u * PLOG_QUADS)
// then per pool grid launch (a ring of PLOG_GRIDS) and workgroup (< PLOG_WGS): entry and exit
// stamps, the quads it ran and how it left (1: idle with nothing announced, 2: POOL_WAIT_TICKS,
// 3: the claim loop's bound)
#define PLOG_GRIDS 64u
#define PLOG_WGS 1024u
#define PLOG_WG_WORDS 4u
#define PLOG_GRID_BASE ((size_t)PLOG_RING * PLOG_WORDS)
#define PLOG_TOTAL (PLOG_GRID_BASE + (size_t)PLOG_GRIDS * (4 + PLOG_WGS * PLOG_WG_WORDS))
// (the shard path's combine: GATH on the caller's stream when ovh_combine_partials_device_async is
// called -- after its all-gather --, COMB once the final stream read the partials, FE after the
// combined check's final exponentiation)
enum : uint32_t { PLOG_EV_PUB = 0, PLOG_EV_DONE = 1, PLOG_EV_FOLD = 2, PLOG_EV_MSM = 3, PLOG_EV_FINAL = 4,
                  PLOG_EV_BACK = 5, PLOG_EV_GATH = 6, PLOG_EV_COMB = 7, PLOG_EV_FE = 8, PLOG_EV_SEQ = 15 };
__global__ void k_grid_hdr(uint64_t* g, uint64_t seq, uint32_t par, uint32_t wgs) {
  for (uint32_t k = threadIdx.x; k < PLOG_WGS * PLOG_WG_WORDS; k += blockDim.x) g[4 + k] = 0;
  __syncthreads();
  if (threadIdx.x == 0) {
    g[0] = seq;
    g[1] = par;
    g[2] = wgs;
    g[3] = __builtin_amdgcn_s_memrealtime();  // its launch point on the pool stream
  }
}
__global__ void k_stamp(uint64_t* p, uint64_t v) {
  if (threadIdx.x == 0) {
    p[0] = __builtin_amdgcn_s_memrealtime();
    if (v != ~0ull) p[PLOG_EV_SEQ] = v;
  }
}

// The pool kernel's arguments: the queue, the descriptors, the two vote programs' instruction
// and side-word streams, the fold program, the constant table and the spill scratch. Everything
// per batch is in the descriptor and read where it is used.
struct PoolArgs {
  uint64_t* q;
  const PoolBatch* descs;
  const uint4* pv_code;
  const uint32_t* pv_side;
  const uint4* pt_code;
  const uint32_t* pt_side;
  const uint4* fold_code;
  const uint32_t* cst;
  uint32_t* scr;  // VM_SLICES x VOTE_NSCR entries per workgroup
  uint64_t* wlog;  // OVH_FLAG_VM_CLOCK: this grid's workgroup log (PLOG_WG_WORDS per workgroup), else null
  uint64_t only;   // ~0: claim any batch; else this grid's own batch: its workgroups leave once
                   // `cur` has passed it (the shard path's grid per batch, ovh_batch_partial_device)
  uint32_t nsimd;  // SIMDs the pool runs on (SIMD spreading, pool_claim)
  uint32_t skip_cu;  // OVH_FLAG_POOL_RESERVE: workgroups on CUs 0 .. skip_cu - 1 of SE 0 / SA 0 of
                     // every XCC leave at once (those CUs stay free for other kernels); 0: none
};

__device__ __forceinline__ uint64_t* pq_done(uint64_t* q, uint32_t slot) { return q + PQ_DONE + slot * POOL_QW; }
__device__ __forceinline__ uint64_t* pq_claim(uint64_t* q, uint32_t slot) { return q + PQ_CLAIM + slot * POOL_QW; }
__device__ __forceinline__ uint32_t* pq_slot_of(uint64_t* q) { return reinterpret_cast<uint32_t*>(q + PQ_SLOTOF); }
__device__ __forceinline__ uint64_t qld(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Publish batch `seq` in slot `slot` (one lane; ovh_stream, after the batch's hash_to_field and
// staging): the descriptor, then (behind a release) its seq, done = 0, the claim word and
// slot_of, then (behind a release) npub.
__global__ __launch_bounds__(64) void k_pool_publish(PoolBatch b, uint32_t slot, uint64_t seq, uint64_t* q,
                                                     PoolBatch* descs) {
  if (threadIdx.x) return;
  b.seq = ~0ull;
  descs[slot] = b;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_store(&descs[slot].seq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(pq_done(q, slot), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(pq_claim(q, slot), seq << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(pq_slot_of(q) + seq % POOL_SEQR, slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (MI355X_MICROARCH.md: the wait the compiler may drop)
  __hip_atomic_store(q + PQ_NPUB, seq + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Announce batch seq: nann = seq + 1 tells idle pool workgroups that a publication is on its way
// (pool_take_slot: on ovh_stream ahead of the slot wait, so the announcement of the next batch
// follows the publication of the previous one and never waits for a slot).
__global__ __launch_bounds__(64) void k_pool_announce(uint64_t* q, uint64_t n) {
  if (threadIdx.x == 0) __hip_atomic_store(q + PQ_NANN, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Claim the next quad (the whole wave, in wave-uniform control flow: every lane reads the same
// queue words, lane 0 alone performs the atomics and the result is broadcast -- r05c ran the
// claim loop in a lane-0 branch, and the workgroup's later quads ran with lane 0 alone active).
// Returns 1 and the quad's slot and index, or 0 when the queue stays empty for
// POOL_IDLE_TICKS. Every quad is handed out by exactly one fetch-add on its batch's claim word; a
// claim past the batch's nq moves `cur` on.
__device__ __forceinline__ uint64_t lane0_fetch_add(uint64_t* p, uint64_t v) {
  uint64_t r = 0;
  if (threadIdx.x == 0) r = __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(r >> 32)) << 32) |
         __builtin_amdgcn_readfirstlane((uint32_t)r);
}
__device__ __forceinline__ uint32_t lane0_fetch_add32(uint32_t* p, uint32_t v) {
  uint32_t r = 0;
  if (threadIdx.x == 0) r = __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return __builtin_amdgcn_readfirstlane(r);
}
__device__ __forceinline__ void lane0_cas(uint64_t* p, uint64_t expect, uint64_t want) {
  if (threadIdx.x == 0) {
    uint64_t e = expect;
    (void)__hip_atomic_compare_exchange_strong(p, &e, want, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
  }
}
__device__ __forceinline__ uint64_t wclock() {
  const uint64_t t = wall_clock64();
  return ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(t >> 32)) << 32) | __builtin_amdgcn_readfirstlane((uint32_t)t);
}
__device__ __forceinline__ uint64_t qldu(const uint64_t* p) {
  const uint64_t v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) | __builtin_amdgcn_readfirstlane((uint32_t)v);
}
__device__ uint32_t pool_claim(uint64_t* q, const PoolBatch* descs, uint32_t* slot_out, uint32_t* quad_out,
                               uint32_t* why, uint64_t only, uint32_t nsimd, uint32_t* how) {
  uint64_t t0 = wclock(), tdef = 0;
  uint32_t hw = 0;  // how the claim went (pool log): 1 last published, 2 SIMD busy, 4 deferred, 8 busy and not deferred
  uint32_t* occ = pq_occ(q) + simd_key();
  *why = 3;
#pragma unroll 1
  for (uint32_t tries = 0; tries < (1u << 22); ++tries) {
    const uint64_t s = qldu(q + PQ_CUR), np = qldu(q + PQ_NPUB);
    if (s > only) {  // a grid of one batch: that batch is fully claimed
      *why = 4;
      return 0;
    }
    if (s >= np) {
      const uint64_t idle = wclock() - t0;
      if (idle > POOL_WAIT_TICKS ||
          (idle > POOL_IDLE_TICKS && qldu(q + PQ_NANN) <= np && qldu(q + PQ_INFL) == 0)) {
        *why = idle > POOL_WAIT_TICKS ? 2 : 1;
        return 0;
      }
      // past the idle window, poll ~16x less often: 1,700 waiting workgroups polling two queue
      // words every ~0.2 us kept a shard batch's all-gather and combine from running while the
      // pool waited for that batch's slot (r06i / r06j pool logs: 20 ms stalls)
      if (idle > POOL_IDLE_TICKS) __builtin_amdgcn_s_sleep(127);
      else __builtin_amdgcn_s_sleep(8);
      continue;
    }
    const uint32_t slot = __builtin_amdgcn_readfirstlane(
        __hip_atomic_load(pq_slot_of(q) + s % POOL_SEQR, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    // SIMD spreading: this SIMD's occupancy is taken first (one fetch-add, so two workgroups of a
    // SIMD polling the same publication cannot both see it idle), then the claim is deferred
    // while the SIMD was busy
    bool held = false;
    if (np == s + 1) {
      hw |= 1u;
      bool busy;
      if (tdef && __builtin_amdgcn_readfirstlane(__hip_atomic_load(occ, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
        busy = true;  // deferring: a plain load while the SIMD stays busy
      } else {
        busy = lane0_fetch_add32(occ, 1u) != 0;
        held = true;
      }
      if (busy) {
        hw |= 2u;
        const uint64_t cw = qldu(pq_claim(q, slot));
        const uint32_t nq = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(&descs[slot].nq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        const uint64_t infl = qldu(q + PQ_INFL);
        const uint32_t taken = (uint32_t)cw;
        // (a slack of nsimd / 16: at nsimd exactly, a lone batch's late arrivals claimed next to a
        // running quad instead of deferring -- pool-log claim flags 11, r05bj)
        if ((cw >> 32) == s && taken < nq && (uint64_t)(nq - taken) + infl <= nsimd + nsimd / 16) {
          const uint64_t now = wclock();
          if (!tdef) tdef = now;
          if (now - tdef < POOL_SPREAD_TICKS) {
            hw |= 4u;
            if (held) (void)lane0_fetch_add32(occ, ~0u);
            __builtin_amdgcn_s_sleep(32);
            continue;
          }
        }
        hw |= 8u;
      }
    }
    if (!held) (void)lane0_fetch_add32(occ, 1u);
    const uint64_t old = lane0_fetch_add(pq_claim(q, slot), 1ull);
    const uint64_t seq = old >> 32;
    const uint32_t idx = (uint32_t)old;
    // the claim counts for batch `seq` (a stale slot_of may have led here): wait for its publication
    const uint64_t tw = wclock();
    while (qldu(q + PQ_NPUB) <= seq && wclock() - tw < 100000000ull) __builtin_amdgcn_s_sleep(2);
    const uint32_t nq = __builtin_amdgcn_readfirstlane(
        __hip_atomic_load(&descs[slot].nq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint64_t dseq = qldu(&descs[slot].seq);
    // dseq != seq: the slot was republished, so batch seq completed -- every quad of it below nq
    // was claimed by others, this one is past its end
    const bool mine = dseq == seq && idx < nq;
    // batch s is fully claimed when this claim went past its end, or when its slot already holds
    // a later batch (seq != s: a slot is republished only after its batch completed): move cur on
    // (whoever wins; a claim that took exactly the last quad does not, the next claimer does)
    if (seq != s || !mine) lane0_cas(q + PQ_CUR, s, s + 1);
    if (mine) {
      (void)lane0_fetch_add(q + PQ_INFL, 1ull);
      *slot_out = slot;
      *quad_out = idx;
      *how = hw;
      return 1;
    }
    (void)lane0_fetch_add32(occ, ~0u);  // - 1: no quad after all
    tdef = 0;
    t0 = wclock();  // progress: the idle window restarts
  }
  return 0;
}

// Descriptor fields are read where they are used (relaxed agent-scope loads: vector loads, never
// the scalar cache), so no batch state stays live across the VM program: the vote program
// already needs every VGPR of a two-waves-per-SIMD budget and most SGPRs.
template <typename T>
__device__ __forceinline__ T dget(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ T* dgetp(T* const* p) {
  return reinterpret_cast<T*>(__hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return ((uint64_t)uni((uint32_t)(v >> 32)) << 32) | uni((uint32_t)v);
}
template <typename T>
__device__ __forceinline__ T* unip(T* p) {
  return reinterpret_cast<T*>(uni64(reinterpret_cast<uint64_t>(p)));
}

// One quad of a batch: votes 4 quad .. 4 quad + 3 on the four slices -- inputs, the vote / vote_t
// program, the per-vote code in the reference's precedence, then fold level 0 of the quad's f
// (fused: -> partial `quad` of R0, the identity for failed votes). Only the VM's own operands
// stay in registers across the program: the slot and quad wait in the LDS header words of slice
// 2 and the clock stamps (OVH_FLAG_VM_CLOCK) in those of slices 0 and 1.
template <bool TABLE>
__device__ __forceinline__ void vote_quad(const PoolArgs& a, uint32_t slot_in, uint32_t quad_in, uint32_t* lds) {
  constexpr uint32_t NSLOTS = TABLE ? VM_VOTE_T_NSLOTS : VM_VOTE_NSLOTS;
  constexpr uint32_t STRIDE = TABLE ? VOTE_T_STRIDE_W : VOTE_STRIDE_W;
  constexpr uint32_t NPH = TABLE ? VM_VOTE_T_NPHASES : VM_VOTE_NPHASES;
  const uint16_t* IN = TABLE ? VM_VOTE_T_IN : VM_VOTE_IN;
  const uint16_t* OUT = TABLE ? VM_VOTE_T_OUT : VM_VOTE_OUT;
  uint32_t* cst = lds;
  const uint32_t slice = threadIdx.x / VM_VOTE_W, lane = threadIdx.x % VM_VOTE_W;
  uint32_t* slots = lds + SLOT_BASE_W + slice * STRIDE;
  uint32_t* hdr = slots + NSLOTS * 12;  // [sig flags, pk flags, (slice 0..2: stamps, slot, quad)]
  uint32_t* park = lds + SLOT_BASE_W + 2 * STRIDE + NSLOTS * 12 + 2;  // slice 2's hdr[2..3]
  {
    const PoolBatch* bd = a.descs + slot_in;
    const uint32_t i = (quad_in & 0x0FFFFFFFu) * VM_SLICES + slice;  // (top bits: the claim flags)
    const uint32_t n = uni(dget(&bd->n));
    const bool active = i < n;
    const uint8_t* sigs = unip(dgetp(&bd->stage));
    const Slab s{unip(dgetp(&bd->state)), uni(dget(&bd->cap))};
    if (active) {
      if (lane == 0) {
        uint32_t x1[12], x0[12], bad, inf, sort, xz;
        parse_hdr(sigs + (size_t)i * 96, 96, x1, x0, bad, inf, sort, xz);
        slot_put(slots, IN[TABLE ? VM_VOTE_T_IN_SIG_X1 : VM_VOTE_IN_SIG_X1], x1);
        slot_put(slots, IN[TABLE ? VM_VOTE_T_IN_SIG_X0 : VM_VOTE_IN_SIG_X0], x0);
        slot_flag(slots, IN[TABLE ? VM_VOTE_T_IN_SIG_SORT : VM_VOTE_IN_SIG_SORT], sort);
        hdr[0] = bad | inf << 1 | xz << 2;
      } else if (lane >= 2 && lane < 6) {
        Fp u;
        s.ld(u, S_U + (lane - 2), i);
        slot_put(slots, IN[(TABLE ? VM_VOTE_T_IN_U00 : VM_VOTE_IN_U00) + (lane - 2)], u.v);
      }
    }
    if (threadIdx.x == 0) {
      park[0] = slot_in;
      park[1] = quad_in;
      if (dgetp(&bd->plog)) {
        uint32_t* h3 = lds + SLOT_BASE_W + 3 * STRIDE + NSLOTS * 12 + 2;
        const uint64_t t = __builtin_amdgcn_s_memrealtime();
        h3[0] = (uint32_t)t;
        h3[1] = (uint32_t)(t >> 32);
      }
    }
    __syncthreads();
    if (active) {
      if constexpr (TABLE) {
        const int32_t* idx = reinterpret_cast<const int32_t*>(sigs + (size_t)n * 144);
        const uint32_t e = uni(dget(&bd->has_idx)) ? (uint32_t)idx[i] : i;
        if (lane == 1) {
          hdr[1] = unip(dgetp(&bd->flags))[e];
        } else if (lane >= 6 && lane < 9) {
          Fp v;
          Slab{const_cast<uint32_t*>(unip(dgetp(&bd->planes))), uni(dget(&bd->pcap))}.ld(v, lane - 6, e);
          slot_put(slots, IN[VM_VOTE_T_IN_PK_X + (lane - 6)], v.v);
        }
      } else {
        if (lane == 1) {
          uint32_t x[12], bad, inf, sort, xz;
          parse_hdr(sigs + (size_t)n * 96 + (size_t)i * 48, 48, x, x, bad, inf, sort, xz);
          slot_put(slots, IN[VM_VOTE_IN_PK_X], x);
          slot_flag(slots, IN[VM_VOTE_IN_PK_SORT], sort);
          hdr[1] = bad | inf << 1 | xz << 2;
        }
      }
    }
    if (threadIdx.x == 0 && dgetp(&bd->clk)) {
      const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
      uint32_t* h0 = lds + SLOT_BASE_W + NSLOTS * 12 + 2;
      uint32_t* h1 = lds + SLOT_BASE_W + STRIDE + NSLOTS * 12 + 2;
      h0[0] = (uint32_t)t0;
      h0[1] = (uint32_t)(t0 >> 32);
      h1[0] = (uint32_t)r0;
      h1[1] = (uint32_t)(r0 >> 32);
    }
    __syncthreads();
    const uint64_t scalar = vote_scalar(uni64(dget(&bd->seed)), uni64(dget(&bd->base)), i);
    vm::run<true>(TABLE ? a.pt_code : a.pv_code, NPH, VM_VOTE_W, lane, active, slots, cst, scalar,
                  vm::Out{s.p, s.cap, i}, nullptr, TABLE ? a.pt_side : a.pv_side,
                  a.scr + (size_t)blockIdx.x * VM_SLICES * VOTE_NSCR * 12 + slice * VOTE_NSCR * 12);
  }
  // after the program: the slot and quad back from LDS (run ends with an LDS wait + barrier)
  const uint32_t slot = uni(park[0]), quad = uni(park[1]) & 0x0FFFFFFFu, how = uni(park[1]) >> 28;
  const PoolBatch* bd = a.descs + slot;
  const uint32_t i = quad * VM_SLICES + slice;
  const uint32_t n = uni(dget(&bd->n));
  int32_t* codes = unip(dgetp(&bd->codes));
  if (uint64_t* clk = dgetp(&bd->clk); clk && threadIdx.x == 0 && blockIdx.x < VM_CLOCK_WGS) {
    const uint32_t* h0 = lds + SLOT_BASE_W + NSLOTS * 12 + 2;
    const uint32_t* h1 = lds + SLOT_BASE_W + STRIDE + NSLOTS * 12 + 2;
    const uint64_t t0 = h0[0] | (uint64_t)h0[1] << 32, r0 = h1[0] | (uint64_t)h1[1] << 32;
    clk[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
    clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
  if (i < n && lane == 0) {
    const uint32_t sf = hdr[0], pf = hdr[1];
    const uint32_t sg_bad = sf & 1, sg_inf = (sf >> 1) & 1, sg_xz = (sf >> 2) & 1;
    const uint32_t sg_ok = slot_flag_get(slots, OUT[TABLE ? VM_VOTE_T_OUT_SIG_OK : VM_VOTE_OUT_SIG_OK]);
    const uint32_t sg_grp = slot_flag_get(slots, OUT[TABLE ? VM_VOTE_T_OUT_SIG_GRP : VM_VOTE_OUT_SIG_GRP]);
    const uint32_t h_inf = slot_flag_get(slots, OUT[TABLE ? VM_VOTE_T_OUT_H_INF : VM_VOTE_OUT_H_INF]);
    // consensus.rs:397-416: pk parse (102) > sig parse (1..3) > [core_verify] sig group (3) >
    // pk infinity (6) > pk group (3) > H(m) = O or sig = O (5) > pairing (batch)
    uint32_t pk_parse, pk_inf, pk_grp;
    if constexpr (TABLE) {
      pk_parse = pf & PKF_PARSE;
      pk_inf = pf & PKF_INF;
      pk_grp = !(pf & PKF_GRP);
    } else {
      const uint32_t pk_bad = pf & 1, pk_xz = (pf >> 2) & 1;
      pk_inf = (pf >> 1) & 1;
      const uint32_t pk_ok = slot_flag_get(slots, OUT[VM_VOTE_OUT_PK_OK]);
      pk_grp = slot_flag_get(slots, OUT[VM_VOTE_OUT_PK_GRP]);
      pk_parse = pk_bad || (!pk_inf && (!pk_ok || pk_xz));
    }
    int32_t c;
    if (pk_parse) c = OVH_ERR_PUBKEY;
    else if (sg_bad) c = BLST_BAD_ENCODING;
    else if (!sg_inf && !sg_ok) c = BLST_POINT_NOT_ON_CURVE;
    else if (!sg_inf && (sg_xz || !sg_grp)) c = BLST_POINT_NOT_IN_GROUP;
    else if (pk_inf) c = BLST_PK_IS_INFINITY;
    else if (!pk_grp) c = BLST_POINT_NOT_IN_GROUP;
    else if (h_inf || sg_inf) c = BLST_VERIFY_FAIL;
    else c = 0;
    codes[i] = c;
  }
  // fold level 0, fused: the quad's 4 votes -> partial `quad` of R0 (F planes 0..11, S planes
  // 12..17), the identity for failed votes. The slices' `st` outputs (HBM) and codes are made
  // visible to the workgroup first; the fold reuses the vote slots' LDS.
  __threadfence();
  __syncthreads();
  // the pool log's pointer and the quad's start stamp (slice 3's LDS header) into registers now:
  // fold_unit reuses the slot LDS, and once done reaches nq the slot may carry the next batch
  // 
  uint64_t* const pl = threadIdx.x == 0 && quad < PLOG_QUADS ? dgetp(&bd->plog) : nullptr;
  uint64_t pl_start = 0;
  if (pl) {
    const uint32_t* h3 = lds + SLOT_BASE_W + 3 * STRIDE + NSLOTS * 12 + 2;
    pl_start = (uint64_t)h3[0] | (uint64_t)(h3[1] & 0xFFFFu) << 32;
  }
  const Slab s{unip(dgetp(&bd->state)), uni(dget(&bd->cap))};
  VmDev fold{};
  fold.code = a.fold_code;
  fold_unit(quad, n, fold, cst, lds + SLOT_BASE_W, threadIdx.x % VM_FOLD_W, threadIdx.x < VM_FOLD_W,
            Slab{s.p + (size_t)S_F * 12 * s.cap, s.cap}, Slab{nullptr, 0},
            Slab{unip(dgetp(&bd->part0)), uni(dget(&bd->part_cap))}, codes);
  if (pl) {  // the quad's pool-log record, ahead of the release below
    pl[16 + 2 * quad] = pl_start | (uint64_t)simd_key() << 48 | (uint64_t)how << 60;
    pl[16 + 2 * quad + 1] = __builtin_amdgcn_s_memrealtime();
  }
  // the quad's codes, planes, partial and log record, then its done count (k_pool_wait)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(pq_done(a.q, slot), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(a.q + PQ_INFL, ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // - 1
    __hip_atomic_fetch_add(pq_occ(a.q) + simd_key(), ~0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// The pool: each workgroup claims quads until the queue stays empty (pool_claim), then exits.
// LDS: constants + four slices of the larger of the vote / vote_t slot files; scratch: the
// workgroup's own spill area (4 x VOTE_NSCR entries), reused quad after quad. Two waves per SIMD
// are declared (the register budget that makes two pool workgroups share a SIMD).
__global__ __launch_bounds__(64, 2) void k_vm_pool(PoolArgs a) {
  __builtin_amdgcn_s_setprio(2);  // above the final streams' fold checks, below k_vm_final (3)
  extern __shared__ uint4 lds4[];
  // reserved CUs (OVH_FLAG_POOL_RESERVE): simd_key bits 2..8 = SE | SA | CU (wave-uniform)
  if (a.skip_cu && ((simd_key() >> 2) & 0x7Fu) < a.skip_cu) return;
  uint32_t* lds = reinterpret_cast<uint32_t*>(lds4);
  load_consts(lds, a.cst, VM_NCONST);
  const uint64_t t_in = __builtin_amdgcn_s_memrealtime();
  vote_stagger();
  uint32_t nquads = 0, why = 0;
#pragma unroll 1
  for (;; ++nquads) {
    uint32_t slot = 0, quad = 0, how = 0;
    if (!pool_claim(a.q, a.descs, &slot, &quad, &why, a.only, a.nsimd, &how)) break;
    slot = uni(slot);
    quad = uni(quad) | uni(how) << 28;  // the claim's flags ride in the top bits to the pool log
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // this batch's descriptor and inputs, fresh
    if (uni(dget(&a.descs[slot].table))) vote_quad<true>(a, slot, quad, lds);
    else vote_quad<false>(a, slot, quad, lds);
  }
  if (a.wlog && threadIdx.x == 0 && blockIdx.x < PLOG_WGS) {
    uint64_t* w = a.wlog + (size_t)blockIdx.x * PLOG_WG_WORDS;
    w[0] = t_in;
    w[1] = __builtin_amdgcn_s_memrealtime();
    w[2] = nquads;
    w[3] = why;
  }
}

// A batch's final stream waits here until the pool completed all `nq` quads of the slot's batch
// (one lane, bounded: after `ticks` of the 100 MHz clock it flags *err and returns, and the host
// reports OVH_ERR_DEVICE at the next synchronisation).
__global__ __launch_bounds__(64) void k_pool_wait(uint64_t* q, uint32_t slot, uint32_t nq, uint64_t ticks,
                                                  uint32_t* err) {
  if (threadIdx.x) return;
  const uint64_t t0 = wall_clock64();
  while (__hip_atomic_load(pq_done(q, slot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < nq) {
    if (wall_clock64() - t0 > ticks) {
      __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    __builtin_amdgcn_s_sleep(32);
  }
}

// Staging of a pool batch (ovh_stream, before its publication): the signatures and keys (or
// table indices) into the slot's own buffer, so the caller's buffers are free once ovh_stream
// has passed this kernel (the pool reads the batch later, on its own schedule).
__global__ __launch_bounds__(WG) void k_pool_stage(uint32_t n, const uint8_t* __restrict__ sigs,
                                                   const uint8_t* __restrict__ pks, const int32_t* __restrict__ idx,
                                                   uint8_t* __restrict__ dst) {
  const size_t nb = (size_t)n * 96 + (pks ? (size_t)n * 48 : 0);
  uint8_t* di = dst + (size_t)n * 144;
  for (size_t k = (size_t)blockIdx.x * WG + threadIdx.x; k < nb + (idx ? (size_t)n * 4 : 0);
       k += (size_t)gridDim.x * WG) {
    if (k < (size_t)n * 96) dst[k] = sigs[k];
    else if (k < nb) dst[k] = pks[k - (size_t)n * 96];
    else di[k - nb] = reinterpret_cast<const uint8_t*>(idx)[k - nb];
  }
}

// Fold level: SLICES units per 64-thread workgroup (4 on the main stream; 1 on the final
// stream, whose 10.8 KB of LDS fits beside a CU's four vote workgroups).
// gate: skip when *gate == 1 (the bisection's refold after a passed combined check)
template <int SLICES>
__global__ __launch_bounds__(64) void k_vm_fold(uint32_t m, VmDev prog, const uint32_t* __restrict__ cst_g, Slab inF,
                                                Slab inS, Slab out, const int32_t* __restrict__ codes,
                                                const int32_t* __restrict__ gate = nullptr) {
  if (gate && *gate == 1) return;
  __builtin_amdgcn_s_setprio(2);  // short, as the pool's waves
  extern __shared__ uint4 lds4[];
  uint32_t* lds = reinterpret_cast<uint32_t*>(lds4);
  uint32_t* cst = lds;
  const uint32_t slice = threadIdx.x / VM_FOLD_W, lane = threadIdx.x % VM_FOLD_W;
  const uint32_t sl = slice < SLICES ? slice : 0;  // idle slices address slice 0 (never write)
  uint32_t* slots = lds + SLOT_BASE_W + sl * FOLD_STRIDE_W;
  const uint32_t t = blockIdx.x * SLICES + slice;
  const bool active = slice < SLICES && 4 * t < m;
  load_consts(cst, cst_g, VM_NCONST);
  fold_unit(t, m, prog, cst, slots, lane, active, inF, inS, out, codes);
}

// Final: prod F * Miller(-G1, sum S) over in[0..m-1] (m <= 4) -> FE == 1 -> *result.
// xS.p: partial 0's S is xS[0] (the batch's MSM result; the folded partials carry S = O).
__global__ __launch_bounds__(64) void k_vm_final(uint32_t m, VmDev prog, const uint32_t* __restrict__ cst_g, Slab inF,
                                                 Slab inS, Slab xS, int32_t* __restrict__ result) {
  // above the pool's waves (2): the one-wave final shares its SIMD with a pool wave and ran
  // 4.2 ms instead of 2.1 at equal or lower priority; its slot ran out first (r05p trace). With
  // this and the MSM levels at 2: 1,432k verifs/s vs 1,131k-1,316k (r05q A/B)
  __builtin_amdgcn_s_setprio(3);
  extern __shared__ uint4 lds4[];
  uint32_t* lds = reinterpret_cast<uint32_t*>(lds4);
  uint32_t* cst = lds;
  uint32_t* slots = lds + SLOT_BASE_W;
  const uint32_t lane = threadIdx.x;
  load_consts(cst, cst_g, VM_NCONST);
  for (uint32_t k = lane; k < 4 * PART_PLANES; k += 64) {
    const uint32_t q = k / PART_PLANES, j = k % PART_PLANES;
    Fp v;
    if (q == 0 && j >= 12 && xS.p) {
      xS.ld(v, j - 12, 0);
    } else if (q < m) {
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

// One standalone vote (ovh_verify, verify_aggregated_signature: a batch of one needs no RLC
// coefficient): programs vote1 / vote_t1 on a whole 64-lane wave compute
// f = Miller(pk, H) Miller(-G1, sigma) as one two-pair Miller loop, stored to the F planes of
// element 0, and the code (precedence as k_vm_vote / k_vm_vote_t); k_vm_final1 then checks
// FE(f) == 1. No MSM, no fold, no bisection: the vote's own pairing equation is the check.
// One vote on a whole 64-lane wave (vote1 / vote_t1 and votew / votew_t: the two pairs share
// input and output layouts): inputs of vote i (pk bytes or table entry e, signature bytes, the u
// planes of slab index i), the program with RLC scalar `scalar` (its `st` ops write the f
// planes of slab index i), then the per-vote code in k_vm_vote's precedence.
static_assert(VM_VOTEW_NIN == VM_VOTE1_NIN && VM_VOTEW_T_NIN == VM_VOTE_T1_NIN && VM_VOTEW_W == 64 &&
                  VM_VOTEW_T_W == 64 && VM_VOTE1_W == 64 && VM_VOTE_T1_W == 64,
              "one-vote-per-wave programs share the vote1 / vote_t1 layouts");
// HIN (vote1h / vote_t1h): H = hash_to_G2(hash) comes from the message cache (planes hc, entry
// he, flag *hinf_in) instead of the u planes; otherwise *hinf_out (if set) receives the
// program's H-is-infinity flag for the cache.
static_assert(VM_VOTE1H_IN_H0 == VM_VOTE1_IN_U00 && VM_VOTE_T1H_IN_H0 == VM_VOTE_T1_IN_U00 &&
                  VM_VOTE1H_OUT_SIG_GRP == VM_VOTE1_OUT_SIG_GRP && VM_VOTE_T1H_OUT_SIG_GRP == VM_VOTE_T1_OUT_SIG_GRP,
              "vote1h / vote_t1h share vote1 / vote_t1's layouts, H in place of the u's");
template <bool TABLE, bool HIN = false>
__device__ __forceinline__ void vote_wave(const VmDev& prog, uint32_t nph, uint32_t ns, const uint16_t* IN,
                                          const uint16_t* OUT, const uint32_t* __restrict__ cst_g,
                                          const uint8_t* __restrict__ pk_bytes, PkSrc pk, uint32_t e,
                                          const uint8_t* __restrict__ sig, Slab s, uint32_t i, uint64_t scalar,
                                          int32_t* __restrict__ code, Slab hc = Slab{nullptr, 0}, uint32_t he = 0,
                                          const uint32_t* __restrict__ hinf_in = nullptr,
                                          uint32_t* __restrict__ hinf_out = nullptr) {
  extern __shared__ uint4 lds4[];
  uint32_t* lds = reinterpret_cast<uint32_t*>(lds4);
  uint32_t* cst = lds;
  uint32_t* slots = lds + SLOT_BASE_W;
  uint32_t* hdr = slots + ns * 12;  // [sig flags, pk flags]
  const uint32_t lane = threadIdx.x;
  load_consts(cst, cst_g, VM_NCONST);
  if (lane == 0) {
    uint32_t x1[12], x0[12], bad, inf, sort, xz;
    parse_hdr(sig, 96, x1, x0, bad, inf, sort, xz);
    if constexpr (TABLE) {
      slot_put(slots, IN[VM_VOTE_T1_IN_SIG_X1], x1);
      slot_put(slots, IN[VM_VOTE_T1_IN_SIG_X0], x0);
      slot_flag(slots, IN[VM_VOTE_T1_IN_SIG_SORT], sort);
    } else {
      slot_put(slots, IN[VM_VOTE1_IN_SIG_X1], x1);
      slot_put(slots, IN[VM_VOTE1_IN_SIG_X0], x0);
      slot_flag(slots, IN[VM_VOTE1_IN_SIG_SORT], sort);
    }
    hdr[0] = bad | inf << 1 | xz << 2;
  } else if (lane == 1) {
    if constexpr (TABLE) {
      hdr[1] = pk.flags[e];
    } else {
      uint32_t x[12], bad, inf, sort, xz;
      parse_hdr(pk_bytes, 48, x, x, bad, inf, sort, xz);
      slot_put(slots, IN[VM_VOTE1_IN_PK_X], x);
      slot_flag(slots, IN[VM_VOTE1_IN_PK_SORT], sort);
      hdr[1] = bad | inf << 1 | xz << 2;
    }
  } else if (!HIN && lane >= 2 && lane < 6) {
    Fp u;
    s.ld(u, S_U + (lane - 2), i);
    if constexpr (TABLE) slot_put(slots, IN[VM_VOTE_T1_IN_U00 + (lane - 2)], u.v);
    else slot_put(slots, IN[VM_VOTE1_IN_U00 + (lane - 2)], u.v);
  } else if (HIN && lane >= 10 && lane < 16) {
    Fp h;
    hc.ld(h, lane - 10, he);
    if constexpr (TABLE) slot_put(slots, IN[VM_VOTE_T1_IN_U00 + (lane - 10)], h.v);
    else slot_put(slots, IN[VM_VOTE1_IN_U00 + (lane - 10)], h.v);
  } else if (TABLE && lane >= 6 && lane < 9) {
    Fp v;
    Slab{const_cast<uint32_t*>(pk.planes), pk.cap}.ld(v, lane - 6, e);
    if constexpr (TABLE) slot_put(slots, IN[VM_VOTE_T1_IN_PK_X + (lane - 6)], v.v);
  }
  __syncthreads();
  vm::run(prog.code, nph, 64, lane, true, slots, cst, scalar, vm::Out{s.p, s.cap, i});
  if (lane == 0) {
    const uint32_t sf = hdr[0], pf = hdr[1];
    const uint32_t sg_bad = sf & 1, sg_inf = (sf >> 1) & 1, sg_xz = (sf >> 2) & 1;
    uint32_t sg_ok, sg_grp, h_inf, pk_ok = 1, pk_grp = 1;
    if constexpr (TABLE) {
      sg_ok = slot_flag_get(slots, OUT[VM_VOTE_T1_OUT_SIG_OK]);
      sg_grp = slot_flag_get(slots, OUT[VM_VOTE_T1_OUT_SIG_GRP]);
      h_inf = HIN ? *hinf_in : slot_flag_get(slots, OUT[VM_VOTE_T1_OUT_H_INF]);
    } else {
      pk_ok = slot_flag_get(slots, OUT[VM_VOTE1_OUT_PK_OK]);
      pk_grp = slot_flag_get(slots, OUT[VM_VOTE1_OUT_PK_GRP]);
      sg_ok = slot_flag_get(slots, OUT[VM_VOTE1_OUT_SIG_OK]);
      sg_grp = slot_flag_get(slots, OUT[VM_VOTE1_OUT_SIG_GRP]);
      h_inf = HIN ? *hinf_in : slot_flag_get(slots, OUT[VM_VOTE1_OUT_H_INF]);
    }
    if (!HIN && hinf_out) *hinf_out = h_inf;
    // key flags in the table's terms, then the precedence of k_vm_vote_t (consensus.rs:397-416)
    uint32_t kf = pf;
    if (!TABLE) {
      const uint32_t pk_bad = pf & 1, pk_inf = (pf >> 1) & 1, pk_xz = (pf >> 2) & 1;
      kf = (pk_bad || (!pk_inf && (!pk_ok || pk_xz))) ? PKF_PARSE : pk_inf ? PKF_INF : !pk_grp ? PKF_GRP : 0u;
    }
    int32_t c;
    if (kf & PKF_PARSE) c = OVH_ERR_PUBKEY;
    else if (sg_bad) c = BLST_BAD_ENCODING;
    else if (!sg_inf && !sg_ok) c = BLST_POINT_NOT_ON_CURVE;
    else if (!sg_inf && (sg_xz || !sg_grp)) c = BLST_POINT_NOT_IN_GROUP;
    else if (kf & PKF_INF) c = BLST_PK_IS_INFINITY;
    else if (kf & PKF_GRP) c = BLST_POINT_NOT_IN_GROUP;
    else if (h_inf || sg_inf) c = BLST_VERIFY_FAIL;
    else c = 0;
    *code = c;
  }
}

// The standalone vote (ovh_verify, one-QC checks): vote1 / vote_t1 at slab index 0, no
// coefficient.
template <bool TABLE>
__global__ __launch_bounds__(64) void k_vm_vote1(VmDev prog, const uint32_t* __restrict__ cst_g,
                                                 const uint8_t* __restrict__ pk_bytes, PkSrc pk,
                                                 const uint8_t* __restrict__ sig, Slab s, int32_t* __restrict__ code,
                                                 uint32_t* __restrict__ hinf_out = nullptr) {
  const uint32_t e = TABLE && pk.idx ? (uint32_t)pk.idx[0] : 0u;
  if constexpr (TABLE)
    vote_wave<true>(prog, VM_VOTE_T1_NPHASES, VM_VOTE_T1_NSLOTS, VM_VOTE_T1_IN, VM_VOTE_T1_OUT, cst_g, pk_bytes, pk, e,
                    sig, s, 0, 1, code, Slab{nullptr, 0}, 0, nullptr, hinf_out);
  else
    vote_wave<false>(prog, VM_VOTE1_NPHASES, VM_VOTE1_NSLOTS, VM_VOTE1_IN, VM_VOTE1_OUT, cst_g, pk_bytes, pk, e, sig,
                     s, 0, 1, code, Slab{nullptr, 0}, 0, nullptr, hinf_out);
}

// The standalone vote on a hash in the message cache: vote1h / vote_t1h with H from entry he.
template <bool TABLE>
__global__ __launch_bounds__(64) void k_vm_vote1h(VmDev prog, const uint32_t* __restrict__ cst_g,
                                                  const uint8_t* __restrict__ pk_bytes, PkSrc pk,
                                                  const uint8_t* __restrict__ sig, Slab s, int32_t* __restrict__ code,
                                                  Slab hc, uint32_t he, const uint32_t* __restrict__ hinf) {
  const uint32_t e = TABLE && pk.idx ? (uint32_t)pk.idx[0] : 0u;
  if constexpr (TABLE)
    vote_wave<true, true>(prog, VM_VOTE_T1H_NPHASES, VM_VOTE_T1H_NSLOTS, VM_VOTE_T1H_IN, VM_VOTE_T1H_OUT, cst_g,
                          pk_bytes, pk, e, sig, s, 0, 1, code, hc, he, hinf + he);
  else
    vote_wave<false, true>(prog, VM_VOTE1H_NPHASES, VM_VOTE1H_NSLOTS, VM_VOTE1H_IN, VM_VOTE1H_OUT, cst_g, pk_bytes, pk,
                           e, sig, s, 0, 1, code, hc, he, hinf + he);
}

// vote1's stored H (the S_RS planes of slab index 0) -> message-cache entry he.
__global__ __launch_bounds__(64) void k_copy_h(Slab s, Slab hc, uint32_t he) {
  for (uint32_t k = threadIdx.x; k < 6 * 12; k += 64) hc.p[(size_t)k * hc.cap + he] = s.p[(size_t)(S_RS * 12 + k) * s.cap];
}

// Small batches (n <= SMALL_MAX, verify_small_locked): vote i = workgroup i on a whole wave,
// program votew / votew_t with the vote's RLC coefficient: f_i = Miller(r pk, H) Miller(-G1,
// r sigma) to the slab's f planes, code to codes[i].
template <bool TABLE>
__global__ __launch_bounds__(64) void k_vm_votew(uint32_t n, VmDev prog, const uint32_t* __restrict__ cst_g,
                                                 const uint8_t* __restrict__ pks, PkSrc pk,
                                                 const uint8_t* __restrict__ sigs, Slab s, uint64_t seed,
                                                 uint64_t base, int32_t* __restrict__ codes) {
  const uint32_t i = blockIdx.x;
  if (i >= n) return;
  const uint32_t e = TABLE ? (pk.idx ? (uint32_t)pk.idx[i] : i) : 0u;
  if constexpr (TABLE)
    vote_wave<true>(prog, VM_VOTEW_T_NPHASES, VM_VOTEW_T_NSLOTS, VM_VOTEW_T_IN, VM_VOTEW_T_OUT, cst_g, nullptr, pk, e,
                    sigs + (size_t)i * 96, s, i, vote_scalar(seed, base, i), codes + i);
  else
    vote_wave<false>(prog, VM_VOTEW_NPHASES, VM_VOTEW_NSLOTS, VM_VOTEW_IN, VM_VOTEW_OUT, cst_g, pks + (size_t)i * 48,
                     pk, e, sigs + (size_t)i * 96, s, i, vote_scalar(seed, base, i), codes + i);
}

// ------------------------------------------------------------------ same-message batches (r04)
// A round's votes all sign one hash (consensus.rs:169-175: Vote carries no voter), so a batch of
// n votes over G distinct hashes is checked as
//   prod_g e(sum_{i in g} r_i pk_i, H_g) * e(-G1, sum_i r_i sigma_i) == 1
// (verify_samemsg_locked): one hash_to_G2 (k_vm_h2g) and one Miller loop
// (k_vm_gmil) per distinct hash; per vote only the key / signature checks and r_i pk_i
// (k_vm_vsame, programs vsame / vsame_t). Group slab planes (per distinct hash, gcap entries):
// u0, u1 | H | f (tools/fpvm/progs.py G_U, G_H, G_F).
constexpr uint32_t VSAME_NSLOTS = VM_VSAME_NSLOTS > VM_VSAME_T_NSLOTS ? VM_VSAME_NSLOTS : VM_VSAME_T_NSLOTS;
constexpr uint32_t VSAME_STRIDE_W = align256w(VSAME_NSLOTS * 12 + 4);
// the 8-lane forms (programs vsame8 / vsame8_t: eight votes per wave) for batches of at least
// VSAME8_MIN votes: 1,504 phases per eight votes against 1,288 per four, so a large batch's
// per-vote waves take ~40% less SIMD time while a small one keeps the 16-lane form's latency
constexpr uint32_t VSAME8_NSLOTS = VM_VSAME8_NSLOTS > VM_VSAME8_T_NSLOTS ? VM_VSAME8_NSLOTS : VM_VSAME8_T_NSLOTS;
constexpr uint32_t VSAME8_STRIDE_W = align256w(VSAME8_NSLOTS * 12 + 4);
#ifndef VSAME8_MIN
#define VSAME8_MIN 2048u
#endif
constexpr uint32_t H2G_STRIDE_W = align256w(VM_H2G_NSLOTS * 12);
static_assert(VM_VSAME_W == 16 && VM_VSAME_T_W == 16 && VM_VSAME8_W == 8 && VM_VSAME8_T_W == 8 && VM_H2G_W == 16 && VM_GMIL_W == 64 && VM_H2G_NIN == 4 &&
                  VM_GMIL_NIN == 9 && VM_G_U == 0 && VM_G_PLANES == 22,
              "same-message program shapes (tools/fpvm/progs.py)");

// Per vote (W-lane slice, 64 / W per workgroup; W = 16: vsame / vsame_t, 8: vsame8 / vsame8_t): votes lo + j, j < cnt (key bytes at pks + 48 j, or
// table entry pk.idx[j]; signature at sigs + 96 j); stores sigma, tau and r pk at slab index
// lo + j; code in the reference precedence without the H = O case (k_samemsg_fix adds it).
// Same-message pipeline (r05ag/r05ah, tools/samemsg_pipe.py, 24 batches of 4,096 votes, ms per
// batch): the per-vote vsame waves at the pool's priority (2), hash_to_G2 and gfin above them (3):
// 2.54 -> 2.43; the one-hash API's hash_to_G2 on SM_H2G_STREAMS streams in turn instead of one:
// 2 streams 2.06-2.08, 3 streams 1.99-2.00, 4 2.03-2.12. (r05aj: vsame in the vote pool ran 4.9
// ms per batch -- hash_to_G2 (24 KB of LDS) and gfin (34 KB) do not fit the pool's one place per
// CU and waited for the pool to drain; reverted)
#ifndef SM_PRIO
#define SM_PRIO 1
#endif
#ifndef SM_H2G_STREAMS
#define SM_H2G_STREAMS 3
#endif
static_assert(SM_H2G_STREAMS >= 1 && SM_H2G_STREAMS <= 4, "hstream[4]");
template <bool TABLE, uint32_t W = 16>
__global__ __launch_bounds__(64) void k_vm_vsame(uint32_t cnt, uint32_t lo, VmDev prog,
                                                 const uint32_t* __restrict__ cst_g, const uint8_t* __restrict__ pks,
                                                 PkSrc pk, const uint8_t* __restrict__ sigs, Slab s, uint64_t seed,
                                                 uint64_t base, int32_t* __restrict__ codes) {
  extern __shared__ uint4 lds4[];
  if (SM_PRIO) __builtin_amdgcn_s_setprio(2);
  uint32_t* lds = reinterpret_cast<uint32_t*>(lds4);
  uint32_t* cst = lds;
  static_assert(W == 16 || W == 8, "vsame slice width");
  constexpr bool W8 = W == 8;
  const uint32_t slice = threadIdx.x / W, lane = threadIdx.x % W;
  uint32_t* slots = lds + SLOT_BASE_W + slice * (W8 ? VSAME8_STRIDE_W : VSAME_STRIDE_W);
  constexpr uint32_t NS = W8 ? (TABLE ? VM_VSAME8_T_NSLOTS : VM_VSAME8_NSLOTS)
                             : (TABLE ? VM_VSAME_T_NSLOTS : VM_VSAME_NSLOTS);
  uint32_t* hdr = slots + NS * 12;  // [sig flags, key flags]
  const uint16_t* IN = W8 ? (TABLE ? VM_VSAME8_T_IN : VM_VSAME8_IN) : (TABLE ? VM_VSAME_T_IN : VM_VSAME_IN);
  const uint16_t* OUT = W8 ? (TABLE ? VM_VSAME8_T_OUT : VM_VSAME8_OUT) : (TABLE ? VM_VSAME_T_OUT : VM_VSAME_OUT);
  const uint32_t j = blockIdx.x * (64 / W) + slice, i = lo + j;
  const bool active = j < cnt;
  load_consts(cst, cst_g, VM_NCONST);
  if (active) {
    if (lane == 0) {
      uint32_t x1[12], x0[12], bad, inf, sort, xz;
      parse_hdr(sigs + (size_t)j * 96, 96, x1, x0, bad, inf, sort, xz);
      slot_put(slots, IN[TABLE ? VM_VSAME_T_IN_SIG_X1 : VM_VSAME_IN_SIG_X1], x1);
      slot_put(slots, IN[TABLE ? VM_VSAME_T_IN_SIG_X0 : VM_VSAME_IN_SIG_X0], x0);
      slot_flag(slots, IN[TABLE ? VM_VSAME_T_IN_SIG_SORT : VM_VSAME_IN_SIG_SORT], sort);
      hdr[0] = bad | inf << 1 | xz << 2;
    } else if (lane == 1) {
      if constexpr (TABLE) {
        hdr[1] = pk.flags[pk.idx[j]];
      } else {
        uint32_t x[12], bad, inf, sort, xz;
        parse_hdr(pks + (size_t)j * 48, 48, x, x, bad, inf, sort, xz);
        slot_put(slots, IN[VM_VSAME_IN_PK_X], x);
        slot_flag(slots, IN[VM_VSAME_IN_PK_SORT], sort);
        hdr[1] = bad | inf << 1 | xz << 2;
      }
    } else if (TABLE && lane >= 2 && lane < 5) {
      Fp v;
      Slab{const_cast<uint32_t*>(pk.planes), pk.cap}.ld(v, lane - 2, (uint32_t)pk.idx[j]);
      slot_put(slots, IN[VM_VSAME_T_IN_PK_X + (lane - 2)], v.v);
    }
  }
  __syncthreads();
  constexpr uint32_t NPH = W8 ? (TABLE ? VM_VSAME8_T_NPHASES : VM_VSAME8_NPHASES)
                              : (TABLE ? VM_VSAME_T_NPHASES : VM_VSAME_NPHASES);
  vm::run(prog.code, NPH, W, lane, active, slots, cst, vote_scalar(seed, base, i), vm::Out{s.p, s.cap, i});
  if (active && lane == 0) {
    const uint32_t sf = hdr[0], pf = hdr[1];
    const uint32_t sg_bad = sf & 1, sg_inf = (sf >> 1) & 1, sg_xz = (sf >> 2) & 1;
    uint32_t kf = pf, sg_ok, sg_grp;
    if constexpr (TABLE) {
      sg_ok = slot_flag_get(slots, OUT[VM_VSAME_T_OUT_SIG_OK]);
      sg_grp = slot_flag_get(slots, OUT[VM_VSAME_T_OUT_SIG_GRP]);
    } else {
      sg_ok = slot_flag_get(slots, OUT[VM_VSAME_OUT_SIG_OK]);
      sg_grp = slot_flag_get(slots, OUT[VM_VSAME_OUT_SIG_GRP]);
      const uint32_t pk_ok = slot_flag_get(slots, OUT[VM_VSAME_OUT_PK_OK]);
      const uint32_t pk_grp = slot_flag_get(slots, OUT[VM_VSAME_OUT_PK_GRP]);
      const uint32_t pk_bad = pf & 1, pk_inf = (pf >> 1) & 1, pk_xz = (pf >> 2) & 1;
      kf = (pk_bad || (!pk_inf && (!pk_ok || pk_xz))) ? PKF_PARSE : pk_inf ? PKF_INF : !pk_grp ? PKF_GRP : 0u;
    }
    int32_t c;  // consensus.rs:397-416, as k_vm_vote; H(m) = O is added per group (k_samemsg_fix)
    if (kf & PKF_PARSE) c = OVH_ERR_PUBKEY;
    else if (sg_bad) c = BLST_BAD_ENCODING;
    else if (!sg_inf && !sg_ok) c = BLST_POINT_NOT_ON_CURVE;
    else if (!sg_inf && (sg_xz || !sg_grp)) c = BLST_POINT_NOT_IN_GROUP;
    else if (kf & PKF_INF) c = BLST_PK_IS_INFINITY;
    else if (kf & PKF_GRP) c = BLST_POINT_NOT_IN_GROUP;
    else if (sg_inf) c = BLST_VERIFY_FAIL;
    else c = 0;
    codes[i] = c;
  }
}

// hash_to_G2 per distinct hash (16-lane slice, 4 per workgroup): u planes of group g -> H planes
// of group g, ghinf[g] = H is the identity.
__global__ __launch_bounds__(64) void k_vm_h2g(uint32_t G, VmDev prog, const uint32_t* __restrict__ cst_g, Slab g,
                                               uint32_t* __restrict__ ghinf) {
  extern __shared__ uint4 lds4[];
  if (SM_PRIO) __builtin_amdgcn_s_setprio(3);
  uint32_t* lds = reinterpret_cast<uint32_t*>(lds4);
  uint32_t* cst = lds;
  const uint32_t slice = threadIdx.x / 16, lane = threadIdx.x % 16;
  uint32_t* slots = lds + SLOT_BASE_W + slice * H2G_STRIDE_W;
  const uint32_t q = blockIdx.x * VM_SLICES + slice;
  const bool active = q < G;
  load_consts(cst, cst_g, VM_NCONST);
  if (active && lane < 4) {
    Fp u;
    g.ld(u, VM_G_U + lane, q);
    slot_put(slots, VM_H2G_IN[lane], u.v);
  }
  __syncthreads();
  vm::run(prog.code, VM_H2G_NPHASES, 16, lane, active, slots, cst, 0, vm::Out{g.p, g.cap, q});
  if (active && lane == 0) ghinf[q] = slot_flag_get(slots, VM_H2G_OUT[VM_H2G_OUT_H_INF]) ? 1u : 0u;
}

// Lane per vote: a vote whose hash maps to the identity (H_g = O) fails with VERIFY_FAIL when
// nothing earlier failed (k_vm_vote's precedence); every vote with a non-zero code contributes
// the identity to its group's key sum (r pk := (0 : 1 : 0)).
__global__ __launch_bounds__(WG) void k_samemsg_fix(uint32_t n, const uint32_t* __restrict__ gid,
                                                    const uint32_t* __restrict__ ghinf, int32_t* __restrict__ codes,
                                                    Slab P) {
  const uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  int32_t c = codes[i];
  if (c == 0 && ghinf[gid[i]]) codes[i] = c = BLST_VERIFY_FAIL;
  if (c != 0) {
    Fp z, o;
    fp_zero(z);
    fp_one(o);
    P.st(z, 0, i);
    P.st(o, 1, i);
    P.st(z, 2, i);
  }
}

// One level of the per-hash key sums: pair k = (a, b) -> P[a] = P[a] + P[b] (g1padd, complete
// formulas), one pair per 8-lane slice. The host plans the levels (samemsg_plan): the pairs of a
// level are disjoint, so the update is in place.
__global__ __launch_bounds__(64) void k_vm_g1pairs(uint32_t npairs, VmDev prog, uint32_t stride_w,
                                                   const uint32_t* __restrict__ cst_g, const uint32_t* __restrict__ pairs,
                                                   Slab P) {
  constexpr uint32_t W = VM_G1PADD_W, SL = 64 / W;
  extern __shared__ uint4 lds4[];
  uint32_t* lds = reinterpret_cast<uint32_t*>(lds4);
  uint32_t* cst = lds;
  const uint32_t slice = threadIdx.x / W, lane = threadIdx.x % W;
  uint32_t* slots = lds + SLOT_BASE_W + slice * stride_w;
  const uint32_t q = blockIdx.x * SL + slice;
  const bool active = q < npairs;
  const uint32_t a = active ? pairs[2 * q] : 0u, b = active ? pairs[2 * q + 1] : 0u;
  load_consts(cst, cst_g, VM_NCONST);
  if (active) {
    for (uint32_t k = lane; k < 6; k += W) {
      Fp v;
      P.ld(v, k % 3, k < 3 ? a : b);
      slot_put(slots, prog.in[k], v.v);
    }
  }
  __syncthreads();
  vm::run(prog.code, prog.nphases, W, lane, active, slots, cst, 0, vm::Out{nullptr, 0, 0});
  if (active) {
    for (uint32_t k = lane; k < 3; k += W) {
      Fp v;
      const uint32_t src = prog.out[k];
      for (int l = 0; l < 12; ++l) v.v[l] = slots[src * 12 + l];
      vm::canon(v, v);
      P.st(v, k, a);
    }
  }
}

// The head hash of a same-message batch (one wave): the first hash whose key sum is not the
// identity (some vote of it passed its checks) and whose H is not O -- its pair joins the final's
// two-pair loop (k_vm_gfin); 0 when there is none (gfin then finds the batch degenerate). ADVICE
// r04: with hash 0 always the head, one malformed vote on a fresh hash arriving first made the
// combined check degenerate and sent every other vote of the batch through the bisection.
__global__ __launch_bounds__(64) void k_pick_head(uint32_t G, const uint32_t* __restrict__ head, Slab P,
                                                  const uint32_t* __restrict__ ghinf, uint32_t* __restrict__ sel) {
  uint32_t best = 0xFFFFFFFFu;
  for (uint32_t q = threadIdx.x; q < G; q += 64) {
    Fp z;
    P.ld(z, 2, head[q]);
    if (!fp_is_zero(z) && !ghinf[q] && q < best) best = q;
  }
  for (uint32_t off = 32; off; off >>= 1) {
    const uint32_t o = __shfl_xor(best, off);
    best = o < best ? o : best;
  }
  if (threadIdx.x == 0) *sel = best == 0xFFFFFFFFu ? 0u : best;
}

// Per distinct hash other than the head (one wave each, hashes 0..G-1 with the head skipped):
// f_g = Miller(apk_g, H_g) -> the group slab's f planes at index g, hash 0's at the head's index
// (so the fold reads f of indices 1..G-1); apk_g = P[head[g]] (its votes' r pk summed, the
// identity when none of them passed its checks or H_g = O), and then f_g = 1 (e(O, H) = 1).
__global__ __launch_bounds__(64) void k_vm_gmil(uint32_t G, const uint32_t* __restrict__ sel, VmDev prog,
                                                const uint32_t* __restrict__ cst_g, const uint32_t* __restrict__ head,
                                                Slab P, Slab g) {
  extern __shared__ uint4 lds4[];
  uint32_t* lds = reinterpret_cast<uint32_t*>(lds4);
  uint32_t* cst = lds;
  uint32_t* slots = lds + SLOT_BASE_W;
  __shared__ uint32_t zinf;
  const uint32_t hsel = *sel;
  const uint32_t q = blockIdx.x, lane = threadIdx.x;
  if (q >= G || q == hsel) return;
  const uint32_t oq = q == 0 ? hsel : q;  // the f index this hash's Miller value goes to
  const uint32_t a = head[q];
  load_consts(cst, cst_g, VM_NCONST);
  if (lane == 0) {
    Fp z;
    P.ld(z, 2, a);
    zinf = fp_is_zero(z) ? 1u : 0u;
  }
  if (lane < 9) {
    Fp v;
    if (lane < 3) P.ld(v, lane, a);
    else g.ld(v, VM_G_H + (lane - 3), q);
    slot_put(slots, VM_GMIL_IN[lane], v.v);
  }
  __syncthreads();
  if (zinf) {  // wave-uniform
    if (lane < 12) {
      Fp v;
      if (lane == 0) fp_one(v);
      else fp_zero(v);
      g.st(v, VM_G_F + lane, oq);
    }
    return;
  }
  vm::run(prog.code, VM_GMIL_NPHASES, 64, lane, true, slots, cst, 0, vm::Out{g.p, g.cap, oq});
}

// The bisection of a same-message batch whose combined check failed (skipped when *verdict == 1):
// every vote with code 0 of [lo, lo + cnt) on a whole wave, vote1h / vote_t1h with its hash's H
// -> f_i = Miller(pk, H) Miller(-G1, sigma) in the slab's f planes; k_vm_votefe then checks
// FE(f_i) == 1 per vote.
template <bool TABLE>
__global__ __launch_bounds__(64) void k_vm_vote1h_b(uint32_t cnt, uint32_t lo, VmDev prog,
                                                    const uint32_t* __restrict__ cst_g,
                                                    const uint8_t* __restrict__ pks, PkSrc pk,
                                                    const uint8_t* __restrict__ sigs, Slab s, int32_t* __restrict__ codes,
                                                    const uint32_t* __restrict__ gid, Slab gH,
                                                    const uint32_t* __restrict__ ghinf,
                                                    const int32_t* __restrict__ verdict) {
  if (*verdict == 1) return;
  const uint32_t j = blockIdx.x, i = lo + j;
  if (j >= cnt || codes[i] != 0) return;
  const uint32_t e = TABLE ? (uint32_t)pk.idx[j] : 0u;
  if constexpr (TABLE)
    vote_wave<true, true>(prog, VM_VOTE_T1H_NPHASES, VM_VOTE_T1H_NSLOTS, VM_VOTE_T1H_IN, VM_VOTE_T1H_OUT, cst_g,
                          nullptr, pk, e, sigs + (size_t)j * 96, s, i, 1, codes + i, gH, gid[i], ghinf + gid[i]);
  else
    vote_wave<false, true>(prog, VM_VOTE1H_NPHASES, VM_VOTE1H_NSLOTS, VM_VOTE1H_IN, VM_VOTE1H_OUT, cst_g,
                           pks + (size_t)j * 48, pk, e, sigs + (size_t)j * 96, s, i, 1, codes + i, gH, gid[i],
                           ghinf + gid[i]);
}

// The combined check of a same-message batch (one wave): F (the Miller values of the other
// hashes, folded to one; the identity when F.p is null) x Miller(apk_h, H_h) x Miller(-G1, S) as
// one two-pair Miller loop, then FE == 1 -> *verdict (program gfin). h = *sel (k_pick_head: a
// hash with a non-identity key sum), apk_h = P[head[h]], S = the MSM's sum. When apk_h or S is
// the identity (no vote passed its checks) the pair cannot enter the shared loop: the verdict is
// 0 and the per-vote bisection decides every code exactly.
static_assert(VM_GFIN_W == 64 && VM_GFIN_NIN == 27, "gfin inputs: F, apk, H, S");
__global__ __launch_bounds__(64) void k_vm_gfin(VmDev prog, const uint32_t* __restrict__ cst_g, Slab F,
                                                const uint32_t* __restrict__ head, const uint32_t* __restrict__ sel,
                                                Slab P, Slab gH, Slab S, int32_t* __restrict__ verdict) {
  extern __shared__ uint4 lds4[];
  if (SM_PRIO) __builtin_amdgcn_s_setprio(3);
  uint32_t* lds = reinterpret_cast<uint32_t*>(lds4);
  uint32_t* cst = lds;
  uint32_t* slots = lds + SLOT_BASE_W;
  __shared__ uint32_t degenerate;
  const uint32_t lane = threadIdx.x, hsel = *sel, a = head[hsel];
  load_consts(cst, cst_g, VM_NCONST);
  if (lane == 0) {
    Fp za, zs;
    P.ld(za, 2, a);
    S.ld(zs, 4, 0);
    Fp zs1;
    S.ld(zs1, 5, 0);
    degenerate = (fp_is_zero(za) || (fp_is_zero(zs) && fp_is_zero(zs1))) ? 1u : 0u;
  }
  if (lane < 27) {
    Fp v;
    if (lane < 12) {
      if (F.p) F.ld(v, lane, 0);
      else if (lane == 0) fp_one(v);
      else fp_zero(v);
    } else if (lane < 15) {
      P.ld(v, lane - 12, a);
    } else if (lane < 21) {
      gH.ld(v, lane - 15, hsel);
    } else {
      S.ld(v, lane - 21, 0);
    }
    slot_put(slots, VM_GFIN_IN[lane], v.v);
  }
  __syncthreads();
  if (degenerate) {  // wave-uniform
    if (lane == 0) *verdict = 0;
    return;
  }
  vm::run(prog.code, VM_GFIN_NPHASES, 64, lane, true, slots, cst, 0, vm::Out{nullptr, 0, 0});
  if (lane == 0) *verdict = slot_flag_get(slots, VM_GFIN_OUT[0]) ? 1 : 0;
}

// verify_aggregated_signature (verify_aggregated_vm), the part without the aggregated key, on a
// side stream beside the keys' decompression / subgroup checks / tree sum: program qcpre (the
// signature's checks, H = hash_to_G2, g = Miller(-G1, sigma)) -> H in the S_RS planes and g in
// the f planes of slab index 0; flags word: signature header flags | sig_ok << 8 | sig_grp << 9
// | h_inf << 10.
__global__ __launch_bounds__(64) void k_vm_qcpre(VmDev prog, const uint32_t* __restrict__ cst_g,
                                                 const uint8_t* __restrict__ sig, Slab s, uint32_t* __restrict__ flags) {
  extern __shared__ uint4 lds4[];
  uint32_t* lds = reinterpret_cast<uint32_t*>(lds4);
  uint32_t* cst = lds;
  uint32_t* slots = lds + SLOT_BASE_W;
  uint32_t* hdr = slots + VM_QCPRE_NSLOTS * 12;
  const uint32_t lane = threadIdx.x;
  load_consts(cst, cst_g, VM_NCONST);
  if (lane == 0) {
    uint32_t x1[12], x0[12], bad, inf, sort, xz;
    parse_hdr(sig, 96, x1, x0, bad, inf, sort, xz);
    slot_put(slots, VM_QCPRE_IN[VM_QCPRE_IN_SIG_X1], x1);
    slot_put(slots, VM_QCPRE_IN[VM_QCPRE_IN_SIG_X0], x0);
    slot_flag(slots, VM_QCPRE_IN[VM_QCPRE_IN_SIG_SORT], sort);
    hdr[0] = bad | inf << 1 | xz << 2;
  } else if (lane >= 2 && lane < 6) {
    Fp u;
    s.ld(u, S_U + (lane - 2), 0);
    slot_put(slots, VM_QCPRE_IN[VM_QCPRE_IN_U00 + (lane - 2)], u.v);
  }
  __syncthreads();
  vm::run(prog.code, VM_QCPRE_NPHASES, VM_QCPRE_W, lane, true, slots, cst, 0, vm::Out{s.p, s.cap, 0});
  if (lane == 0)
    *flags = hdr[0] | slot_flag_get(slots, VM_QCPRE_OUT[VM_QCPRE_OUT_SIG_OK]) << 8 |
             slot_flag_get(slots, VM_QCPRE_OUT[VM_QCPRE_OUT_SIG_GRP]) << 9 |
             slot_flag_get(slots, VM_QCPRE_OUT[VM_QCPRE_OUT_H_INF]) << 10;
}

// ... and the rest once the aggregated key (table entry 0 of pk: projective planes + flags) and
// qcpre are done: program qcmil, f = Miller(apk, H) g -> the f planes of slab index 1, then the
// code in vote_t1's precedence (consensus.rs:397-416 via verify_aggregated_signature).
__global__ __launch_bounds__(64) void k_vm_qcmil(VmDev prog, const uint32_t* __restrict__ cst_g, PkSrc pk, Slab s,
                                                 const uint32_t* __restrict__ flags, int32_t* __restrict__ code) {
  extern __shared__ uint4 lds4[];
  uint32_t* lds = reinterpret_cast<uint32_t*>(lds4);
  uint32_t* cst = lds;
  uint32_t* slots = lds + SLOT_BASE_W;
  const uint32_t lane = threadIdx.x;
  load_consts(cst, cst_g, VM_NCONST);
  if (lane < 21) {
    Fp v;
    if (lane < 3) Slab{const_cast<uint32_t*>(pk.planes), pk.cap}.ld(v, lane, 0);
    else if (lane < 9) s.ld(v, S_RS + (lane - 3), 0);
    else s.ld(v, S_F + (lane - 9), 0);
    slot_put(slots, VM_QCMIL_IN[lane], v.v);
  }
  __syncthreads();
  vm::run(prog.code, VM_QCMIL_NPHASES, VM_QCMIL_W, lane, true, slots, cst, 0, vm::Out{s.p, s.cap, 1});
  if (lane == 0) {
    const uint32_t sf = *flags, kf = pk.flags[0];
    const uint32_t sg_bad = sf & 1, sg_inf = (sf >> 1) & 1, sg_xz = (sf >> 2) & 1;
    const uint32_t sg_ok = (sf >> 8) & 1, sg_grp = (sf >> 9) & 1, h_inf = (sf >> 10) & 1;
    int32_t c;
    if (kf & PKF_PARSE) c = OVH_ERR_PUBKEY;
    else if (sg_bad) c = BLST_BAD_ENCODING;
    else if (!sg_inf && !sg_ok) c = BLST_POINT_NOT_ON_CURVE;
    else if (!sg_inf && (sg_xz || !sg_grp)) c = BLST_POINT_NOT_IN_GROUP;
    else if (kf & PKF_INF) c = BLST_PK_IS_INFINITY;
    else if (kf & PKF_GRP) c = BLST_POINT_NOT_IN_GROUP;
    else if (h_inf || sg_inf) c = BLST_VERIFY_FAIL;
    else c = 0;
    *code = c;
  }
}
static_assert(VM_QCMIL_NIN == 21 && VM_QCPRE_W == 64 && VM_QCMIL_W == 64, "qcmil inputs: apk X Y Z, H, g");

// FE(F_u) == 1 for unit u of the F planes (program final1): the shared body of the FE kernels.
__device__ __forceinline__ bool fe_one(const VmDev& prog, const uint32_t* __restrict__ cst_g, Slab F, uint32_t u) {
  extern __shared__ uint4 lds4[];
  uint32_t* lds = reinterpret_cast<uint32_t*>(lds4);
  uint32_t* cst = lds;
  uint32_t* slots = lds + SLOT_BASE_W;
  const uint32_t lane = threadIdx.x;
  load_consts(cst, cst_g, VM_NCONST);
  if (lane < 12) {
    Fp v;
    F.ld(v, lane, u);
    slot_put(slots, VM_FINAL1_IN[lane], v.v);
  }
  __syncthreads();
  vm::run(prog.code, VM_FINAL1_NPHASES, VM_FINAL1_W, lane, true, slots, cst, 0, vm::Out{nullptr, 0, 0});
  return slot_flag_get(slots, VM_FINAL1_OUT[0]) != 0;
}

// A small batch's combined check: FE(prod f_i) == 1 on the folded partial (unit 0) -> *verdict.
__global__ __launch_bounds__(64) void k_vm_fe(VmDev prog, const uint32_t* __restrict__ cst_g, Slab F,
                                              int32_t* __restrict__ verdict) {
  const bool ok = fe_one(prog, cst_g, F, 0);
  if (threadIdx.x == 0) *verdict = ok ? 1 : 0;
}

// A small batch's bisection (skipped when *verdict == 1): every vote with code 0 on its own,
// FE(f_i) = (e(pk, H) / e(G1, sigma))^r == 1 exactly when the vote verifies (r != 0 mod the
// group order).
__global__ __launch_bounds__(64) void k_vm_votefe(uint32_t n, VmDev prog, const uint32_t* __restrict__ cst_g, Slab s,
                                                  int32_t* __restrict__ codes, const int32_t* __restrict__ verdict) {
  if (*verdict == 1) return;
  const uint32_t i = blockIdx.x;
  if (i >= n || codes[i] != 0) return;
  const bool ok = fe_one(prog, cst_g, Slab{s.p + (size_t)S_F * 12 * s.cap, s.cap}, i);
  if (threadIdx.x == 0) codes[i] = ok ? 0 : BLST_VERIFY_FAIL;
}

// FE(f) == 1 for the standalone vote (skipped when its code is already an error): *verdict,
// and code BLST_VERIFY_FAIL when the pairing check fails.
__global__ __launch_bounds__(64) void k_vm_final1(VmDev prog, const uint32_t* __restrict__ cst_g, Slab F,
                                                  int32_t* __restrict__ code, int32_t* __restrict__ verdict) {
  if (*code != 0) {
    if (threadIdx.x == 0) *verdict = 0;
    return;
  }
  const bool ok = fe_one(prog, cst_g, F, 0);
  if (threadIdx.x == 0) {
    *verdict = ok ? 1 : 0;
    if (!ok) *code = BLST_VERIFY_FAIL;
  }
}

// The final program on one unit given as (F planes, S planes) at index u (the other three
// partials are the identity): prod F * Miller(-G1, S) -> FE == 1.
__device__ __forceinline__ bool final_one(uint32_t u, const VmDev& prog, const uint32_t* __restrict__ cst_g, Slab inF,
                                          Slab inS) {
  extern __shared__ uint4 lds4[];
  uint32_t* lds = reinterpret_cast<uint32_t*>(lds4);
  uint32_t* cst = lds;
  uint32_t* slots = lds + SLOT_BASE_W;
  const uint32_t lane = threadIdx.x;
  load_consts(cst, cst_g, VM_NCONST);
  for (uint32_t k = lane; k < 4 * PART_PLANES; k += 64) {
    const uint32_t q = k / PART_PLANES, j = k % PART_PLANES;
    Fp v;
    if (q == 0) {
      if (j < 12) inF.ld(v, j, u);
      else inS.ld(v, j - 12, u);
    } else if (j == 0 || j == 12 + 2) {
      fp_one(v);
    } else {
      fp_zero(v);
    }
    slot_put(slots, VM_FINAL_IN[k], v.v);
  }
  __syncthreads();
  vm::run(prog.code, VM_FINAL_NPHASES, VM_FINAL_W, lane, true, slots, cst, 0, vm::Out{nullptr, 0, 0});
  return slot_flag_get(slots, VM_FINAL_OUT[0]) != 0;
}

// Bisection, level 1 (only when the combined check failed, *verdict == 0; verdict null: always):
// grp_ok[g] := the group of votes 16g .. 16g + 15 passes its own combined check.
#define GROUP_VOTES 16
__global__ __launch_bounds__(64) void k_vm_group(uint32_t m, VmDev prog, const uint32_t* __restrict__ cst_g, Slab inF,
                                                 Slab inS, const int32_t* __restrict__ verdict,
                                                 int32_t* __restrict__ grp_ok) {
  if (verdict && *verdict == 1) return;
  const uint32_t g = blockIdx.x;
  if (g >= m) return;
  const bool ok = final_one(g, prog, cst_g, inF, inS);
  if (threadIdx.x == 0) grp_ok[g] = ok ? 1 : 0;
}

// Bisection, vote level: every vote of a failing group whose code is still 0 is checked on its
// own stored (f_i, r_i sigma_i): e(r pk, H) e(-G1, r sigma) = (e(pk, H) / e(G1, sigma))^r,
// r != 0 mod the group order, so it is 1 exactly when the vote verifies (the per-call verdict).
__global__ __launch_bounds__(64) void k_vm_votechk(uint32_t n, VmDev prog, const uint32_t* __restrict__ cst_g, Slab s,
                                                   int32_t* __restrict__ codes, const int32_t* __restrict__ verdict,
                                                   const int32_t* __restrict__ grp_ok) {
  if (verdict && *verdict == 1) return;
  const uint32_t i = blockIdx.x;
  if (i >= n || codes[i] != 0 || grp_ok[i / GROUP_VOTES]) return;
  const bool ok = final_one(i, prog, cst_g, Slab{s.p + (size_t)S_F * 12 * s.cap, s.cap},
                            Slab{s.p + (size_t)S_RS * 12 * s.cap, s.cap});
  if (threadIdx.x == 0) codes[i] = ok ? 0 : BLST_VERIFY_FAIL;
}

// Bisection, first step (skipped when *verdict == 1): r_i sigma_i of every vote with code 0 from
// its stored sigma / tau (program "rs", the vote's RLC value) -> S_RS planes, for the group and
// per-vote checks (the batch path sums these terms by the MSM instead).
constexpr uint32_t RS_STRIDE_W = align256w(VM_RS_NSLOTS * 12);
__global__ __launch_bounds__(64) void k_vm_rs(uint32_t n, VmDev prog, const uint32_t* __restrict__ cst_g, Slab s,
                                              uint64_t seed, uint64_t base, const int32_t* __restrict__ codes,
                                              const int32_t* __restrict__ verdict) {
  if (verdict && *verdict == 1) return;
  extern __shared__ uint4 lds4[];
  uint32_t* lds = reinterpret_cast<uint32_t*>(lds4);
  uint32_t* cst = lds;
  const uint32_t slice = threadIdx.x / VM_RS_W, lane = threadIdx.x % VM_RS_W;
  uint32_t* slots = lds + SLOT_BASE_W + slice * RS_STRIDE_W;
  const uint32_t i = blockIdx.x * (64 / VM_RS_W) + slice;
  const bool active = i < n && codes[i] == 0;
  load_consts(cst, cst_g, VM_NCONST);
  if (active && lane < VM_RS_NIN) {
    Fp v;
    s.ld(v, (lane < 4 ? S_SIG : S_TAU - 4) + lane, i);
    slot_put(slots, VM_RS_IN[lane], v.v);
  }
  __syncthreads();
  vm::run(prog.code, VM_RS_NPHASES, VM_RS_W, lane, active, slots, cst, vote_scalar(seed, base, i),
          vm::Out{s.p, s.cap, i});
}

#define GROUPCHECK_FAIL (0x100 | BLST_POINT_NOT_IN_GROUP)
// aggregate_signatures (consensus.rs:418-444) on the VM: one 96-byte signature per 16-lane slice
// (program "sigchk": decompression + G2 subgroup check) -> the code k_parse_sig_list gives and
// sigma projective (Z = 1; the identity for infinity or a failure) in planes 0..5 of `pts`.
constexpr uint32_t SIGCHK_STRIDE_W = align256w(VM_SIGCHK_NSLOTS * 12 + 4);
__global__ __launch_bounds__(64) void k_vm_sigchk(uint32_t n, VmDev prog, const uint32_t* __restrict__ cst_g,
                                                  const uint8_t* __restrict__ data, const uint64_t* __restrict__ off,
                                                  int gc, int32_t* __restrict__ codes, Slab pts) {
  extern __shared__ uint4 lds4[];
  uint32_t* lds = reinterpret_cast<uint32_t*>(lds4);
  uint32_t* cst = lds;
  const uint32_t slice = threadIdx.x / VM_SIGCHK_W, lane = threadIdx.x % VM_SIGCHK_W;
  uint32_t* slots = lds + SLOT_BASE_W + slice * SIGCHK_STRIDE_W;
  uint32_t* hdr = slots + VM_SIGCHK_NSLOTS * 12;
  const uint32_t i = blockIdx.x * (64 / VM_SIGCHK_W) + slice;
  const bool active = i < n;
  load_consts(cst, cst_g, VM_NCONST);
  if (active && lane == 0) {
    uint32_t x1[12], x0[12], bad, inf, sort, xz;
    parse_hdr(data + off[i], 96, x1, x0, bad, inf, sort, xz);
    slot_put(slots, VM_SIGCHK_IN[VM_SIGCHK_IN_SIG_X1], x1);
    slot_put(slots, VM_SIGCHK_IN[VM_SIGCHK_IN_SIG_X0], x0);
    slot_flag(slots, VM_SIGCHK_IN[VM_SIGCHK_IN_SIG_SORT], sort);
    hdr[0] = bad | inf << 1 | xz << 2;
  }
  __syncthreads();
  vm::run(prog.code, VM_SIGCHK_NPHASES, VM_SIGCHK_W, lane, active, slots, cst, 0, vm::Out{nullptr, 0, 0});
  __syncthreads();
  if (!active) return;
  const uint32_t pf = hdr[0];
  int32_t c = BLST_SUCCESS;
  bool pt = false;
  if (pf & 1) {
    c = BLST_BAD_ENCODING;
  } else if (!(pf & 2)) {  // not the infinity encoding (that one is the identity)
    if (!slot_flag_get(slots, VM_SIGCHK_OUT[VM_SIGCHK_OUT_SIG_OK])) c = BLST_POINT_NOT_ON_CURVE;
    else if (gc && ((pf & 4) || !slot_flag_get(slots, VM_SIGCHK_OUT[VM_SIGCHK_OUT_SIG_GRP]))) c = GROUPCHECK_FAIL;
    else pt = true;
  }
  for (uint32_t k = lane; k < 6; k += VM_SIGCHK_W) {
    Fp v;
    if (pt && k < 4) {
      const uint32_t src = VM_SIGCHK_OUT[VM_SIGCHK_OUT_Q0 + k];
      for (int l = 0; l < 12; ++l) v.v[l] = slots[src * 12 + l];
      vm::canon(v, v);
    } else if (k == (pt ? 4u : 2u)) {
      fp_one(v);
    } else {
      fp_zero(v);
    }
    pts.st(v, k, i);
  }
  if (lane == 0) codes[i] = c;
}

// One level of aggregate_signatures' pairwise sum: out[q] = in[2q] + in[2q + 1] (padd, complete
// formulas; the identity past the end), q < ceil(m / 2), one pair per 8-lane slice.
__global__ __launch_bounds__(64) void k_vm_g2tree(uint32_t m, VmDev prog, uint32_t stride_w,
                                                  const uint32_t* __restrict__ cst_g, Slab in, Slab out) {
  constexpr uint32_t W = VM_PADD_W, SL = 64 / W;
  extern __shared__ uint4 lds4[];
  uint32_t* lds = reinterpret_cast<uint32_t*>(lds4);
  uint32_t* cst = lds;
  const uint32_t slice = threadIdx.x / W, lane = threadIdx.x % W;
  uint32_t* slots = lds + SLOT_BASE_W + slice * stride_w;
  const uint32_t q = blockIdx.x * SL + slice;
  const bool active = q < (m + 1) / 2;
  load_consts(cst, cst_g, VM_NCONST);
  if (active) {
    for (uint32_t k = lane; k < 12; k += W) {
      const uint32_t e = 2 * q + k / 6, c = k % 6;
      Fp v;
      if (e < m) in.ld(v, c, e);
      else if (c == 2) fp_one(v);
      else fp_zero(v);
      slot_put(slots, prog.in[k], v.v);
    }
  }
  __syncthreads();
  vm::run(prog.code, prog.nphases, W, lane, active, slots, cst, 0, vm::Out{nullptr, 0, 0});
  if (active) {
    for (uint32_t k = lane; k < 6; k += W) {
      Fp v;
      const uint32_t src = prog.out[k];
      for (int l = 0; l < 12; ++l) v.v[l] = slots[src * 12 + l];
      vm::canon(v, v);
      out.st(v, k, q);
    }
  }
}

// projective (X : Y : Z) -> Jacobian (X Z, Y Z^2, Z) -> 96-byte compressed (one lane)
__global__ __launch_bounds__(64) void k_g2p_compress(Slab in, uint8_t* out) {
  if (threadIdx.x) return;
  Fp2 X, Y, Z, zz;
  in.ld2(X, 0, 0);
  in.ld2(Y, 2, 0);
  in.ld2(Z, 4, 0);
  G2J j;
  fp2_mul(j.X, X, Z);
  fp2_sqr(zz, Z);
  fp2_mul(j.Y, Y, zz);
  j.Z = Z;
  g2_compress(out, j);
}

// Public keys from secret scalars (ovh_sk_to_pk, ovh_sk_to_pk_batch_device): program pkgen four
// times from the identity, acc -> [2^64] acc + [k] G1 over the scalar's 64-bit chunks (most
// significant first; the secret enters only as selb bits), on a 16-lane slice per key, then one
// lane converts (X : Y : Z) to Jacobian coordinates and compresses (one inversion).
constexpr uint32_t PKGEN_STRIDE_W = align256w(VM_PKGEN_NSLOTS * 12 + 3 * 12);
// bl: a uniform random nonzero blinding factor per key (plane 0, host getrandom): the one-lane
// compression inverts beta Z instead of the secret-dependent Z (its divsteps run variable time)
__global__ __launch_bounds__(64) void k_vm_pkgen(uint32_t n, VmDev prog, const uint32_t* __restrict__ cst_g,
                                                 const uint8_t* __restrict__ sks, uint8_t* __restrict__ out, Slab bl) {
  static_assert(VM_PKGEN_NIN == 3 && VM_PKGEN_NOUT == 3, "pkgen program shape (tools/fpvm/progs.py)");
  constexpr uint32_t W = VM_PKGEN_W;
  extern __shared__ uint4 lds4[];
  uint32_t* lds = reinterpret_cast<uint32_t*>(lds4);
  uint32_t* cst = lds;
  const uint32_t slice = threadIdx.x / W, lane = threadIdx.x % W;
  uint32_t* slots = lds + SLOT_BASE_W + slice * PKGEN_STRIDE_W;
  uint32_t* acc = slots + VM_PKGEN_NSLOTS * 12;  // (X, Y, Z) between the launches
  const uint32_t i = blockIdx.x * (64 / W) + slice;
  const bool active = i < n;
  load_consts(cst, cst_g, VM_NCONST);
  uint64_t k[4] = {0, 0, 0, 0};  // big-endian 64-bit chunks, k[0] the most significant
  if (active) {
    const uint8_t* b = sks + (size_t)i * 32;
    for (int j = 0; j < 4; ++j)
      for (int t = 0; t < 8; ++t) k[j] = k[j] << 8 | b[8 * j + t];
    if (lane < 3)
      for (int l = 0; l < 12; ++l) acc[lane * 12 + l] = lane == 1 ? ONE_M[l] : 0u;  // the identity (0 : 1 : 0)
  }
  __syncthreads();
  for (int r = 0; r < 4; ++r) {
    if (active && lane < 3) slot_put(slots, VM_PKGEN_IN[lane], acc + lane * 12);
    __syncthreads();
    vm::run(prog.code, VM_PKGEN_NPHASES, W, lane, active, slots, cst, k[r], vm::Out{nullptr, 0, 0});
    __syncthreads();
    if (active && lane < 3) {
      Fp t;
      for (int l = 0; l < 12; ++l) t.v[l] = slots[VM_PKGEN_OUT[lane] * 12 + l];
      vm::canon(t, t);
      for (int l = 0; l < 12; ++l) acc[lane * 12 + l] = t.v[l];
    }
    __syncthreads();
  }
  k[0] = k[1] = k[2] = k[3] = 0;
  if (active && lane == 0) {
    Fp X, Y, Z, zz, beta;
    for (int l = 0; l < 12; ++l) {
      X.v[l] = acc[l];
      Y.v[l] = acc[12 + l];
      Z.v[l] = acc[24 + l];
    }
    bl.ld(beta, 0, i);  // (X : Y : Z) = (beta X : beta Y : beta Z)
    fp_mul(X, X, beta);
    fp_mul(Y, Y, beta);
    fp_mul(Z, Z, beta);
    G1J j;  // (X : Y : Z) homogeneous = (X Z : Y Z^2 : Z) Jacobian
    fp_mul(j.X, X, Z);
    fp_sqr(zz, Z);
    fp_mul(j.Y, Y, zz);
    j.Z = Z;
    g1_compress(out + (size_t)i * 48, j);
  }
}

// Crypto::sign (consensus.rs:390-395) by the 4-dimensional GLS decomposition (program signg0
// + 3 x signg1 on a 16-lane slice per signature, u0, u1 from k_h2f; lane 0 of the slice
// computes the digits and compresses the result): k mod r = sum d_i |x|^i with 0 <= d_i < |x| < 2^64, [|x|^i] H =
// (-psi)^i (H), and one 64-step chain acc -> 2 acc + T[b] over the 15 sums T of those points,
// b = the four digits' bits at the step (selb: the secret enters only as select bits; launch j
// takes digit bits 63 - 16 j .. 48 - 16 j, bit 4 t + i of its scalar = bit 48 - 16 j + t of
// d_i). 2,123 phases on a 32-lane slice (2,280 at 16 lanes) against 3,764 for 2-bit windows over the
// 255-bit scalar (r03s: 4.9 -> 3.5 ms).
constexpr uint64_t X_ABS64 = 0xD201000000010000ull;
constexpr uint64_t R64[4] = {0xFFFFFFFF00000001ull, 0x53BDA402FFFE5BFEull, 0x3339D80809A1D805ull,
                             0x73EDA753299D7D48ull};
// little-endian 256-bit n -> digits d (n reduced mod r first: n < 2^256 < 3 r)
__device__ __forceinline__ void gls_digits(uint64_t d[4], uint64_t n[4]) {
  // branch-free on the secret scalar (no early exit, no data-dependent branch): the
  // reductions and the long division select by masks
  for (int rep = 0; rep < 2; ++rep) {  // n >= r -> n - r
    uint64_t t[4], br = 0;
    for (int l = 0; l < 4; ++l) {
      const uint64_t a = n[l], b = R64[l];
      const uint64_t d1 = a - b;
      const uint64_t b1 = (uint64_t)(a < b);
      t[l] = d1 - br;
      br = b1 | (uint64_t)(d1 < br);
    }
    const uint64_t keep = 0ull - br;  // all ones when n < r (the subtraction borrowed)
    for (int l = 0; l < 4; ++l) n[l] = (n[l] & keep) | (t[l] & ~keep);
  }
  for (int i = 0; i < 3; ++i) {  // n /= |x|, d_i = remainder (bit-serial long division)
    uint64_t rem = 0;
    for (int l = 3; l >= 0; --l) {
      uint64_t q = 0;
      for (int b = 63; b >= 0; --b) {
        const uint64_t top = rem >> 63;
        rem = (rem << 1) | ((n[l] >> b) & 1u);
        const uint64_t ge = top | (uint64_t)(rem >= X_ABS64);
        rem -= X_ABS64 & (0ull - ge);
        q |= ge << b;
      }
      n[l] = q;
    }
    d[i] = rem;
  }
  d[3] = n[0];  // n < r < |x|^4: the last quotient is below |x|
}

__device__ __forceinline__ uint64_t signg_scalar(const uint64_t d[4], int j) {
  uint64_t v = 0;
  for (int t = 0; t < 16; ++t)
    for (int i = 0; i < 4; ++i) v |= ((d[i] >> (48 - 16 * j + t)) & 1ull) << (4 * t + i);
  return v;
}

constexpr uint32_t SIGNG_NSLOTS = VM_SIGNG0_NSLOTS > VM_SIGNG1_NSLOTS ? VM_SIGNG0_NSLOTS : VM_SIGNG1_NSLOTS;
constexpr uint32_t SIGNG_STRIDE_W = align256w(SIGNG_NSLOTS * 12 + 96 * 12 + 8);  // + acc, T stash, digits
// bl: a uniform random nonzero Fp2 blinding factor per signature (planes 0, 1; host getrandom),
// multiplied into (X : Y : Z) before the one-lane compression inverts Z (as k_vm_pkgen)
__global__ __launch_bounds__(64) void k_vm_signg(uint32_t n, VmDev p0, VmDev p1, const uint32_t* __restrict__ cst_g,
                                                 const uint8_t* __restrict__ sks, Slab s, uint8_t* __restrict__ out,
                                                 Slab bl) {
  static_assert(VM_SIGNG0_W == VM_SIGNG1_W && VM_SIGNG0_NOUT == 96 && VM_SIGNG1_NIN == 96 && VM_SIGNG1_NOUT == 6,
                "signg program shapes (tools/fpvm/progs.py)");
  constexpr uint32_t W = VM_SIGNG0_W;
  extern __shared__ uint4 lds4[];
  uint32_t* lds = reinterpret_cast<uint32_t*>(lds4);
  uint32_t* cst = lds;
  const uint32_t slice = threadIdx.x / W, lane = threadIdx.x % W;
  uint32_t* slots = lds + SLOT_BASE_W + slice * SIGNG_STRIDE_W;
  uint32_t* hst = slots + SIGNG_NSLOTS * 12;  // 96 values: acc (6), T[1..15] (90)
  uint64_t* dig = reinterpret_cast<uint64_t*>(hst + 96 * 12);  // the four digits
  const uint32_t i = blockIdx.x * (64 / W) + slice;
  const bool active = i < n;
  load_consts(cst, cst_g, VM_NCONST);
  if (active) {
    if (lane == 0) {
      const uint8_t* b = sks + (size_t)i * 32;
      uint64_t k[4] = {0, 0, 0, 0}, d[4];
      for (int j = 0; j < 4; ++j)
        for (int t = 0; t < 8; ++t) k[3 - j] = k[3 - j] << 8 | b[8 * j + t];  // little-endian limbs
      gls_digits(d, k);
      for (int j = 0; j < 4; ++j) dig[j] = d[j];
      k[0] = k[1] = k[2] = k[3] = 0;
      d[0] = d[1] = d[2] = d[3] = 0;
    } else if (lane >= 1 && lane < 5) {
      Fp u;
      s.ld(u, S_U + (lane - 1), i);
      slot_put(slots, VM_SIGNG0_IN[lane - 1], u.v);
    }
  }
  __syncthreads();
  uint64_t d[4] = {0, 0, 0, 0};
  if (active)
    for (int j = 0; j < 4; ++j) d[j] = dig[j];
  vm::run(p0.code, VM_SIGNG0_NPHASES, W, lane, active, slots, cst, signg_scalar(d, 0), vm::Out{nullptr, 0, 0});
  __syncthreads();
  if (active)
    for (uint32_t q = lane; q < 96; q += W)
      for (int l = 0; l < 12; ++l) hst[q * 12 + l] = slots[VM_SIGNG0_OUT[q] * 12 + l];
  __syncthreads();
  for (int r = 1; r < 4; ++r) {
    if (active)
      for (uint32_t q = lane; q < 96; q += W) slot_put(slots, VM_SIGNG1_IN[q], hst + q * 12);
    __syncthreads();
    vm::run(p1.code, VM_SIGNG1_NPHASES, W, lane, active, slots, cst, signg_scalar(d, r), vm::Out{nullptr, 0, 0});
    __syncthreads();
    if (active && lane < 6)
      for (int l = 0; l < 12; ++l) hst[lane * 12 + l] = slots[VM_SIGNG1_OUT[lane] * 12 + l];
    __syncthreads();
  }
  d[0] = d[1] = d[2] = d[3] = 0;
  if (active && lane < 4) dig[lane] = 0;
  if (active && lane < 6) {
    Fp t;
    for (int l = 0; l < 12; ++l) t.v[l] = hst[lane * 12 + l];
    vm::canon(t, t);
    for (int l = 0; l < 12; ++l) hst[lane * 12 + l] = t.v[l];
  }
  __syncthreads();
  if (active && lane == 0) {
    Fp2 X, Y, Z, zz;
    for (int l = 0; l < 12; ++l) {
      X.c0.v[l] = hst[l];
      X.c1.v[l] = hst[12 + l];
      Y.c0.v[l] = hst[24 + l];
      Y.c1.v[l] = hst[36 + l];
      Z.c0.v[l] = hst[48 + l];
      Z.c1.v[l] = hst[60 + l];
    }
    Fp2 beta;
    bl.ld2(beta, 0, i);
    fp2_mul(X, X, beta);
    fp2_mul(Y, Y, beta);
    fp2_mul(Z, Z, beta);
    G2J j;
    fp2_mul(j.X, X, Z);
    fp2_sqr(zz, Z);
    fp2_mul(j.Y, Y, zz);
    j.Z = Z;
    g2_compress(out + (size_t)i * 96, j);
  }
}

#include "msm.hpp"

// Validator table (ovh_set_validators) and the keys of verify_aggregated_signature: one 48-byte
// compressed key per 16-lane slice (program "pkchk": decompression + G1 subgroup check) -> flags
// + the point (X : Y : Z) Montgomery, (0 : 1 : 0) for infinity or a failed parse. Flag precedence
// as the vote kernel's (k_vm_vote): bad encoding, off the curve or x = 0 -> PKF_PARSE.
constexpr uint32_t PKCHK_STRIDE_W = align256w(VM_PKCHK_NSLOTS * 12 + 4);
__global__ __launch_bounds__(64) void k_vm_pkchk(uint32_t n, VmDev prog, const uint32_t* __restrict__ cst_g,
                                                 const uint8_t* __restrict__ pks, Slab pts, uint32_t* __restrict__ flags) {
  extern __shared__ uint4 lds4[];
  uint32_t* lds = reinterpret_cast<uint32_t*>(lds4);
  uint32_t* cst = lds;
  const uint32_t slice = threadIdx.x / VM_PKCHK_W, lane = threadIdx.x % VM_PKCHK_W;
  uint32_t* slots = lds + SLOT_BASE_W + slice * PKCHK_STRIDE_W;
  uint32_t* hdr = slots + VM_PKCHK_NSLOTS * 12;
  const uint32_t i = blockIdx.x * (64 / VM_PKCHK_W) + slice;
  const bool active = i < n;
  load_consts(cst, cst_g, VM_NCONST);
  if (active && lane == 0) {
    uint32_t x[12], bad, inf, sort, xz;
    parse_hdr(pks + (size_t)i * 48, 48, x, x, bad, inf, sort, xz);
    slot_put(slots, VM_PKCHK_IN[VM_PKCHK_IN_PK_X], x);
    slot_flag(slots, VM_PKCHK_IN[VM_PKCHK_IN_PK_SORT], sort);
    hdr[0] = bad | inf << 1 | xz << 2;
  }
  __syncthreads();
  vm::run(prog.code, VM_PKCHK_NPHASES, VM_PKCHK_W, lane, active, slots, cst, 0, vm::Out{nullptr, 0, 0});
  __syncthreads();
  if (!active) return;
  const uint32_t pf = hdr[0];
  uint32_t f = 0;
  if ((pf & 1) || (!(pf & 2) && (!slot_flag_get(slots, VM_PKCHK_OUT[VM_PKCHK_OUT_PK_OK]) || (pf & 4)))) f = PKF_PARSE;
  else if (pf & 2) f = PKF_INF;
  else if (!slot_flag_get(slots, VM_PKCHK_OUT[VM_PKCHK_OUT_PK_GRP])) f = PKF_GRP;
  const bool pt = f == 0 || f == PKF_GRP;
  for (uint32_t k = lane; k < 3; k += VM_PKCHK_W) {
    Fp v;
    if (pt && k < 2) {
      const uint32_t src = VM_PKCHK_OUT[VM_PKCHK_OUT_P0 + k];
      for (int l = 0; l < 12; ++l) v.v[l] = slots[src * 12 + l];
      vm::canon(v, v);
    } else if (k == (pt ? 2u : 1u)) {
      fp_one(v);
    } else {
      fp_zero(v);
    }
    pts.st(v, k, i);
  }
  if (lane == 0) flags[i] = f;
}

// One level of an aggregated key's pairwise sum: out[q] = in[2q] + in[2q + 1] (g1padd, complete
// formulas; the identity past the end), one pair per 8-lane slice.
__global__ __launch_bounds__(64) void k_vm_g1tree(uint32_t m, VmDev prog, uint32_t stride_w,
                                                  const uint32_t* __restrict__ cst_g, Slab in, Slab out) {
  constexpr uint32_t W = VM_G1PADD_W, SL = 64 / W;
  extern __shared__ uint4 lds4[];
  uint32_t* lds = reinterpret_cast<uint32_t*>(lds4);
  uint32_t* cst = lds;
  const uint32_t slice = threadIdx.x / W, lane = threadIdx.x % W;
  uint32_t* slots = lds + SLOT_BASE_W + slice * stride_w;
  const uint32_t q = blockIdx.x * SL + slice;
  const bool active = q < (m + 1) / 2;
  load_consts(cst, cst_g, VM_NCONST);
  if (active) {
    for (uint32_t k = lane; k < 6; k += W) {
      const uint32_t e = 2 * q + k / 3, c = k % 3;
      Fp v;
      if (e < m) in.ld(v, c, e);
      else if (c == 1) fp_one(v);
      else fp_zero(v);
      slot_put(slots, prog.in[k], v.v);
    }
  }
  __syncthreads();
  vm::run(prog.code, prog.nphases, W, lane, active, slots, cst, 0, vm::Out{nullptr, 0, 0});
  if (active) {
    for (uint32_t k = lane; k < 3; k += W) {
      Fp v;
      const uint32_t src = prog.out[k];
      for (int l = 0; l < 12; ++l) v.v[l] = slots[src * 12 + l];
      vm::canon(v, v);
      out.st(v, k, q);
    }
  }
}

// element 0 of a tree's last level -> the QC key slot (out element 0), PKF_INF when it is O
__global__ __launch_bounds__(64) void k_apk_finish(Slab in, Slab out, uint32_t* __restrict__ flags) {
  const uint32_t k = threadIdx.x;
  if (k >= 3) return;
  Fp v;
  in.ld(v, k, 0);
  out.st(v, k, 0);
  if (k == 2) {
    uint32_t z = 0;
    for (int l = 0; l < 12; ++l) z |= v.v[l];
    flags[0] = z ? 0u : PKF_INF;
  }
}

// verify_aggregated_signature when some key is outside G1 (BlsPublicKey::aggregate does not
// group-check; blst's verify checks the aggregated key, consensus.rs:371,378-380): program g1grp
// on element 0 of `apk` (one 16-lane slice) -> PKF_GRP in flags[0] when the sum is not in G1
// (an infinite sum keeps PKF_INF, which takes precedence in k_vm_qcmil).
constexpr uint32_t G1GRP_STRIDE_W = align256w(VM_G1GRP_NSLOTS * 12);
__global__ __launch_bounds__(64) void k_vm_g1grp(VmDev prog, const uint32_t* __restrict__ cst_g, Slab apk,
                                                 uint32_t* __restrict__ flags) {
  extern __shared__ uint4 lds4[];
  uint32_t* lds = reinterpret_cast<uint32_t*>(lds4);
  uint32_t* cst = lds;
  const uint32_t slice = threadIdx.x / VM_G1GRP_W, lane = threadIdx.x % VM_G1GRP_W;
  uint32_t* slots = lds + SLOT_BASE_W;
  const bool active = slice == 0;
  load_consts(cst, cst_g, VM_NCONST);
  if (active && lane < 3) {
    Fp v;
    apk.ld(v, lane, 0);
    slot_put(slots, VM_G1GRP_IN[lane], v.v);
  }
  __syncthreads();
  vm::run(prog.code, VM_G1GRP_NPHASES, VM_G1GRP_W, lane, active, slots, cst, 0, vm::Out{nullptr, 0, 0});
  if (active && lane == 0 && !(flags[0] & PKF_INF) && !slot_flag_get(slots, VM_G1GRP_OUT[VM_G1GRP_OUT_PK_GRP]))
    flags[0] |= PKF_GRP;
}

// QC batch: one workgroup per QC, apk = sum of the table keys selected by the QC's voter list
// (sorted-order indices, CSR): each lane sums a strided share (Jacobian), then a 6-level LDS tree;
// out = homogeneous projective (X Z : Y : Z^3); flags: PKF_INF when the sum is O.
__global__ __launch_bounds__(64) void k_qc_apk(uint32_t nq, const uint32_t* __restrict__ off,
                                               const uint32_t* __restrict__ ent, Slab table, Slab out,
                                               uint32_t* __restrict__ flags) {
  __shared__ uint32_t red[64 * 36];
  const uint32_t q = blockIdx.x, t = threadIdx.x;
  if (q >= nq) return;
  G1J acc, x;
  jac_set_inf(acc);
  for (uint32_t k = off[q] + t; k < off[q + 1]; k += 64) {
    const uint32_t e = ent[k];
    table.ld(x.X, 0, e);
    table.ld(x.Y, 1, e);
    table.ld(x.Z, 2, e);
    jac_add(acc, acc, x);
  }
  for (uint32_t s = 32; s >= 1; s >>= 1) {
    if (t >= s && t < 2 * s) {
      for (int l = 0; l < 12; ++l) {
        red[(t - s) * 36 + l] = acc.X.v[l];
        red[(t - s) * 36 + 12 + l] = acc.Y.v[l];
        red[(t - s) * 36 + 24 + l] = acc.Z.v[l];
      }
    }
    __syncthreads();
    if (t < s) {
      for (int l = 0; l < 12; ++l) {
        x.X.v[l] = red[t * 36 + l];
        x.Y.v[l] = red[t * 36 + 12 + l];
        x.Z.v[l] = red[t * 36 + 24 + l];
      }
      jac_add(acc, acc, x);
    }
    __syncthreads();
  }
  if (t) return;
  Fp X, Y, Z;
  uint32_t f = 0;
  if (jac_is_inf(acc)) {
    fp_zero(X);
    fp_one(Y);
    fp_zero(Z);
    f = PKF_INF;
  } else {
    Fp zz;
    fp_mul(X, acc.X, acc.Z);
    Y = acc.Y;
    fp_sqr(zz, acc.Z);
    fp_mul(Z, zz, acc.Z);
  }
  out.st(X, 0, q);
  out.st(Y, 1, q);
  out.st(Z, 2, q);
  flags[q] = f;
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
// ovh_verify with other encodings (uncompressed keys / signatures, other lengths): parse them
// with blst's from_bytes semantics (ec.hpp; an uncompressed point costs an on-curve check, a few
// products) and write the compressed form of one staged vote, so the vote runs the fixed-size
// path (vote1 + final1). A parsed point is re-encoded (the compressed path decompresses it to the
// same point); a failure is replaced by a compressed encoding that fails the same way in the same
// place: x >= p (BAD_ENCODING; for the key every failure is 102 in verify_one's order, 
// consensus.rs:406-407), an x with x^3 + 4 (1 + i) not a square (POINT_NOT_ON_CURVE).
__device__ __noinline__ void canon_sig(const uint8_t* __restrict__ sig, uint32_t sl, uint8_t* __restrict__ sig96) {
  if (sl == 96 && (sig[0] & 0x80)) {
    for (int i = 0; i < 96; ++i) sig96[i] = sig[i];
    return;
  }
  G2A a;
  bool inf;
  const int e = g2_from_bytes(a, inf, sig, sl);
  for (int i = 0; i < 96; ++i) sig96[i] = 0;
  if (e == BLST_SUCCESS && inf) {
    sig96[0] = 0xc0;
  } else if (e == BLST_SUCCESS || e == BLST_POINT_NOT_IN_GROUP) {  // x = 0 (never on E2)
    fp_to_be48(sig96, a.x.c1);
    fp_to_be48(sig96 + 48, a.x.c0);
    sig96[0] |= 0x80 | (fp2_lex_largest(a.y) ? 0x20 : 0);
  } else if (e == BLST_POINT_NOT_ON_CURVE) {
    sig96[0] = 0x80;  // x = 1: 5 + 4i is not a square in Fp2
    sig96[95] = 1;
  } else {
    sig96[0] = 0x9f;
    for (int i = 1; i < 96; ++i) sig96[i] = 0xff;
  }
}

__device__ __noinline__ void canon_pk(const uint8_t* __restrict__ pk, uint32_t pl, uint8_t* __restrict__ pk48) {
  if (pl == 48 && (pk[0] & 0x80)) {
    for (int i = 0; i < 48; ++i) pk48[i] = pk[i];
    return;
  }
  G1A a;
  bool inf;
  const int e = g1_from_bytes(a, inf, pk, pl);
  for (int i = 0; i < 48; ++i) pk48[i] = 0;
  if (e == BLST_SUCCESS && inf) {
    pk48[0] = 0xc0;
  } else if (e == BLST_SUCCESS) {
    fp_to_be48(pk48, a.x);
    pk48[0] |= 0x80 | (fp_lex_largest(a.y) ? 0x20 : 0);
  } else {
    pk48[0] = 0x9f;
    for (int i = 1; i < 48; ++i) pk48[i] = 0xff;
  }
}

__global__ __launch_bounds__(64) void k_canon_one(const uint8_t* __restrict__ sig, uint32_t sl,
                                                  const uint8_t* __restrict__ pk, uint32_t pl, uint8_t* __restrict__ sig96,
                                                  uint8_t* __restrict__ pk48) {
  if (threadIdx.x != 0) return;
  canon_sig(sig, sl, sig96);
  canon_pk(pk, pl, pk48);
}

// verify_aggregated_signature with other encodings: key i re-encoded to out[48 i, 48 i + 48),
// the signature to out[48 n, 48 n + 96) (one lane per item).
__global__ __launch_bounds__(WG) void k_canon_qc(uint32_t n, const uint8_t* __restrict__ data,
                                                 const uint64_t* __restrict__ off, const uint64_t* __restrict__ len,
                                                 const uint8_t* __restrict__ sig, uint32_t sl, uint8_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i < n) canon_pk(data + off[i], (uint32_t)len[i], out + (size_t)48 * i);
  if (i == n) canon_sig(sig, sl, out + (size_t)48 * n);
}

// ovh_aggregate_sigs over a list with other encodings: item i re-encoded to out[96 i, 96 i + 96)
// (one lane per item), then the list runs k_vm_sigchk as a compressed one; offs[i] = 96 i.
__global__ __launch_bounds__(WG) void k_canon_sig_list(uint32_t n, const uint8_t* __restrict__ data,
                                                       const uint64_t* __restrict__ off, const uint64_t* __restrict__ len,
                                                       uint8_t* __restrict__ out, uint64_t* __restrict__ offs) {
  const uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  canon_sig(data + off[i], (uint32_t)len[i], out + (size_t)96 * i);
  offs[i] = (uint64_t)96 * i;
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

// aggregate_signatures' key validation on the VM (program pkdec: the decompression alone, no
// subgroup check -- the keys are only parsed, consensus.rs:435-436), one 48-byte key per 4-lane
// slice: codes[i] = BLST_SUCCESS or the parse failure as k_parse_pk_list reports it (bad
// encoding, off the curve, x = 0; infinity parses).
constexpr uint32_t PKDEC_STRIDE_W = align128w(VM_PKDEC_NSLOTS * 12 + 4);
__global__ __launch_bounds__(64) void k_vm_pkdec(uint32_t n, VmDev prog, const uint32_t* __restrict__ cst_g,
                                                 const uint8_t* __restrict__ data, const uint64_t* __restrict__ off,
                                                 int32_t* __restrict__ codes) {
  constexpr uint32_t W = VM_PKDEC_W, SL = 64 / W;
  extern __shared__ uint4 lds4[];
  uint32_t* lds = reinterpret_cast<uint32_t*>(lds4);
  uint32_t* cst = lds;
  const uint32_t slice = threadIdx.x / W, lane = threadIdx.x % W;
  uint32_t* slots = lds + SLOT_BASE_W + slice * PKDEC_STRIDE_W;
  uint32_t* hdr = slots + VM_PKDEC_NSLOTS * 12;
  const uint32_t i = blockIdx.x * SL + slice;
  const bool active = i < n;
  load_consts(cst, cst_g, VM_NCONST);
  if (active && lane == 0) {
    uint32_t x[12], bad, inf, sort, xz;
    parse_hdr(data + off[i], 48, x, x, bad, inf, sort, xz);
    slot_put(slots, VM_PKDEC_IN[VM_PKCHK_IN_PK_X], x);
    slot_flag(slots, VM_PKDEC_IN[VM_PKCHK_IN_PK_SORT], sort);
    hdr[0] = bad | inf << 1 | xz << 2;
  }
  __syncthreads();
  vm::run(prog.code, VM_PKDEC_NPHASES, W, lane, active, slots, cst, 0, vm::Out{nullptr, 0, 0});
  if (active && lane == 0) {
    const uint32_t pf = hdr[0];
    int32_t c = BLST_SUCCESS;
    if (pf & 1) c = BLST_BAD_ENCODING;
    else if (!(pf & 2) && !slot_flag_get(slots, VM_PKDEC_OUT[VM_PKDEC_OUT_PK_OK])) c = BLST_POINT_NOT_ON_CURVE;
    else if (!(pf & 2) && (pf & 4)) c = BLST_POINT_NOT_IN_GROUP;  // x = 0: (0, +-2) has order 3
    codes[i] = c;
  }
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

// ------------------------------------------------------------------------ host side
// Validator table (ovh_set_validators): keys as points in HBM + host lookup structures.
struct ValidatorTable {
  uint32_t n = 0, cap = 0;
  uint32_t* planes = nullptr;   // X, Y, Z planes of `cap` entries
  uint32_t* flags = nullptr;    // device PKF_* per entry
  std::vector<uint32_t> hflags;  // host copy
  std::vector<std::string> keys;
  std::unordered_map<std::string, uint32_t> index;  // key bytes -> first entry
  std::vector<uint32_t> sorted;                     // entries by key bytes (overlord authority order)
};

// Verdict cache of ovh_prefetch: exact (sig, hash, voter) bytes -> per-vote code.
struct VerdictCache {
  std::mutex mu;
  std::unordered_map<std::string, int32_t> map;
  std::deque<std::string> fifo;
  size_t cap = 1u << 16;
  uint64_t hits = 0, misses = 0;
};

// A pipelined host-buffer batch in flight (ovh_verify_batch_async): per device its shard, the
// staging order (table_split perm) and the ring slot whose pinned buffer receives its codes.
struct HostBatch {
  int32_t* codes = nullptr;  // the caller's, written when the batch completes
  size_t n = 0;
  int ring = 0;
  struct Dev {
    size_t d, lo, cnt;
    std::vector<uint32_t> perm;
  };
  std::vector<Dev> dev;
};

#define NFIN_STREAMS 4u
struct ovh_ctx {
  int device = 0;
  uint32_t flags = 0;
  hipStream_t stream = nullptr;
  // pipelined batches (ovh_verify_batch_device_async): the per-vote work of every batch runs in
  // the vote pool (pool_st, high priority); batch k's fold levels, MSM, final check and bisection
  // on a final stream (lowest priority) while later batches' votes run. OVH_BATCH_SLOTS slots of
  // batch state rotate (a slot is reused only after its final-stream work finished). Batches
  // take the NFIN_STREAMS final streams in turn, so that many chains run at once.
  hipStream_t fstream = nullptr, fstream2 = nullptr, fstream3 = nullptr;
  hipStream_t fstream4 = nullptr;
  uint32_t nfin = NFIN_STREAMS;  // final streams in turn (OVH_NFIN: 2, 3 or 4, A/B)
  hipStream_t xstream = nullptr;  // per-call side work beside `stream` (aggregate_signatures' key parse; lazy)
  // ovh_verify_samemsg_device_async: [0], [1] the per-vote streams, in turn; [2] hash_to_G2 (lazy)
  hipStream_t vstream[3] = {};
  hipStream_t hstream[4] = {};  // the one-hash API's hash_to_G2 streams in turn ([0] unused: xstream; lazy)
  // the vote pool (k_vm_pool): its two streams (created with the context, high priority), the
  // device queue (PQ_WORDS words), the published batches' descriptors (one per slot), the
  // workgroups' spill scratch (2 x pool_wgs x 4 x VOTE_NSCR entries: one area per pool stream),
  // the grid size, the next batch's sequence number, and the timeout flag of k_pool_wait
  // (coherent host memory)
  hipStream_t pool_st[3] = {};  // every batch has a pool grid on [0] and [1] (see batch_front); [2]: OVH_SHARD_STREAMS
  uint64_t* pool_q = nullptr;
  void* pool_desc = nullptr;
  uint32_t* pool_scr = nullptr;
  uint32_t pool_wgs = 0;
  uint32_t pool_grid0 = 0;  // workgroups of pool stream 0's grid (4 per CU); stream 1's: 2 pool_wgs - it
  uint32_t ncu = 256;
  // OVH_FLAG_POOL_RESERVE: CUs left free of the pool, pool_rsv / 8 per XCC (0: none), and the
  // CUs the pool runs on (ncu - pool_rsv: SIMD spreading)
  uint32_t pool_rsv = 0;
  uint32_t pool_ncu = 256;
  uint64_t pool_seq = 0;
  uint32_t* pool_err = nullptr;
  uint64_t* plog = nullptr;  // OVH_FLAG_VM_CLOCK: the pool log (PLOG_RING records)
  uint64_t plog_seq[OVH_BATCH_SLOTS] = {};  // the seq of the batch in each slot
  uint64_t plog_grids = 0;
  hipStream_t fs[OVH_BATCH_SLOTS] = {};  // final stream of the batch in each slot (take_slot)
  hipEvent_t ev_front[OVH_BATCH_SLOTS] = {}, ev_back[OVH_BATCH_SLOTS] = {};
  hipEvent_t ev_x[4] = {};  // stream-order handoffs with a caller's stream / other devices
  // per slot: the state slab, the fold regions R0..R3 (R1: the 16-vote groups) and the pool's
  // staged inputs -- views into one allocation each (slot k at k x the stride: PoolArgs)
  uint32_t* state_slot[OVH_BATCH_SLOTS] = {};
  uint32_t* red_slot[OVH_BATCH_SLOTS] = {};
  uint32_t *state_all = nullptr, *red_all = nullptr;
  uint8_t* pstage_all = nullptr;
  size_t state_w = 0, red_w = 0, pstage_b = 0;
  int32_t* grp_ok[OVH_BATCH_SLOTS] = {};
  uint32_t slot_n[OVH_BATCH_SLOTS] = {};
  uint32_t* fin = nullptr;  // OVH_BATCH_SLOTS x FIN_STRIDE words: per-slot combine scratch
  uint32_t pipe_k = 0;
  int last_slot = 0;
  // batches of 2 .. small_max votes checked alone run the small-batch path (verify_small_locked);
  // OVH_SMALL_MAX=0 turns it off (A/B builds and tests of the standard path)
  uint32_t small_max = SMALL_MAX;
  XmdTemplates xmd;
  std::mutex mu;  // Crypto is Send + Sync: every entry point holds it for its whole call
  uint32_t cap = 0, red_cap = 0;
  uint8_t* in_buf = nullptr;   // staging for host inputs
  size_t in_cap = 0;
  // single-call scratch (aggregation, sums): separate from the batch slots
  uint32_t* scr = nullptr;
  int32_t *scr_pk = nullptr, *scr_sig = nullptr;
  uint32_t scr_cap = 0;
  uint32_t* comb = nullptr;  // ovh_combine_partials_device scratch
  uint32_t comb_cap = 0;
  uint32_t* part_out = nullptr;  // multi-device: this device's partials (ring slot x {table, other votes} x 216 words)
  int32_t* result = nullptr;     // device verdict words
  uint32_t last_n = 0;
  // RLC coefficients: fresh getrandom seed per batch, or the test seed (OVH_FLAG_TEST_RLC)
  uint64_t test_seed = 0, test_base = 0;
  ValidatorTable tab;
  uint32_t* qc_buf = nullptr;  // QC batch: apk planes + flags
  uint32_t qc_cap = 0;
  uint32_t* qt_buf = nullptr;  // explicit-key QC (ovh_verify_aggregated): decoded keys + flags
  uint32_t qt_cap = 0;
  VerdictCache cache;
  // multi-device (ovh_create_multi): sub-contexts, one per device; the root owns no streams
  std::vector<ovh_ctx*> sub;
  std::atomic<uint32_t> rr{0};
  std::vector<uint8_t> peer;   // sub.size()^2: peer[a * n + b] = device a reaches b's memory (xGMI)
  std::vector<int> fin_devs;   // sub indices the pipelined combined check rotates over
  uint8_t* gather = nullptr;  // on sub[0]'s device: ndev x 864 B
  uint32_t* mfin = nullptr;   // on sub[0]'s device: unpack scratch of the gathered partials
  // Pippenger MSM scratch per batch slot (msm.hpp: counts, offsets, level prefixes, sorted
  // entries, bucket trees, bit-plane sums) and the slot's RLC seed (the bisection's k_vm_rs)
  uint32_t* msm_buf[OVH_BATCH_SLOTS] = {};
  uint64_t slot_seed[OVH_BATCH_SLOTS] = {}, slot_base[OVH_BATCH_SLOTS] = {};
  // pipelined host batches (ovh_verify_batch_async): per ring slot a pinned host staging buffer
  // (inputs, then the codes read back) and its device copy; events per ring slot: [0], [1] the
  // packed partials of the slot's two parts, [2] the combined verdict (final device), [3] the codes
  // in the pinned buffer
  uint8_t* hst_h[OVH_BATCH_SLOTS] = {};
  uint8_t* hst_d[OVH_BATCH_SLOTS] = {};
  size_t hst_cap[OVH_BATCH_SLOTS] = {};
  hipEvent_t ev_m[OVH_BATCH_SLOTS][4] = {};
  uint8_t* mg = nullptr;  // as a multi context's final device: OVH_BATCH_SLOTS x 16 gathered partials
  std::deque<HostBatch> hq;  // batches in flight (the root context / a single context)
  uint64_t hb_k = 0;
  // Fp-VM programs + constant table in device memory
  // same-message batches (verify_samemsg_locked): programs, per slot the group slab (G_PLANES
  // planes + the H-is-infinity words, gcap entries); OVH_SAMEMSG=0 turns the path off
  VmDev vm_vsame{}, vm_vsame_t{}, vm_vsame8{}, vm_vsame8_t{}, vm_h2g{}, vm_gmil{}, vm_pkdec{}, vm_g1grp{}, vm_gfin{};
  uint32_t* gslab[OVH_BATCH_SLOTS] = {};
  uint32_t gcap[OVH_BATCH_SLOTS] = {};
  // 0: off; 1 (default): batches above small_max votes (below it the small-batch path has the
  // lower latency); 2: every batch with at most n / 2 distinct hashes
  int samemsg = 1;
  // the shard path's grid per batch also claims the next shard_span batches' quads (OVH_SHARD_SPAN,
  // A/B): it leaves once batch seq + shard_span is claimed, so the grid two batches on finds the
  // stream free while the caller's collective still gets places between grids
  uint32_t shard_span = 0;
  // pool streams the shard path's grids rotate over (OVH_SHARD_STREAMS, A/B: 2 or 3)
  uint32_t shard_streams = 2;
  // a pool batch's signatures | keys | table indices, staged per slot (k_pool_stage; views)
  uint8_t* pstage[OVH_BATCH_SLOTS] = {};
  uint64_t sm_batches = 0, sm_votes = 0, sm_hashes = 0;
  // ovh_verify_samemsg_device_async: the one-hash plan of sm1_n votes (gid = 0 | head 0 | pairs)
  // and its level offsets; the hash of each slot (32 B per slot)
  uint32_t* sm1_plan = nullptr;
  size_t sm1_n = 0;
  std::vector<uint32_t> sm1_lo;
  uint8_t* sm1_hash = nullptr;
  VmDev vm_vote{}, vm_vote_t{}, vm_fold{}, vm_final{}, vm_rs{}, vm_madd{}, vm_padd{}, vm_hdbl[5]{}, vm_sigchk{},
      vm_pkchk{}, vm_g1padd{}, vm_vote1{}, vm_vote_t1{}, vm_final1{}, vm_votew{},
      vm_votew_t{}, vm_qcpre{}, vm_qcmil{}, vm_vote1h{}, vm_vote_t1h{}, vm_pkgen{}, vm_signg0{}, vm_signg1{};
  // message cache (verify_one_locked): H = hash_to_G2(hash) of the last HC_CAP hashes verified
  // per call, projective planes + H-is-infinity flags, FIFO replacement
  uint32_t* hc_planes = nullptr;
  uint32_t* hc_inf = nullptr;
  std::unordered_map<std::string, uint32_t> hc_index;
  std::vector<std::string> hc_keys;
  uint32_t hc_next = 0;
  uint64_t hc_hits = 0, hc_misses = 0;
  uint32_t* vm_consts = nullptr;
  std::vector<void*> vm_bufs;
  uint32_t clk_wgs = 0;    // OVH_FLAG_VM_CLOCK: workgroups of the last vote launch
  bool clk_table = false;  // ... and whether it was vote_t
  std::vector<uint32_t> blind_h;  // host copy of the last compression blinds (upload_blinds)
  // OVH_FLAG_PROFILE: start/stop events per stage of the last batch call
  hipEvent_t ev0[OVH_NSTAGES] = {}, ev1[OVH_NSTAGES] = {};
  // OVH_FLAG_PROFILE: start / end events of the last VEV_CAP batch vote kernels (ovh_vote_spans:
  // pipelined vote grids overlap, so their device-level rate is the work over the union span)
  static constexpr uint32_t VEV_CAP = 256;
  hipEvent_t vev0[VEV_CAP] = {}, vev1[VEV_CAP] = {};
  uint32_t vev_n = 0;
  uint32_t ev_mask = 0;
};

#define HIPCHK(x)                                  \
  do {                                             \
    if ((x) != hipSuccess) return OVH_ERR_DEVICE;  \
  } while (0)
#define CHK(x)                \
  do {                              \
    const int e_ = (x);             \
    if (e_) return e_;              \
  } while (0)

static const char* const STAGE_NAMES[OVH_NSTAGES] = {"hash_to_field", "vote", "fold", "final", "bisect", "msm"};

// LDS bytes of the VM kernels: constants + slices x slots (+ a 16-byte slice header for vote)
static constexpr size_t LDS_VOTE = ((size_t)SLOT_BASE_W + VM_SLICES * (size_t)VOTE_STRIDE_W) * 4;
static constexpr size_t LDS_VOTE_T = ((size_t)SLOT_BASE_W + VM_SLICES * (size_t)VOTE_T_STRIDE_W) * 4;
static constexpr size_t LDS_FOLD = ((size_t)SLOT_BASE_W + VM_FOLD_UNITS * (size_t)FOLD_STRIDE_W) * 4;
static constexpr size_t LDS_FINAL = ((size_t)SLOT_BASE_W + (size_t)VM_FINAL_NSLOTS * 12) * 4;
static_assert(VM_VOTE_W * VM_SLICES == 64 && VM_VOTE_T_W * VM_SLICES == 64 && VM_FOLD_W * VM_FOLD_UNITS == 64 &&
                  VM_FINAL_W == 64, "VM slice widths");
static constexpr size_t LDS_FOLD1 = ((size_t)SLOT_BASE_W + (size_t)FOLD_STRIDE_W) * 4;
// bisection r sigma and the MSM pair kernels (8-lane madd / padd, 16-lane hdbl<m>)
static constexpr size_t LDS_RS = ((size_t)SLOT_BASE_W + (64 / VM_RS_W) * (size_t)RS_STRIDE_W) * 4;
constexpr uint32_t cmax(uint32_t a, uint32_t b) { return a > b ? a : b; }
static constexpr uint32_t MSM8_STRIDE_W = align128w(cmax(VM_MADD_NSLOTS, VM_PADD_NSLOTS) * 12);
static constexpr uint32_t HDBL_STRIDE_W =
    align128w(cmax(cmax(cmax(VM_HDBL1_NSLOTS, VM_HDBL2_NSLOTS), cmax(VM_HDBL4_NSLOTS, VM_HDBL8_NSLOTS)), VM_HDBL16_NSLOTS) * 12);
static constexpr size_t LDS_MSM8 = ((size_t)SLOT_BASE_W + (64 / VM_MADD_W) * (size_t)MSM8_STRIDE_W) * 4;
static constexpr size_t LDS_HDBL = ((size_t)SLOT_BASE_W + (64 / VM_HDBL1_W) * (size_t)HDBL_STRIDE_W) * 4;
static_assert(VM_MADD_W == VM_PADD_W && VM_HDBL1_W == VM_HDBL2_W && VM_HDBL1_W == VM_HDBL4_W && VM_HDBL1_W == VM_HDBL8_W &&
                  VM_HDBL1_W == VM_HDBL16_W && VM_MADD_NIN == 10 && VM_PADD_NIN == 12 && VM_HDBL1_NIN == 12,
              "MSM program shapes (tools/fpvm/progs.py)");
static constexpr size_t LDS_SIGCHK = ((size_t)SLOT_BASE_W + (64 / VM_SIGCHK_W) * (size_t)SIGCHK_STRIDE_W) * 4;
static constexpr uint32_t VOTE1_NSLOTS = VM_VOTE1_NSLOTS > VM_VOTE_T1_NSLOTS ? VM_VOTE1_NSLOTS : VM_VOTE_T1_NSLOTS;
static constexpr size_t LDS_VOTE1 = ((size_t)SLOT_BASE_W + VOTE1_NSLOTS * 12 + 4) * 4;
static constexpr uint32_t VOTE1H_NSLOTS = VM_VOTE1H_NSLOTS > VM_VOTE_T1H_NSLOTS ? VM_VOTE1H_NSLOTS : VM_VOTE_T1H_NSLOTS;
static constexpr size_t LDS_VOTE1H = ((size_t)SLOT_BASE_W + VOTE1H_NSLOTS * 12 + 4) * 4;
static constexpr uint32_t VOTEW_NSLOTS = VM_VOTEW_NSLOTS > VM_VOTEW_T_NSLOTS ? VM_VOTEW_NSLOTS : VM_VOTEW_T_NSLOTS;
static constexpr size_t LDS_VOTEW = ((size_t)SLOT_BASE_W + VOTEW_NSLOTS * 12 + 4) * 4;
static constexpr size_t LDS_QCPRE = ((size_t)SLOT_BASE_W + VM_QCPRE_NSLOTS * 12 + 4) * 4;
static constexpr size_t LDS_QCMIL = ((size_t)SLOT_BASE_W + VM_QCMIL_NSLOTS * 12) * 4;
static constexpr size_t LDS_FINAL1 = ((size_t)SLOT_BASE_W + (size_t)VM_FINAL1_NSLOTS * 12) * 4;
static constexpr size_t LDS_SIGNG = ((size_t)SLOT_BASE_W + (64 / VM_SIGNG0_W) * (size_t)SIGNG_STRIDE_W) * 4;
static_assert(LDS_SIGNG <= 80 * 1024, "signg LDS (raised limit, ovh_create)");
static constexpr size_t LDS_PKGEN = ((size_t)SLOT_BASE_W + (64 / VM_PKGEN_W) * (size_t)PKGEN_STRIDE_W) * 4;
static constexpr size_t LDS_PKCHK = ((size_t)SLOT_BASE_W + (64 / VM_PKCHK_W) * (size_t)PKCHK_STRIDE_W) * 4;
static constexpr uint32_t G1PADD_STRIDE_W = align128w(VM_G1PADD_NSLOTS * 12);
static constexpr size_t LDS_G1PADD = ((size_t)SLOT_BASE_W + (64 / VM_G1PADD_W) * (size_t)G1PADD_STRIDE_W) * 4;
static_assert(LDS_RS <= 64 * 1024 && LDS_MSM8 <= 64 * 1024 && LDS_HDBL <= 64 * 1024 && LDS_SIGCHK <= 64 * 1024 &&
                  LDS_PKCHK <= 64 * 1024 && LDS_G1PADD <= 64 * 1024 && LDS_PKGEN <= 64 * 1024 &&
                  LDS_VOTE1 <= 64 * 1024 && LDS_FINAL1 <= 64 * 1024 && LDS_VOTEW <= 64 * 1024 && LDS_QCPRE <= 64 * 1024 && LDS_VOTE1H <= 64 * 1024 &&
                  LDS_QCMIL <= 64 * 1024 && VM_G1PADD_NIN == 6,
              "default LDS limit");
static_assert(LDS_VOTE <= 160 * 1024 && LDS_VOTE_T <= 160 * 1024 && LDS_FINAL <= 160 * 1024, "VM LDS budget");
static constexpr size_t LDS_VSAME = ((size_t)SLOT_BASE_W + VM_SLICES * (size_t)VSAME_STRIDE_W) * 4;
static constexpr size_t LDS_VSAME8 = ((size_t)SLOT_BASE_W + 8 * (size_t)VSAME8_STRIDE_W) * 4;
static_assert(LDS_VSAME8 <= 64 * 1024, "vsame8 LDS (default limit)");
static constexpr size_t LDS_H2G = ((size_t)SLOT_BASE_W + VM_SLICES * (size_t)H2G_STRIDE_W) * 4;
static constexpr size_t LDS_GMIL = ((size_t)SLOT_BASE_W + (size_t)VM_GMIL_NSLOTS * 12) * 4;
static_assert(LDS_VSAME <= 64 * 1024 && LDS_H2G <= 64 * 1024 && LDS_GMIL + 16 <= 64 * 1024, "same-message LDS");
static constexpr size_t LDS_PKDEC = ((size_t)SLOT_BASE_W + (64 / VM_PKDEC_W) * (size_t)PKDEC_STRIDE_W) * 4;
static_assert(LDS_PKDEC <= 64 * 1024 && VM_PKDEC_NIN == 2, "pkdec LDS / shape");
static constexpr size_t LDS_G1GRP = ((size_t)SLOT_BASE_W + (size_t)G1GRP_STRIDE_W) * 4;
static_assert(LDS_G1GRP <= 64 * 1024 && VM_G1GRP_NIN == 3, "g1grp LDS / shape");
static constexpr size_t LDS_GFIN = ((size_t)SLOT_BASE_W + (size_t)VM_GFIN_NSLOTS * 12) * 4;
static_assert(LDS_GFIN + 16 <= 64 * 1024, "gfin LDS");
// a CU holds its four vote workgroups beside the two finals that may be in flight (1 KiB
// allocation granules assumed)
constexpr size_t lds_granule(size_t b) { return (b + 1023) / 1024 * 1024; }
// the vote pool: eight workgroups per CU (constants + four slices of the larger slot file)
static constexpr size_t LDS_POOL = LDS_VOTE > LDS_VOTE_T ? LDS_VOTE : LDS_VOTE_T;
static_assert(8 * lds_granule(LDS_POOL) <= 160 * 1024, "eight pool workgroups per CU");
static_assert(VOTE_NSCR <= 4096 && VM_VOTE_NSLOTS <= 2048 && VM_VOTE_T_NSLOTS <= 2048,
              "side words: 12-bit scratch entries, 11-bit slots (fpvm.hpp side_spill)");
// pool workgroups left out per eight CUs (their places hold the final streams' kernels and
// hash_to_field beside the pool), and the largest pool grid (the scratch is sized by it)
// r05m (bench, 20 batches): 2 holes per 8 CUs 198k verifs/s, 4 373k, 8 (one place per CU)
// 1,325k -- with fewer, the side kernels wait, the next batch's publication with them, and the
// pool idles
#ifndef POOL_HOLES_PER_8CU
#define POOL_HOLES_PER_8CU 8u
#endif
// (r05s: CU-masked pool streams -- the pool on 8 places of 240 or 224 CUs, the rest for the side
// kernels -- ran 1.02M / 0.96M verifs/s against 1.42M; removed)
#define POOL_MAX_WGS 4096u
static_assert(FOLD_STRIDE_W <= VM_SLICES * VOTE_STRIDE_W && FOLD_STRIDE_W <= VM_SLICES * VOTE_T_STRIDE_W,
              "fused fold reuses the vote slots");

static int vm_upload(ovh_ctx* c, VmDev& d, const uint32_t* code, uint32_t nphases, uint32_t W, uint32_t NW,
                     const uint16_t* in, uint32_t nin, const uint16_t* out, uint32_t nout,
                     const uint32_t* side = nullptr) {
  // + PREFETCH trailing NOP phases (instruction prefetch)
  const size_t words = (size_t)nphases * W * NW, pad = (size_t)vm::PREFETCH * W * NW;
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
  d.clk = nullptr;
  d.side = nullptr;
  if (side) {  // nphases x W side words + PREFETCH phases of zeros
    void* ds = nullptr;
    HIPCHK(hipMalloc(&ds, ((size_t)nphases + vm::PREFETCH) * W * 4));
    c->vm_bufs.push_back(ds);
    HIPCHK(hipMemcpy(ds, side, (size_t)nphases * W * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemset((uint32_t*)ds + (size_t)nphases * W, 0, (size_t)vm::PREFETCH * W * 4));
    d.side = (const uint32_t*)ds;
  }
  if ((c->flags & OVH_FLAG_VM_CLOCK) && (code == VM_VOTE_CODE || code == VM_VOTE_T_CODE)) {
    void* dk = nullptr;
    HIPCHK(hipMalloc(&dk, (size_t)2 * VM_CLOCK_WGS * 8));
    c->vm_bufs.push_back(dk);
    HIPCHK(hipMemset(dk, 0, (size_t)2 * VM_CLOCK_WGS * 8));
    d.clk = (uint64_t*)dk;
  }
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
  CHK(vm_upload(c, c->vm_vote, VM_VOTE_CODE, VM_VOTE_NPHASES, VM_VOTE_W, VM_VOTE_NW, VM_VOTE_IN, VM_VOTE_NIN, VM_VOTE_OUT,
                VM_VOTE_NOUT,
#if VM_VOTE_NSCR > 0
                VM_VOTE_SIDE
#else
                nullptr
#endif
                ));
  CHK(vm_upload(c, c->vm_vote_t, VM_VOTE_T_CODE, VM_VOTE_T_NPHASES, VM_VOTE_T_W, VM_VOTE_T_NW, VM_VOTE_T_IN, VM_VOTE_T_NIN,
                VM_VOTE_T_OUT, VM_VOTE_T_NOUT,
#if VM_VOTE_T_NSCR > 0
                VM_VOTE_T_SIDE
#else
                nullptr
#endif
                ));
  CHK(vm_upload(c, c->vm_fold, VM_FOLD_CODE, VM_FOLD_NPHASES, VM_FOLD_W, VM_FOLD_NW, VM_FOLD_IN, VM_FOLD_NIN, VM_FOLD_OUT,
                VM_FOLD_NOUT));
  CHK(vm_upload(c, c->vm_final, VM_FINAL_CODE, VM_FINAL_NPHASES, VM_FINAL_W, VM_FINAL_NW, VM_FINAL_IN, VM_FINAL_NIN, VM_FINAL_OUT,
                VM_FINAL_NOUT));
  CHK(vm_upload(c, c->vm_rs, VM_RS_CODE, VM_RS_NPHASES, VM_RS_W, VM_RS_NW, VM_RS_IN, VM_RS_NIN, VM_RS_OUT, 0));
  CHK(vm_upload(c, c->vm_sigchk, VM_SIGCHK_CODE, VM_SIGCHK_NPHASES, VM_SIGCHK_W, VM_SIGCHK_NW, VM_SIGCHK_IN,
                VM_SIGCHK_NIN, VM_SIGCHK_OUT, VM_SIGCHK_NOUT));
  CHK(vm_upload(c, c->vm_pkchk, VM_PKCHK_CODE, VM_PKCHK_NPHASES, VM_PKCHK_W, VM_PKCHK_NW, VM_PKCHK_IN, VM_PKCHK_NIN,
                VM_PKCHK_OUT, VM_PKCHK_NOUT));
  CHK(vm_upload(c, c->vm_vote1, VM_VOTE1_CODE, VM_VOTE1_NPHASES, VM_VOTE1_W, VM_VOTE1_NW, VM_VOTE1_IN, VM_VOTE1_NIN,
                VM_VOTE1_OUT, VM_VOTE1_NOUT));
  CHK(vm_upload(c, c->vm_vote_t1, VM_VOTE_T1_CODE, VM_VOTE_T1_NPHASES, VM_VOTE_T1_W, VM_VOTE_T1_NW, VM_VOTE_T1_IN,
                VM_VOTE_T1_NIN, VM_VOTE_T1_OUT, VM_VOTE_T1_NOUT));
  CHK(vm_upload(c, c->vm_signg0, VM_SIGNG0_CODE, VM_SIGNG0_NPHASES, VM_SIGNG0_W, VM_SIGNG0_NW, VM_SIGNG0_IN,
                VM_SIGNG0_NIN, VM_SIGNG0_OUT, VM_SIGNG0_NOUT));
  CHK(vm_upload(c, c->vm_signg1, VM_SIGNG1_CODE, VM_SIGNG1_NPHASES, VM_SIGNG1_W, VM_SIGNG1_NW, VM_SIGNG1_IN,
                VM_SIGNG1_NIN, VM_SIGNG1_OUT, VM_SIGNG1_NOUT));
  CHK(vm_upload(c, c->vm_pkgen, VM_PKGEN_CODE, VM_PKGEN_NPHASES, VM_PKGEN_W, VM_PKGEN_NW, VM_PKGEN_IN, VM_PKGEN_NIN,
                VM_PKGEN_OUT, VM_PKGEN_NOUT));
  CHK(vm_upload(c, c->vm_vote1h, VM_VOTE1H_CODE, VM_VOTE1H_NPHASES, VM_VOTE1H_W, VM_VOTE1H_NW, VM_VOTE1H_IN,
                VM_VOTE1H_NIN, VM_VOTE1H_OUT, VM_VOTE1H_NOUT));
  CHK(vm_upload(c, c->vm_vote_t1h, VM_VOTE_T1H_CODE, VM_VOTE_T1H_NPHASES, VM_VOTE_T1H_W, VM_VOTE_T1H_NW, VM_VOTE_T1H_IN,
                VM_VOTE_T1H_NIN, VM_VOTE_T1H_OUT, VM_VOTE_T1H_NOUT));
  CHK(vm_upload(c, c->vm_qcpre, VM_QCPRE_CODE, VM_QCPRE_NPHASES, VM_QCPRE_W, VM_QCPRE_NW, VM_QCPRE_IN, VM_QCPRE_NIN,
                VM_QCPRE_OUT, VM_QCPRE_NOUT));
  CHK(vm_upload(c, c->vm_qcmil, VM_QCMIL_CODE, VM_QCMIL_NPHASES, VM_QCMIL_W, VM_QCMIL_NW, VM_QCMIL_IN, VM_QCMIL_NIN,
                VM_QCMIL_OUT, VM_QCMIL_NOUT));
  CHK(vm_upload(c, c->vm_votew, VM_VOTEW_CODE, VM_VOTEW_NPHASES, VM_VOTEW_W, VM_VOTEW_NW, VM_VOTEW_IN, VM_VOTEW_NIN,
                VM_VOTEW_OUT, VM_VOTEW_NOUT));
  CHK(vm_upload(c, c->vm_votew_t, VM_VOTEW_T_CODE, VM_VOTEW_T_NPHASES, VM_VOTEW_T_W, VM_VOTEW_T_NW, VM_VOTEW_T_IN,
                VM_VOTEW_T_NIN, VM_VOTEW_T_OUT, VM_VOTEW_T_NOUT));
  CHK(vm_upload(c, c->vm_final1, VM_FINAL1_CODE, VM_FINAL1_NPHASES, VM_FINAL1_W, VM_FINAL1_NW, VM_FINAL1_IN,
                VM_FINAL1_NIN, VM_FINAL1_OUT, VM_FINAL1_NOUT));
  CHK(vm_upload(c, c->vm_vsame, VM_VSAME_CODE, VM_VSAME_NPHASES, VM_VSAME_W, VM_VSAME_NW, VM_VSAME_IN, VM_VSAME_NIN,
                VM_VSAME_OUT, VM_VSAME_NOUT));
  CHK(vm_upload(c, c->vm_vsame_t, VM_VSAME_T_CODE, VM_VSAME_T_NPHASES, VM_VSAME_T_W, VM_VSAME_T_NW, VM_VSAME_T_IN,
                VM_VSAME_T_NIN, VM_VSAME_T_OUT, VM_VSAME_T_NOUT));
  CHK(vm_upload(c, c->vm_vsame8, VM_VSAME8_CODE, VM_VSAME8_NPHASES, VM_VSAME8_W, VM_VSAME8_NW, VM_VSAME8_IN,
                VM_VSAME8_NIN, VM_VSAME8_OUT, VM_VSAME8_NOUT));
  CHK(vm_upload(c, c->vm_vsame8_t, VM_VSAME8_T_CODE, VM_VSAME8_T_NPHASES, VM_VSAME8_T_W, VM_VSAME8_T_NW, VM_VSAME8_T_IN,
                VM_VSAME8_T_NIN, VM_VSAME8_T_OUT, VM_VSAME8_T_NOUT));
  CHK(vm_upload(c, c->vm_h2g, VM_H2G_CODE, VM_H2G_NPHASES, VM_H2G_W, VM_H2G_NW, VM_H2G_IN, VM_H2G_NIN, VM_H2G_OUT,
                VM_H2G_NOUT));
  CHK(vm_upload(c, c->vm_gfin, VM_GFIN_CODE, VM_GFIN_NPHASES, VM_GFIN_W, VM_GFIN_NW, VM_GFIN_IN, VM_GFIN_NIN, VM_GFIN_OUT,
                VM_GFIN_NOUT));
  CHK(vm_upload(c, c->vm_g1grp, VM_G1GRP_CODE, VM_G1GRP_NPHASES, VM_G1GRP_W, VM_G1GRP_NW, VM_G1GRP_IN, VM_G1GRP_NIN,
                VM_G1GRP_OUT, VM_G1GRP_NOUT));
  CHK(vm_upload(c, c->vm_pkdec, VM_PKDEC_CODE, VM_PKDEC_NPHASES, VM_PKDEC_W, VM_PKDEC_NW, VM_PKDEC_IN, VM_PKDEC_NIN,
                VM_PKDEC_OUT, VM_PKDEC_NOUT));
  CHK(vm_upload(c, c->vm_gmil, VM_GMIL_CODE, VM_GMIL_NPHASES, VM_GMIL_W, VM_GMIL_NW, VM_GMIL_IN, VM_GMIL_NIN, nullptr, 0));
  CHK(vm_upload(c, c->vm_g1padd, VM_G1PADD_CODE, VM_G1PADD_NPHASES, VM_G1PADD_W, VM_G1PADD_NW, VM_G1PADD_IN,
                VM_G1PADD_NIN, VM_G1PADD_OUT, VM_G1PADD_NOUT));
  CHK(vm_upload(c, c->vm_madd, VM_MADD_CODE, VM_MADD_NPHASES, VM_MADD_W, VM_MADD_NW, VM_MADD_IN, VM_MADD_NIN, VM_MADD_OUT,
                VM_MADD_NOUT));
  CHK(vm_upload(c, c->vm_padd, VM_PADD_CODE, VM_PADD_NPHASES, VM_PADD_W, VM_PADD_NW, VM_PADD_IN, VM_PADD_NIN, VM_PADD_OUT,
                VM_PADD_NOUT));
#define UPLOAD_HDBL(k, M)                                                                                               \
  CHK(vm_upload(c, c->vm_hdbl[k], VM_HDBL##M##_CODE, VM_HDBL##M##_NPHASES, VM_HDBL##M##_W, VM_HDBL##M##_NW, VM_HDBL##M##_IN, \
                VM_HDBL##M##_NIN, VM_HDBL##M##_OUT, VM_HDBL##M##_NOUT))
  UPLOAD_HDBL(0, 1);
  UPLOAD_HDBL(1, 2);
  UPLOAD_HDBL(2, 4);
  UPLOAD_HDBL(3, 8);
  UPLOAD_HDBL(4, 16);
#undef UPLOAD_HDBL
  HIPCHK(hipFuncSetAttribute((const void*)k_vm_pool, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_POOL));
  HIPCHK(hipFuncSetAttribute((const void*)k_vm_signg, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_SIGNG));
  HIPCHK(hipFuncSetAttribute((const void*)k_vm_fold<VM_FOLD_UNITS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)LDS_FOLD));
  HIPCHK(hipFuncSetAttribute((const void*)k_vm_fold<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_FOLD1));
  for (const void* k : {(const void*)k_vm_final, (const void*)k_vm_group, (const void*)k_vm_votechk})
    HIPCHK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_FINAL));
  return 0;
}

// Stage bracket: events on a stream around the stage's kernels.
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

// ---- buffers
static Slab region_F(ovh_ctx* c, int slot, int r) {
  return Slab{c->red_slot[slot] + (size_t)r * PART_PLANES * 12 * c->red_cap, c->red_cap};
}
static Slab region_S(ovh_ctx* c, int slot, int r) {
  return Slab{c->red_slot[slot] + (size_t)r * PART_PLANES * 12 * c->red_cap + (size_t)12 * 12 * c->red_cap,
              c->red_cap};
}

// ---- streams
// A context's streams are never destroyed: ovh_destroy synchronises them and parks them here,
// per device and priority, and the next context created on that device takes them back. A
// caller may have recorded events of its own on a context's stream (torch's pinned-host
// allocator does so for every non-blocking copy from pinned memory issued on
// torch.cuda.ExternalStream(ctx.stream)) and query them after ovh_destroy; an event recorded on
// a destroyed stream dereferences the freed queue when it is queried (the r05ab segfault, in the
// test's teardown, after Context.close(): VERDICT r05). Parked streams keep every such event
// valid for the life of the process; the number of streams is bounded by the most contexts ever
// alive at once. include/ovhip.h states the contract.
namespace {
struct ParkedStream {
  int device;
  int prio;
  hipStream_t s;
};
std::mutex g_park_mu;
std::vector<ParkedStream> g_parked;
}  // namespace

// A non-blocking stream of priority `prio` on the current device (a parked one if any).
static hipError_t stream_new(hipStream_t* s, int prio) {
  int dev = 0;
  const hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  {
    std::lock_guard<std::mutex> g(g_park_mu);
    for (size_t k = 0; k < g_parked.size(); ++k)
      if (g_parked[k].device == dev && g_parked[k].prio == prio) {
        *s = g_parked[k].s;
        g_parked.erase(g_parked.begin() + (ptrdiff_t)k);
        return hipSuccess;
      }
  }
  return hipStreamCreateWithPriority(s, hipStreamNonBlocking, prio);
}

// Park stream s of `device` (its work drained first).
static void stream_park(int device, hipStream_t s) {
  if (!s) return;
  (void)hipStreamSynchronize(s);
  int prio = 0;
  if (hipStreamGetPriority(s, &prio) != hipSuccess) return;  // (never destroyed either way)
  std::lock_guard<std::mutex> g(g_park_mu);
  g_parked.push_back(ParkedStream{device, prio, s});
}

// OVH_ERR_DEVICE once a final stream gave up waiting for the vote pool (k_pool_wait: that batch's
// partial, verdict and codes are not trustworthy). The flag is sticky: the pool queue may still
// hold the batch, so the context stays failed until ovh_destroy (include/ovhip.h). Every
// synchronous return that hands out results derived from a pool batch checks it after its
// synchronisation.
static int pool_failed(const ovh_ctx* c) {
  return c->pool_err && __atomic_load_n(c->pool_err, __ATOMIC_ACQUIRE) ? OVH_ERR_DEVICE : 0;
}

// Every stream of the context idle, then the pool check above.
static int sync_all(ovh_ctx* c) {
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipStreamSynchronize(c->fstream));
  HIPCHK(hipStreamSynchronize(c->fstream2));
  HIPCHK(hipStreamSynchronize(c->fstream3));
  if (c->fstream4) HIPCHK(hipStreamSynchronize(c->fstream4));
  for (hipStream_t s : {c->pool_st[0], c->pool_st[1], c->pool_st[2], c->vstream[0], c->vstream[1], c->vstream[2],
                        c->hstream[1], c->hstream[2], c->hstream[3]})
    if (s) HIPCHK(hipStreamSynchronize(s));
  return pool_failed(c);
}

// MSM scratch of a slot (msm.hpp MsmArgs), in words: cnt, off, cur, level prefixes, entries
// (2 points x 4 windows per vote), bucket trees (level-0 outputs: <= 4 cap + NB), U planes.
static size_t msm_acap(uint32_t cap) { return (size_t)4 * cap + MSM_NB; }
static size_t msm_round(size_t w) { return (w + 63) / 64 * 64; }
static size_t msm_words(uint32_t cap) {
  return msm_round(MSM_NB) + msm_round(MSM_NB + 1) + msm_round(MSM_NB) + msm_round((size_t)MSM_LV * (MSM_NB + 1)) +
         msm_round((size_t)8 * cap) + msm_round((size_t)6 * 12 * msm_acap(cap)) + (size_t)6 * 12 * MSM_U;
}
static MsmArgs msm_args(ovh_ctx* c, int slot, uint32_t** cur) {
  uint32_t* p = c->msm_buf[slot];
  MsmArgs a;
  a.cnt = p;
  p += msm_round(MSM_NB);
  a.off = p;
  p += msm_round(MSM_NB + 1);
  *cur = p;
  p += msm_round(MSM_NB);
  a.pf = p;
  p += msm_round((size_t)MSM_LV * (MSM_NB + 1));
  a.ent = p;
  p += msm_round((size_t)8 * c->cap);
  a.A = Slab{p, (uint32_t)msm_acap(c->cap)};
  p += msm_round((size_t)6 * 12 * msm_acap(c->cap));
  a.U = Slab{p, MSM_U};
  a.st = Slab{c->state_slot[slot], c->cap};
  return a;
}
static Slab msm_S(ovh_ctx* c, int slot) {
  uint32_t* cur;
  return msm_args(c, slot, &cur).U;  // element 0: sum r_i sigma_i
}

// Batch state for n votes: per slot S_TOTAL planes, fold regions R0..R3 (cap/4 partials each),
// the group verdicts and the MSM scratch. A reallocation waits for all work and forgets the
// last batch.
static int ensure_cap(ovh_ctx* c, size_t n) {
  if (n > (1u << 24)) return OVH_ERR_ARG;
  if (n <= c->cap && c->state_slot[0]) return 0;
  uint32_t cap = 256;
  while (cap < n) cap <<= 1;
  CHK(sync_all(c));
  for (int k = 0; k < OVH_BATCH_SLOTS; ++k) {
    for (void* p : {(void*)c->grp_ok[k], (void*)c->msm_buf[k]})
      if (p) (void)hipFree(p);
    c->state_slot[k] = c->red_slot[k] = c->msm_buf[k] = nullptr;
    c->pstage[k] = nullptr;
    c->grp_ok[k] = nullptr;
    c->slot_n[k] = 0;
  }
  for (void* p : {(void*)c->state_all, (void*)c->red_all, (void*)c->pstage_all})
    if (p) (void)hipFree(p);
  c->state_all = c->red_all = nullptr;
  c->pstage_all = nullptr;
  c->last_n = 0;
  c->cap = 0;
  c->red_cap = cap / 4 > 64 ? cap / 4 : 64;
  c->state_w = (size_t)S_TOTAL * 12 * cap;
  c->red_w = (size_t)4 * PART_PLANES * 12 * c->red_cap;
  c->pstage_b = ((size_t)cap * 148 + 255) / 256 * 256;
  HIPCHK(hipMalloc(&c->state_all, c->state_w * 4 * OVH_BATCH_SLOTS));
  HIPCHK(hipMalloc(&c->red_all, c->red_w * 4 * OVH_BATCH_SLOTS));
  HIPCHK(hipMalloc(&c->pstage_all, c->pstage_b * OVH_BATCH_SLOTS));
  for (int k = 0; k < OVH_BATCH_SLOTS; ++k) {
    c->state_slot[k] = c->state_all + k * c->state_w;
    c->red_slot[k] = c->red_all + k * c->red_w;
    c->pstage[k] = c->pstage_all + k * c->pstage_b;
    HIPCHK(hipMalloc(&c->grp_ok[k], ((size_t)cap / GROUP_VOTES + 1) * 4));
    HIPCHK(hipMalloc(&c->msm_buf[k], msm_words(cap) * 4));
  }
  c->cap = cap;
  return 0;
}

// Single-call scratch (aggregation / key sums): 9 planes + two code arrays of n entries.
static int ensure_scr(ovh_ctx* c, size_t n) {
  if (n > (1u << 24)) return OVH_ERR_ARG;
  if (n <= c->scr_cap && c->scr) return 0;
  uint32_t cap = 256;
  while (cap < n) cap <<= 1;
  HIPCHK(hipStreamSynchronize(c->stream));
  for (void* p : {(void*)c->scr, (void*)c->scr_pk, (void*)c->scr_sig})
    if (p) (void)hipFree(p);
  c->scr = nullptr;
  c->scr_pk = c->scr_sig = nullptr;
  c->scr_cap = 0;
  HIPCHK(hipMalloc(&c->scr, (size_t)9 * 12 * cap * 4));
  HIPCHK(hipMalloc(&c->scr_pk, (size_t)cap * 4));
  HIPCHK(hipMalloc(&c->scr_sig, (size_t)cap * 4));
  c->scr_cap = cap;
  return 0;
}

static int ensure_in(ovh_ctx* c, size_t bytes) {
  if (bytes <= c->in_cap && c->in_buf) return 0;
  size_t cap = 4096;
  while (cap < bytes) cap <<= 1;
  HIPCHK(hipStreamSynchronize(c->stream));
  if (c->in_buf) (void)hipFree(c->in_buf);
  c->in_buf = nullptr;
  c->in_cap = 0;
  HIPCHK(hipMalloc(&c->in_buf, cap));
  c->in_cap = cap;
  return 0;
}

// Batch state slot k for the next batch on the main stream: the stream first waits until the
// final stream has finished with the slot's previous batch (its bisection reads that state).
// final streams: a batch's fold levels, MSM, final and bisection take 4-6 ms beside the pool
// (r05y pool log), so two in turn held the pipeline to one batch per ~3 ms; three: 1,378k-1,386k
// verifs/s vs 1,254k-1,260k (r05z). Four (the low-priority hardware queues' count): the pool path
// unchanged (1,600-1,608k vs 1,607-1,608k), pipelined same-message batches 1.58-1.62 ms per
// batch against 1.82-1.84 (r06o)
static int take_slot(ovh_ctx* c, int* slot) {
  const int k = (int)(c->pipe_k % OVH_BATCH_SLOTS);
  HIPCHK(hipStreamWaitEvent(c->stream, c->ev_back[k], 0));
  const uint64_t f = c->pipe_k % c->nfin;
  c->fs[k] = f == 0 ? c->fstream : f == 1 ? c->fstream2 : f == 2 ? c->fstream3 : c->fstream4;
  ++c->pipe_k;
  c->last_slot = k;
  *slot = k;
  return 0;
}

// take_slot for a batch the pool will run (batch_front): its announcement first, on ovh_stream
// ahead of the slot wait. Idle pool workgroups stay while nann > npub (pool_claim); announced
// behind the slot wait -- or on a stream of its own, whose hardware queue the runtime may share
// with ovh_stream -- the next batch's announcement waited for a final stream, the spare
// workgroups left, and the rest of the run had 1,024 of the pool's 1,792 (r05v pool log; the
// slow mode of r05q-r05u, 3.9-4.0 ms per batch)
static int pool_take_slot(ovh_ctx* c, int* slot) {
  k_pool_announce<<<1, 64, 0, c->stream>>>(c->pool_q, c->pool_seq + 1);
  return take_slot(c, slot);
}

// RLC coefficients of the next batch: SplitMix64(seed, base + i) with a fresh secret seed from
// the OS (the coefficients must be unknown to whoever produced the signatures).
static int draw_seed(ovh_ctx* c, uint64_t* seed, uint64_t* base) {
  if (c->flags & OVH_FLAG_TEST_RLC) {
    *seed = c->test_seed;
    *base = c->test_base;
    return 0;
  }
  uint8_t b[8];
  size_t got = 0;
  while (got < sizeof b) {
    const ssize_t r = getrandom(b + got, sizeof b - got, 0);
    if (r < 0) {
      if (errno == EINTR) continue;
      return OVH_ERR_RNG;
    }
    got += (size_t)r;
  }
  memcpy(seed, b, 8);
  *base = 0;
  return 0;
}

// Key source of a batch: compressed bytes (vote program) or points (vote_t program).
struct KeySrc {
  const uint8_t* bytes;  // n x 48, or null
  PkSrc pts;
};

static uint32_t groups_of(uint32_t n) { return (n + GROUP_VOTES - 1) / GROUP_VOTES; }

// Per-vote stages of a batch in `slot` (n >= 1 votes): on ovh_stream the staging of its
// signatures and keys into the slot (k_pool_stage: the caller's buffers are then free in
// ovh_stream order) and hash_to_field, then its publication to the vote pool and, on the pool
// stream, a pool grid ("Vote pool"): the pool writes the codes, the state
// planes and the fold level-0 partials (R0) and counts the batch's quads done. ev_front[slot] is
// recorded after the publication (pool_join's stream waits for it). alone: the batch's combined
// check covers only this batch (not a shard of a larger combined check).
static int batch_front(ovh_ctx* c, int slot, uint32_t n, const uint8_t* d_sigs, const uint8_t* d_hashes, KeySrc key,
                       int32_t* d_codes, bool alone = false, bool launch = true, bool shard = false) {
  Slab s{c->state_slot[slot], c->cap};
  c->ev_mask = 0;
  uint64_t seed, base;
  CHK(draw_seed(c, &seed, &base));
  // one vote checked on its own (alone: never combined with other partials): its pairing
  // equation needs no random coefficient, scalar 1 (vote_scalar). A one-vote shard keeps its
  // random scalar: its partial is combined with the other shards'.
  if (n == 1 && alone) base = UNIT_BASE;
  c->slot_seed[slot] = seed;
  c->slot_base[slot] = base;
  uint8_t* ps = c->pstage[slot];
  const bool table = key.bytes == nullptr;
  const uint64_t seq = c->pool_seq++;
  {
    StageScope p(c, ST_H2F, c->stream);
    const uint32_t bytes = n * (table ? 96u : 144u) + (table && key.pts.idx ? n * 4u : 0u);
    k_pool_stage<<<std::min(1024u, (bytes + 16 * WG - 1) / (16 * WG)), WG, 0, c->stream>>>(
        n, d_sigs, key.bytes, table ? key.pts.idx : nullptr, ps);
    k_h2f<<<nblk(n), WG, 0, c->stream>>>(n, d_hashes, c->xmd, s);
  }
  PoolBatch b{};
  b.n = n;
  b.nq = (n + VM_SLICES - 1) / VM_SLICES;
  b.table = table;
  b.has_idx = table && key.pts.idx;
  b.seed = seed;
  b.base = base;
  b.codes = d_codes;
  b.planes = key.pts.planes;
  b.flags = key.pts.flags;
  b.pcap = key.pts.cap;
  b.state = s.p;
  b.cap = s.cap;
  const Slab r0 = region_F(c, slot, 0);
  b.part0 = r0.p;
  b.part_cap = r0.cap;
  b.stage = ps;
  b.clk = table ? c->vm_vote_t.clk : c->vm_vote.clk;
  b.plog = c->plog ? c->plog + (size_t)(seq % PLOG_RING) * PLOG_WORDS : nullptr;
  c->plog_seq[slot] = seq;
  k_pool_publish<<<1, 64, 0, c->stream>>>(b, (uint32_t)slot, seq, c->pool_q, (PoolBatch*)c->pool_desc);
  if (b.plog) k_stamp<<<1, 64, 0, c->stream>>>(b.plog + PLOG_EV_PUB, seq);
  HIPCHK(hipEventRecord(c->ev_front[slot], c->stream));
  c->slot_n[slot] = n;
  c->last_n = n;
  // the batch's pool grids: one on each pool stream, each with half of the pool's places. A grid
  // queued behind a running one on its stream starts only once that one's last workgroup has
  // exited, so with one stream the workgroups that left during a gap in the queue were not
  // replaced while the rest kept the grid alive (r05k); with a grid per stream per batch the pool
  // refills from the next batch's grids, and a batch alone still gets every place
  const bool vev = (c->flags & OVH_FLAG_PROFILE) != 0;
  const uint32_t vk = c->vev_n % ovh_ctx::VEV_CAP;
  const uint32_t wgs = c->pool_wgs;
  PoolArgs pa;
  pa.only = ~0ull;
  pa.nsimd = 4 * c->pool_ncu;
  pa.skip_cu = c->pool_rsv / 8;
  // a grid per shard batch unless the pool leaves CUs to the collective (OVH_FLAG_POOL_RESERVE):
  // then shard batches share the persistent pool like the others
  shard = shard && !c->pool_rsv;
  pa.q = c->pool_q;
  pa.descs = (const PoolBatch*)c->pool_desc;
  pa.pv_code = c->vm_vote.code;
  pa.pv_side = c->vm_vote.side;
  pa.pt_code = c->vm_vote_t.code;
  pa.pt_side = c->vm_vote_t.side;
  pa.fold_code = c->vm_fold.code;
  pa.cst = c->vm_consts;
  for (uint32_t par = 0; launch && par < (shard ? c->shard_streams : 2u); ++par) {
    // the shard path without reserved CUs: one grid of this batch alone per batch, on the pool
    // streams in turn (its workgroups leave when the batch is claimed, so the caller's collective
    // finds places between batches -- with persistent grids and the pool on every CU it waited for
    // the pool to drain, r05an / r05aq pool logs)
    if (shard && par != (uint32_t)(seq % c->shard_streams)) continue;
    if (shard) pa.only = seq + c->shard_span;
    hipStream_t pst = c->pool_st[par];
    HIPCHK(hipStreamWaitEvent(pst, c->ev_front[slot], 0));
    if (par == 0 || shard) {  // the vote stage's and the vote spans' start (stream 0), end (stream 1)
      if (c->flags & OVH_FLAG_PROFILE) HIPCHK(hipEventRecord(c->ev0[ST_VOTE], pst));
      if (vev) HIPCHK(hipEventRecord(c->vev0[vk], pst));
    }
    // each workgroup's own scratch: one fixed region of 2 x wgs workgroups per pool stream, for
    // every grid shape (a normal grid or a shard grid of the whole pool). Grids of one stream run
    // one after the other; grids of the two streams may be co-resident -- including a normal grid
    // and a shard grid when a caller mixes the APIs without ovh_batch_wait -- and
    // never share a workgroup's spill area
    const uint32_t gw = shard ? 2 * wgs : par == 0 ? c->pool_grid0 : 2 * wgs - c->pool_grid0;
    pa.scr = c->pool_scr + (size_t)par * 2 * wgs * VM_SLICES * VOTE_NSCR * 12;
    pa.wlog = nullptr;
    if (c->plog) {  // grid record: [seq, par, workgroups, -], then the workgroups'
      uint64_t* g = c->plog + PLOG_GRID_BASE + (size_t)(c->plog_grids++ % PLOG_GRIDS) * (4 + PLOG_WGS * PLOG_WG_WORDS);
      k_grid_hdr<<<1, 64, 0, pst>>>(g, seq, par, gw);
      pa.wlog = g + 4;
    }
    k_vm_pool<<<gw, 64, LDS_POOL, pst>>>(pa);
    if (par == 1 || shard) {
      if (c->flags & OVH_FLAG_PROFILE) {
        HIPCHK(hipEventRecord(c->ev1[ST_VOTE], pst));
        c->ev_mask |= 1u << ST_VOTE;
      }
      if (vev) {
        HIPCHK(hipEventRecord(c->vev1[vk], pst));
        ++c->vev_n;
      }
    }
  }
  c->clk_table = table;
  c->clk_wgs = c->pool_wgs < VM_CLOCK_WGS ? c->pool_wgs : VM_CLOCK_WGS;
  HIPCHK(hipGetLastError());
  return 0;
}

// Timeout of a final stream's wait for the pool (k_pool_wait): far above any real batch -- the
// pool may still be working through the OVH_BATCH_SLOTS - 1 batches published before this one.
static uint64_t pool_wait_ticks(uint32_t n) { return 100000000ull * 4 + (uint64_t)n * 100 * OVH_BATCH_SLOTS; }

// On stream st (after ev_front[slot]): wait for the pool to finish the batch in `slot`, then fold
// level 1 (R0 -> R1: one partial per 16-vote group). *reg = 1, *m = the groups.
// OVH_FLAG_VM_CLOCK: a stamp of event ev of the batch in `slot` on stream st (the pool log)
static void plog_stamp(ovh_ctx* c, int slot, uint32_t ev, hipStream_t st) {
  if (c->plog)
    k_stamp<<<1, 64, 0, st>>>(c->plog + (size_t)(c->plog_seq[slot] % PLOG_RING) * PLOG_WORDS + ev, ~0ull);
}

static int pool_join(ovh_ctx* c, int slot, hipStream_t st, int* reg, uint32_t* m) {
  const uint32_t n = c->slot_n[slot], nq = (n + VM_SLICES - 1) / VM_SLICES;
  k_pool_wait<<<1, 64, 0, st>>>(c->pool_q, (uint32_t)slot, nq, pool_wait_ticks(n), c->pool_err);
  plog_stamp(c, slot, PLOG_EV_DONE, st);
  *m = groups_of(n);
  *reg = 1;
  StageScope p(c, ST_FOLD, st);
  k_vm_fold<1><<<*m, 64, LDS_FOLD1, st>>>(nq, c->vm_fold, c->vm_consts, region_F(c, slot, 0), region_S(c, slot, 0),
                                           region_F(c, slot, 1), nullptr);
  return hipGetLastError() == hipSuccess ? 0 : OVH_ERR_DEVICE;
}


// Fold levels from region *reg (m partials) down to <= until, on stream st, alternating regions
// R2 / R3 (R1 stays intact for the bisection). slices = 4 (main stream) or 1 (the final
// stream, beside the next batch's vote workgroups).
static int fold_down(ovh_ctx* c, int slot, hipStream_t st, int slices, int* reg, uint32_t* m, uint32_t until) {
  StageScope p(c, ST_FOLD, st);
  while (*m > until) {
    const uint32_t mo = (*m + 3) / 4;
    const int ro = *reg == 2 ? 3 : 2;
    if (slices == 1)
      k_vm_fold<1><<<mo, 64, LDS_FOLD1, st>>>(*m, c->vm_fold, c->vm_consts, region_F(c, slot, *reg),
                                              region_S(c, slot, *reg), region_F(c, slot, ro), nullptr);
    else
      k_vm_fold<VM_FOLD_UNITS><<<(mo + VM_FOLD_UNITS - 1) / VM_FOLD_UNITS, 64, LDS_FOLD, st>>>(
          *m, c->vm_fold, c->vm_consts, region_F(c, slot, *reg), region_S(c, slot, *reg), region_F(c, slot, ro),
          nullptr);
    *reg = ro;
    *m = mo;
  }
  return hipGetLastError() == hipSuccess ? 0 : OVH_ERR_DEVICE;
}

// Verdict words in c->result: [0] single calls, then per slot the batch verdicts, the combine
// verdicts, then the synchronous combine's and the multi-device combine's.
enum { RES_WORDS = 32 };
enum { RES_BATCH = 4, RES_COMBINE = RES_BATCH + OVH_BATCH_SLOTS, RES_SYNC = RES_COMBINE + OVH_BATCH_SLOTS, RES_MULTI };
// RES_MULTI: the synchronous multi-device verdict; RES_MULTI + 1 + ring slot: the pipelined ones
static_assert(RES_MULTI + 1 + OVH_BATCH_SLOTS <= RES_WORDS, "verdict words fit c->result");

// Final check on <= 4 partials given as planes: k_vm_final on stream `st`, verdict to *d_res;
// xS: the batch's MSM result (partial 0's S), or {nullptr} when the partials carry their S.
static void enqueue_final(ovh_ctx* c, hipStream_t st, Slab F, Slab S, uint32_t m, int32_t* d_res,
                          Slab xS = Slab{nullptr, 0}) {
  StageScope p(c, ST_FINAL, st);
  k_vm_final<<<1, 64, LDS_FINAL, st>>>(m, c->vm_final, c->vm_consts, F, S, xS, d_res);
}

// Pippenger MSM of the batch in `slot` on stream st (msm.hpp): S = sum of r_i sigma_i over the
// votes with code 0 -> msm_S(c, slot). Needs the vote kernel's codes and sigma / tau planes.
static int enqueue_msm(ovh_ctx* c, hipStream_t st, int slot, uint32_t n, const int32_t* d_codes) {
  StageScope p(c, ST_MSM, st);
  uint32_t* cur;
  const MsmArgs a = msm_args(c, slot, &cur);
  const uint64_t seed = c->slot_seed[slot], base = c->slot_base[slot];
  if (base == UNIT_BASE) {  // a single vote with scalar 1: S = sigma
    k_sig_as_S<<<1, 64, 0, st>>>(a.st, d_codes, a.U);
    return hipGetLastError() == hipSuccess ? 0 : OVH_ERR_DEVICE;
  }
  uint32_t nlev = 1;  // tree levels: 2^nlev >= the largest possible bucket (2n points)
  while ((1ull << nlev) < 2ull * n) ++nlev;
  if (nlev > MSM_LV) return OVH_ERR_ARG;
  k_msm_zero<<<(MSM_NB + MSM_TPB - 1) / MSM_TPB, MSM_TPB, 0, st>>>((uint32_t*)a.cnt);  // (one-wave workgroups)
  const uint32_t nb = (n + MSM_TPB - 1) / MSM_TPB;
  k_msm_count<<<nb, MSM_TPB, 0, st>>>(n, seed, base, d_codes, (uint32_t*)a.cnt);
  k_msm_scan<<<1, 64, 0, st>>>(nlev, a.cnt, (uint32_t*)a.off, cur, (uint32_t*)a.pf);
  k_msm_scatter<<<nb, MSM_TPB, 0, st>>>(n, seed, base, d_codes, cur, (uint32_t*)a.ent);
  constexpr uint32_t SL8 = 64 / VM_MADD_W, SL16 = 64 / VM_HDBL1_W;
  auto grid = [](uint64_t pairs, uint32_t sl) { return (uint32_t)((pairs + sl - 1) / sl); };
  // bucket trees: level 0 pairs (<= 4n + NB), level l (<= 8n / 2^(l+1) + NB), in place
  k_msm_pair<VM_MADD_W, MSM_L0><<<grid(4ull * n + MSM_NB, SL8), 64, LDS_MSM8, st>>>(0, c->vm_madd, VM_MADD_NIN,
                                                                                     MSM8_STRIDE_W, c->vm_consts, a);
  for (uint32_t lv = 1; lv < nlev; ++lv)
    k_msm_pair<VM_PADD_W, MSM_LVL><<<grid((8ull * n >> (lv + 1)) + MSM_NB, SL8), 64, LDS_MSM8, st>>>(
        lv, c->vm_padd, VM_PADD_NIN, MSM8_STRIDE_W, c->vm_consts, a);
  // bit-plane sums T_t (128 buckets each): pairs of buckets, then 6 levels
  k_msm_pair<VM_PADD_W, MSM_T0><<<grid(MSM_U, SL8), 64, LDS_MSM8, st>>>(0, c->vm_padd, VM_PADD_NIN, MSM8_STRIDE_W,
                                                                        c->vm_consts, a);
  for (uint32_t lv = 1; lv <= 6; ++lv)
    k_msm_pair<VM_PADD_W, MSM_TL><<<grid(MSM_NT * (MSM_TM >> lv), SL8), 64, LDS_MSM8, st>>>(
        lv, c->vm_padd, VM_PADD_NIN, MSM8_STRIDE_W, c->vm_consts, a);
  // sum_t 2^t T_t: five levels of A + [2^m] B, m = 1, 2, 4, 8, 16
  for (uint32_t h = 1; h <= 5; ++h)
    k_msm_pair<VM_HDBL1_W, MSM_HRN><<<grid(MSM_NT >> h, SL16), 64, LDS_HDBL, st>>>(
        h, c->vm_hdbl[h - 1], VM_HDBL1_NIN, HDBL_STRIDE_W, c->vm_consts, a);
  return hipGetLastError() == hipSuccess ? 0 : OVH_ERR_DEVICE;
}

// Bisection of the batch in `slot` on stream `st`, skipped on the device when *d_verdict == 1
// (d_verdict null: always runs): the 16-vote groups' own checks (R1 partials), then per-vote
// checks of the votes in failing groups.
// up to one vote per SIMD (256 CUs x 4): the per-vote checks of a whole batch run side by side
#ifndef BISECT_DIRECT_MAX
#define BISECT_DIRECT_MAX 1024u
#endif
static void enqueue_bisect(ovh_ctx* c, hipStream_t st, int slot, uint32_t n, int32_t* d_codes,
                           const int32_t* d_verdict) {
  StageScope p(c, ST_FALLBACK, st);
  const uint32_t g = groups_of(n);
  // r_i sigma_i per vote, then fold levels 0 and 1 of (f, r sigma) -> R1 (16-vote groups)
  Slab s{c->state_slot[slot], c->cap};
  k_vm_rs<<<(n + 64 / VM_RS_W - 1) / (64 / VM_RS_W), 64, LDS_RS, st>>>(n, c->vm_rs, c->vm_consts, s, c->slot_seed[slot],
                                                                     c->slot_base[slot], d_codes, d_verdict);
  if (n <= BISECT_DIRECT_MAX) {
    // small batches: every vote with code 0 straight through the per-vote check (one level of
    // final-program latency instead of the group level and then the vote level)
    (void)hipMemsetAsync(c->grp_ok[slot], 0, (size_t)g * 4, st);
    k_vm_votechk<<<n, 64, LDS_FINAL, st>>>(n, c->vm_final, c->vm_consts, Slab{c->state_slot[slot], c->cap}, d_codes,
                                           d_verdict, c->grp_ok[slot]);
    return;
  }
  const uint32_t nwg = (n + 3) / 4;
  k_vm_fold<VM_FOLD_UNITS><<<(nwg + VM_FOLD_UNITS - 1) / VM_FOLD_UNITS, 64, LDS_FOLD, st>>>(
      n, c->vm_fold, c->vm_consts, Slab{s.p + (size_t)S_F * 12 * s.cap, s.cap}, Slab{s.p + (size_t)S_RS * 12 * s.cap, s.cap},
      region_F(c, slot, 0), d_codes, d_verdict);
  k_vm_fold<VM_FOLD_UNITS><<<(g + VM_FOLD_UNITS - 1) / VM_FOLD_UNITS, 64, LDS_FOLD, st>>>(
      nwg, c->vm_fold, c->vm_consts, region_F(c, slot, 0), region_S(c, slot, 0), region_F(c, slot, 1), nullptr,
      d_verdict);
  k_vm_group<<<g, 64, LDS_FINAL, st>>>(g, c->vm_final, c->vm_consts, region_F(c, slot, 1), region_S(c, slot, 1),
                                       d_verdict, c->grp_ok[slot]);
  k_vm_votechk<<<n, 64, LDS_FINAL, st>>>(n, c->vm_final, c->vm_consts, Slab{c->state_slot[slot], c->cap}, d_codes,
                                         d_verdict, c->grp_ok[slot]);
}

// The final stream of `slot` after the batch's publication: waits for the pool (pool_join), then
// the fold levels R0 -> R1 -> ... down to <= until partials (*reg, *m).
static int side_front(ovh_ctx* c, int slot, uint32_t until, int* reg, uint32_t* m) {
  hipStream_t fst = c->fs[slot];
  HIPCHK(hipStreamWaitEvent(fst, c->ev_front[slot], 0));
  CHK(pool_join(c, slot, fst, reg, m));
  return fold_down(c, slot, fst, 1, reg, m, until);
}

// One standalone vote on the main stream (k_h2f, k_vm_vote1 / k_vm_vote_t1, k_vm_final1): its
// own pairing equation, no coefficient (section 1 of DESIGN.md). Caller holds c->mu and waits.
// h_host: the hash's host bytes, for the message cache (every vote of a round signs the same
// hash): a hash seen before runs vote1h / vote_t1h on its cached H, without hash_to_G2 (vote1
// 2,061 -> 1,444 phases); a new one runs vote1 / vote_t1, whose stored H is copied into the
// cache (FIFO, HC_CAP entries). Null: no cache.
#define HC_CAP 256u
static int verify_one_locked(ovh_ctx* c, const uint8_t* d_sig, const uint8_t* d_hash, KeySrc key, int32_t* d_code,
                             const uint8_t* h_host = nullptr) {
  CHK(ensure_cap(c, 1));
  int slot;
  CHK(take_slot(c, &slot));
  c->last_n = 0;  // no partial state for ovh_batch_partial_device / fallback
  Slab s{c->state_slot[slot], c->cap};
  hipStream_t st = c->stream;
  if (h_host && !c->hc_planes) {
    HIPCHK(hipMalloc(&c->hc_planes, (size_t)6 * 12 * HC_CAP * 4));
    HIPCHK(hipMalloc(&c->hc_inf, (size_t)HC_CAP * 4));
    c->hc_keys.assign(HC_CAP, std::string());
  }
  const Slab hc{c->hc_planes, HC_CAP};
  std::string hk;
  if (h_host) {
    hk.assign((const char*)h_host, 32);
    auto it = c->hc_index.find(hk);
    if (it != c->hc_index.end()) {
      ++c->hc_hits;
      const uint32_t he = it->second;
      if (key.bytes)
        k_vm_vote1h<false><<<1, 64, LDS_VOTE1H, st>>>(c->vm_vote1h, c->vm_consts, key.bytes, PkSrc{}, d_sig, s, d_code,
                                                      hc, he, c->hc_inf);
      else
        k_vm_vote1h<true><<<1, 64, LDS_VOTE1H, st>>>(c->vm_vote_t1h, c->vm_consts, nullptr, key.pts, d_sig, s, d_code,
                                                     hc, he, c->hc_inf);
      k_vm_final1<<<1, 64, LDS_FINAL1, st>>>(c->vm_final1, c->vm_consts, Slab{s.p + (size_t)S_F * 12 * s.cap, s.cap},
                                              d_code, c->result + RES_BATCH + slot);
      HIPCHK(hipEventRecord(c->ev_back[slot], st));
      HIPCHK(hipGetLastError());
      return 0;
    }
    ++c->hc_misses;
  }
  uint32_t he = 0;
  if (h_host) {  // the entry is filled in stream order, before any later call can read it
    he = c->hc_next;
    c->hc_next = (c->hc_next + 1) % HC_CAP;
    // the old entry's planes are about to be overwritten: drop it now; the new key is entered
    // only once every launch that fills the planes was accepted (below)
    if (!c->hc_keys[he].empty()) c->hc_index.erase(c->hc_keys[he]);
    c->hc_keys[he].clear();
  }
  k_h2f<<<1, WG, 0, st>>>(1, d_hash, c->xmd, s);
  if (key.bytes)
    k_vm_vote1<false><<<1, 64, LDS_VOTE1, st>>>(c->vm_vote1, c->vm_consts, key.bytes, PkSrc{}, d_sig, s, d_code,
                                                h_host ? c->hc_inf + he : nullptr);
  else
    k_vm_vote1<true><<<1, 64, LDS_VOTE1, st>>>(c->vm_vote_t1, c->vm_consts, nullptr, key.pts, d_sig, s, d_code,
                                               h_host ? c->hc_inf + he : nullptr);
  if (h_host) k_copy_h<<<1, 64, 0, st>>>(s, hc, he);
  // a failed launch of k_h2f / vote1 / k_copy_h leaves the entry unregistered
  HIPCHK(hipGetLastError());
  if (h_host) {
    c->hc_keys[he] = hk;
    c->hc_index[hk] = he;
  }
  k_vm_final1<<<1, 64, LDS_FINAL1, st>>>(c->vm_final1, c->vm_consts, Slab{s.p + (size_t)S_F * 12 * s.cap, s.cap},
                                          d_code, c->result + RES_BATCH + slot);
  HIPCHK(hipEventRecord(c->ev_back[slot], st));
  HIPCHK(hipGetLastError());
  return 0;
}

// A small batch checked alone (2 <= n <= c->small_max): hash_to_field and
// k_vm_votew (one vote per wave: its checks, H(m), r pk, r sigma and f_i = Miller(r pk, H)
// Miller(-G1, r sigma)) on the main stream; on the slot's final stream the fold of the f_i of
// the votes with code 0 down to one partial, FE(prod f_i) == 1 (k_vm_fe) and, when that fails,
// FE(f_i) == 1 per vote (k_vm_votefe). No MSM, no Miller loop in the final: one final
// exponentiation per batch. Caller holds c->mu.
static int verify_small_locked(ovh_ctx* c, uint32_t n, const uint8_t* d_sigs, const uint8_t* d_hashes, KeySrc key,
                               int32_t* d_codes) {
  int slot;
  CHK(take_slot(c, &slot));
  Slab s{c->state_slot[slot], c->cap};
  hipStream_t st = c->stream;
  c->ev_mask = 0;
  uint64_t seed, base;
  CHK(draw_seed(c, &seed, &base));
  c->slot_seed[slot] = seed;
  c->slot_base[slot] = base;
  {
    StageScope p(c, ST_H2F);
    k_h2f<<<nblk(n), WG, 0, st>>>(n, d_hashes, c->xmd, s);
  }
  {
    StageScope p(c, ST_VOTE);
    if (key.bytes)
      k_vm_votew<false><<<n, 64, LDS_VOTEW, st>>>(n, c->vm_votew, c->vm_consts, key.bytes, PkSrc{}, d_sigs, s, seed,
                                                  base, d_codes);
    else
      k_vm_votew<true><<<n, 64, LDS_VOTEW, st>>>(n, c->vm_votew_t, c->vm_consts, nullptr, key.pts, d_sigs, s, seed,
                                                 base, d_codes);
  }
  hipStream_t fst = c->fs[slot];
  HIPCHK(hipEventRecord(c->ev_front[slot], st));
  HIPCHK(hipStreamWaitEvent(fst, c->ev_front[slot], 0));
  int reg = 0;
  uint32_t m = (n + 3) / 4;
  {
    StageScope p(c, ST_FOLD, fst);
    k_vm_fold<VM_FOLD_UNITS><<<(m + VM_FOLD_UNITS - 1) / VM_FOLD_UNITS, 64, LDS_FOLD, fst>>>(
        n, c->vm_fold, c->vm_consts, Slab{s.p + (size_t)S_F * 12 * s.cap, s.cap}, Slab{nullptr, 0},
        region_F(c, slot, 0), d_codes);
  }
  CHK(fold_down(c, slot, fst, VM_SLICES, &reg, &m, 1));
  int32_t* verdict = c->result + RES_BATCH + slot;
  {
    StageScope p(c, ST_FINAL, fst);
    k_vm_fe<<<1, 64, LDS_FINAL1, fst>>>(c->vm_final1, c->vm_consts, region_F(c, slot, reg), verdict);
  }
  {
    StageScope p(c, ST_FALLBACK, fst);
    k_vm_votefe<<<n, 64, LDS_FINAL1, fst>>>(n, c->vm_final1, c->vm_consts, s, d_codes, verdict);
  }
  HIPCHK(hipEventRecord(c->ev_back[slot], fst));
  HIPCHK(hipGetLastError());
  c->slot_n[slot] = n;
  c->last_n = 0;  // no (f, r sigma) state for ovh_batch_partial_device / the standard bisection
  return 0;
}

// One batch through the pool (or the small-batch path for 2 <= n <= small_max): per-vote stages
// (batch_front), then on the slot's final stream the fold levels, the MSM, the combined check and
// the device-gated bisection. Nothing waits on the host. Caller holds c->mu.
static int verify_async_locked(ovh_ctx* c, size_t n, const uint8_t* d_sigs, const uint8_t* d_hashes, KeySrc key,
                               int32_t* d_codes) {
  CHK(ensure_cap(c, n));
  if (n >= 2 && n <= c->small_max) return verify_small_locked(c, (uint32_t)n, d_sigs, d_hashes, key, d_codes);
  int slot;
  CHK(pool_take_slot(c, &slot));
  CHK(batch_front(c, slot, (uint32_t)n, d_sigs, d_hashes, key, d_codes, true));
  hipStream_t fst = c->fs[slot];
  uint32_t m;
  int reg;
  CHK(side_front(c, slot, 4, &reg, &m));
  plog_stamp(c, slot, PLOG_EV_FOLD, fst);
  int32_t* verdict = c->result + RES_BATCH + slot;
  CHK(enqueue_msm(c, fst, slot, (uint32_t)n, d_codes));
  plog_stamp(c, slot, PLOG_EV_MSM, fst);
  enqueue_final(c, fst, region_F(c, slot, reg), region_S(c, slot, reg), m, verdict, msm_S(c, slot));
  plog_stamp(c, slot, PLOG_EV_FINAL, fst);
  enqueue_bisect(c, fst, slot, (uint32_t)n, d_codes, verdict);
  plog_stamp(c, slot, PLOG_EV_BACK, fst);
  HIPCHK(hipEventRecord(c->ev_back[slot], fst));
  HIPCHK(hipGetLastError());
  return 0;
}

// Host inputs -> staging buffer (sigs, hashes, pks, codes) on the main stream.
static int stage_batch(ovh_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* hashes, const uint8_t* pks,
                       uint8_t** d) {
  CHK(ensure_in(c, n * (96 + 32 + 48 + 4 + 4) + 64));
  *d = c->in_buf;
  HIPCHK(hipMemcpyAsync(*d, sigs, n * 96, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(*d + n * 96, hashes, n * 32, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(*d + n * 128, pks, n * 48, hipMemcpyHostToDevice, c->stream));
  return 0;
}

// The validator-table entry of each voter: votes whose key is in the table run the vote_t
// program (no key decompression / subgroup check), the others the vote program. perm lists the
// votes table-first (perm[j] = the caller's index of staged vote j), idx the table entry of each
// staged table vote; returns the number of table votes. perm stays empty when no reordering is
// needed (no table vote, or every vote in the table).
static size_t table_split(ovh_ctx* c, size_t n, const uint8_t* pks, std::vector<uint32_t>& perm,
                          std::vector<int32_t>& idx) {
  perm.clear();
  idx.clear();
  if (!c->tab.n) return 0;
  std::vector<int32_t> e(n);
  std::string k(48, '\0');
  size_t t = 0;
  for (size_t i = 0; i < n; ++i) {
    memcpy(&k[0], pks + 48 * i, 48);
    auto it = c->tab.index.find(k);
    e[i] = it == c->tab.index.end() ? -1 : (int32_t)it->second;
    t += e[i] >= 0;
  }
  if (t == n) {
    idx = std::move(e);
    return n;
  }
  if (t == 0) return 0;
  perm.reserve(n);
  for (size_t i = 0; i < n; ++i)
    if (e[i] >= 0) {
      perm.push_back((uint32_t)i);
      idx.push_back(e[i]);
    }
  for (size_t i = 0; i < n; ++i)
    if (e[i] < 0) perm.push_back((uint32_t)i);
  return t;
}

// Host inputs of n votes staged table-first (table_split) on the main stream: sigs | hashes |
// pks | codes | table indices. *t = the number of table votes; perm as table_split.
static int stage_split(ovh_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* hashes, const uint8_t* pks,
                       uint8_t** d, size_t* t, std::vector<uint32_t>& perm) {
  std::vector<int32_t> idx;
  *t = table_split(c, n, pks, perm, idx);
  if (perm.empty()) {
    CHK(stage_batch(c, n, sigs, hashes, pks, d));
  } else {
    std::vector<uint8_t> h(n * 176);
    for (size_t j = 0; j < n; ++j) {
      const size_t i = perm[j];
      memcpy(&h[96 * j], sigs + 96 * i, 96);
      memcpy(&h[n * 96 + 32 * j], hashes + 32 * i, 32);
      memcpy(&h[n * 128 + 48 * j], pks + 48 * i, 48);
    }
    CHK(stage_batch(c, n, h.data(), h.data() + n * 96, h.data() + n * 128, d));
    HIPCHK(hipStreamSynchronize(c->stream));  // the pageable copy of h completed before h dies
  }
  if (*t) HIPCHK(hipMemcpyAsync(*d + n * 180, idx.data(), *t * 4, hipMemcpyHostToDevice, c->stream));
  return 0;
}

// The key source of staged votes [lo, lo + cnt): the table for lo < t, else the key bytes.
static KeySrc staged_key(ovh_ctx* c, size_t n, uint8_t* d, size_t t, size_t lo) {
  if (lo < t) return KeySrc{nullptr, PkSrc{c->tab.planes, c->tab.cap, c->tab.flags, (int32_t*)(d + n * 180) + lo}};
  return KeySrc{d + n * 128 + 48 * lo, PkSrc{}};
}

// ---- same-message batches
// Host plan of a staged batch: the distinct hashes (in first-seen order), each vote's group, the
// per-group pairwise-sum levels of its votes' r pk (pairs (a, b): P[a] += P[b], disjoint within a
// level) and each group's root. Device layout at offset `off` of the staging buffer:
// gid (4 n) | distinct hashes (32 G) | heads (4 G) | pairs (8 per pair, level by level).
struct SameMsgPlan {
  uint32_t G = 0;
  std::vector<uint32_t> gid, head, pairs, level_off;  // level_off: pair offsets, one past the last
  std::vector<uint8_t> ghash;
  size_t off = 0, bytes = 0;
};

static void samemsg_plan(size_t n, const uint8_t* hashes, const std::vector<uint32_t>& perm, SameMsgPlan& pl) {
  std::unordered_map<std::string, uint32_t> idx;
  std::vector<std::vector<uint32_t>> members;
  pl.gid.resize(n);
  std::string k(32, '\0');
  for (size_t j = 0; j < n; ++j) {
    const size_t i = perm.empty() ? j : perm[j];
    memcpy(&k[0], hashes + 32 * i, 32);
    auto it = idx.find(k);
    uint32_t g;
    if (it == idx.end()) {
      g = (uint32_t)members.size();
      idx.emplace(k, g);
      members.emplace_back();
      pl.ghash.insert(pl.ghash.end(), hashes + 32 * i, hashes + 32 * i + 32);
    } else {
      g = it->second;
    }
    pl.gid[j] = g;
    members[g].push_back((uint32_t)j);
  }
  pl.G = (uint32_t)members.size();
  for (const auto& m : members) pl.head.push_back(m[0]);
  pl.level_off.push_back(0);
  for (size_t stride = 1;; stride <<= 1) {
    bool any = false;
    for (const auto& m : members)
      for (size_t q = 0; q + stride < m.size(); q += 2 * stride) {
        pl.pairs.push_back(m[q]);
        pl.pairs.push_back(m[q + stride]);
        any = true;
      }
    if (!any) break;
    pl.level_off.push_back((uint32_t)(pl.pairs.size() / 2));
  }
  pl.bytes = 4 * n + 32 * (size_t)pl.G + 4 * (size_t)pl.G + 4 * pl.pairs.size();
}

// A same-message batch in `slot` (taken by the caller): sigs (n x 96), the table votes [0, t)
// with their table indices tidx, the other votes' keys pks (n - t x 48); the plan's device arrays
// gid | ghash | head | pairs (SameMsgPlan) and its host level offsets. Main stream: the per-vote
// programs (vsame_t over the table votes, vsame over the others); the side stream, beside them:
// hash_to_field + hash_to_G2 per distinct hash; then (final stream) the H = O codes, (side stream)
// the per-hash sums of r pk, the per-hash Miller loops and their fold, beside (final stream) the
// MSM of sum r_i sigma_i, the final check, and -- gated on its verdict -- the per-vote bisection.
// Nothing waits on the host: ovh_verify_batch syncs, ovh_verify_samemsg_device_async does not.
// one (that API: a single hash, as a kernel argument): vsame runs on one of two per-vote streams
// in turn, so consecutive batches' vsame grids are co-resident (two waves per SIMD: 1.36x the
// throughput of one, profiles/r04e_occupancy_ab.json), and the hash goes to the slot's hash
// stream without waiting for the per-vote work. Caller holds c->mu and has called
// ensure_cap(c, n).
// The 32-byte hash of a one-hash batch into its slot's device word (a kernel argument, so the
// host's copy may change as soon as the launch returns).
struct Hash32 {
  uint32_t w[8];
};
__global__ void k_put_hash(Hash32 h, uint8_t* dst) {
  if (threadIdx.x < 8) reinterpret_cast<uint32_t*>(dst)[threadIdx.x] = h.w[threadIdx.x];
}

struct SameMsgDev {
  uint32_t G;
  const uint32_t* gid;
  const uint8_t* ghash;
  const uint32_t* head;
  const uint32_t* pairs;
  const std::vector<uint32_t>* level_off;
};

static int verify_samemsg_locked(ovh_ctx* c, int slot, size_t n, const uint8_t* sigs, size_t t, const int32_t* tidx,
                                 const uint8_t* pks, const SameMsgDev& pl, int32_t* dc, const Hash32* one = nullptr) {
  if (!c->gslab[slot] || c->gcap[slot] < c->cap) {
    if (c->gslab[slot]) (void)hipFree(c->gslab[slot]);
    c->gslab[slot] = nullptr;
    HIPCHK(hipMalloc(&c->gslab[slot], (((size_t)VM_G_PLANES * 12 + 1) * c->cap + 16) * 4));
    c->gcap[slot] = c->cap;
  }
  const uint32_t G = pl.G, N = (uint32_t)n, T = (uint32_t)t;
  const Slab g{c->gslab[slot], c->gcap[slot]};
  uint32_t* ghinf = c->gslab[slot] + (size_t)VM_G_PLANES * 12 * g.cap;
  uint32_t* hsel = ghinf + g.cap;  // k_pick_head's choice (the word after the H = O flags)
  const Slab gH{g.p + (size_t)VM_G_H * 12 * g.cap, g.cap};
  const Slab s{c->state_slot[slot], c->cap};
  const Slab P{s.p + (size_t)S_F * 12 * s.cap, s.cap};  // r pk of every vote, then the sums in place
  const uint32_t* gid = pl.gid;
  const uint8_t* ghash = pl.ghash;
  const uint32_t* head = pl.head;
  const uint32_t* pairs = pl.pairs;
  c->ev_mask = 0;
  uint64_t seed, base;
  CHK(draw_seed(c, &seed, &base));
  c->slot_seed[slot] = seed;
  c->slot_base[slot] = base;
  const hipStream_t fst = c->fs[slot];
  hipStream_t st = c->stream;
  if (one) {
    // high priority: that pool's four hardware queues hold only these three streams -- the
    // batch path's per-vote pair when the context has it (a fourth and fifth high-priority
    // stream shared queue 8 with the hash_to_G2 stream and serialised vsame behind it, r04ab)
    hipStream_t* pair = c->vstream;
    for (hipStream_t* v : {&pair[0], &pair[1]})
      if (!*v) {
        int lo = 0, hi = 0;
        (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
        HIPCHK(stream_new(v, hi));
      }
    st = pair[c->pipe_k & 1];
  }
  // hash_to_G2 per hash beside the per-vote programs at normal priority (at the final streams'
  // low priority it took 2.8 ms beside 1,024 vsame waves, r04g): on the side stream for a staged
  // batch; for the one-hash API on ovh_stream itself, which carries nothing else of the batch.
  // HIP maps streams onto GPU_MAX_HW_QUEUES (4) hardware queues per priority, and two streams on
  // one queue run in order: a stream per slot for hash_to_G2 landed on the per-vote streams'
  // queues and serialised them (r04m trace), and on ovh_stream it delayed the next batch's
  // per-vote work (r04n), so the one-hash path runs on three high-priority streams (a pool of
  // their own: the two per-vote streams and this one) and the final streams (its key sums there).
  if (!c->xstream) HIPCHK(stream_new(&c->xstream, 0));
  // hash_to_G2 of the one-hash API: SM_H2G_STREAMS streams in turn (one wave each; on a single
  // stream consecutive batches' hash_to_G2 ran back to back)
  const uint32_t hk = one ? (uint32_t)(c->pipe_k % SM_H2G_STREAMS) : 0u;
  if (hk && !c->hstream[hk]) HIPCHK(stream_new(&c->hstream[hk], 0));
  // (the one-hash path's key sums on the final stream: on the side stream, beside the MSM, a
  // pipelined batch took 1.78-1.81 ms against 1.57-1.63, r06p)
  const hipStream_t xs = one ? fst : c->xstream, hs = hk ? c->hstream[hk] : c->xstream;
  HIPCHK(hipEventRecord(c->ev_front[slot], c->stream));  // the inputs (and the slot free: take_slot)
  HIPCHK(hipStreamWaitEvent(hs, c->ev_front[slot], 0));
  HIPCHK(hipStreamWaitEvent(fst, c->ev_front[slot], 0));
  if (st != c->stream) HIPCHK(hipStreamWaitEvent(st, c->ev_front[slot], 0));
  {
    StageScope p(c, ST_H2F, hs);
    if (one) k_put_hash<<<1, 64, 0, hs>>>(*one, (uint8_t*)ghash);
    k_h2f<<<nblk(G), WG, 0, hs>>>(G, ghash, c->xmd, g);
    k_vm_h2g<<<(G + VM_SLICES - 1) / VM_SLICES, 64, LDS_H2G, hs>>>(G, c->vm_h2g, c->vm_consts, g, ghinf);
  }
  HIPCHK(hipEventRecord(c->ev_x[1], hs));
  HIPCHK(hipStreamWaitEvent(fst, c->ev_x[1], 0));
  const PkSrc tab{c->tab.planes, c->tab.cap, c->tab.flags, tidx};
  {
    StageScope p(c, ST_VOTE, st);
    if (N >= VSAME8_MIN) {  // eight votes per wave (VSAME8_MIN)
      if (T)
        k_vm_vsame<true, 8><<<(T + 7) / 8, 64, LDS_VSAME8, st>>>(T, 0, c->vm_vsame8_t, c->vm_consts, nullptr, tab, sigs,
                                                                 s, seed, base, dc);
      if (N > T)
        k_vm_vsame<false, 8><<<(N - T + 7) / 8, 64, LDS_VSAME8, st>>>(
            N - T, T, c->vm_vsame8, c->vm_consts, pks, PkSrc{}, sigs + 96 * (size_t)T, s, seed, base, dc);
    } else {
      if (T)
        k_vm_vsame<true><<<(T + VM_SLICES - 1) / VM_SLICES, 64, LDS_VSAME, st>>>(T, 0, c->vm_vsame_t, c->vm_consts,
                                                                                nullptr, tab, sigs, s, seed, base, dc);
      if (N > T)
        k_vm_vsame<false><<<(N - T + VM_SLICES - 1) / VM_SLICES, 64, LDS_VSAME, st>>>(
            N - T, T, c->vm_vsame, c->vm_consts, pks, PkSrc{}, sigs + 96 * (size_t)T, s, seed, base, dc);
    }
  }
  HIPCHK(hipEventRecord(c->ev_front[slot], st));
  HIPCHK(hipStreamWaitEvent(fst, c->ev_front[slot], 0));
  int reg = 0;
  uint32_t m = (G + 3) / 4;
  k_samemsg_fix<<<nblk(n), WG, 0, fst>>>(N, gid, ghinf, dc, P);
  // the per-hash key sums, Miller loops and their fold on the side stream, beside the MSM
  if (xs != fst) {
    HIPCHK(hipEventRecord(c->ev_x[2], fst));
    HIPCHK(hipStreamWaitEvent(xs, c->ev_x[2], 0));
  }
  {
    StageScope p(c, ST_FOLD, xs);
    const std::vector<uint32_t>& lo = *pl.level_off;
    for (size_t l = 0; l + 1 < lo.size(); ++l) {
      const uint32_t a = lo[l], np = lo[l + 1] - a;
      k_vm_g1pairs<<<(np + 64 / VM_G1PADD_W - 1) / (64 / VM_G1PADD_W), 64, LDS_G1PADD, xs>>>(
          np, c->vm_g1padd, G1PADD_STRIDE_W, c->vm_consts, pairs + 2 * (size_t)a, P);
    }
    // the head hash (k_pick_head) joins the final's loop; the others run their own Miller loops,
    // folded to one F
    k_pick_head<<<1, 64, 0, xs>>>(G, head, P, ghinf, hsel);
    if (G > 1) {
      m = (G - 1 + 3) / 4;
      k_vm_gmil<<<G, 64, LDS_GMIL, xs>>>(G, hsel, c->vm_gmil, c->vm_consts, head, P, g);
      k_vm_fold<VM_FOLD_UNITS><<<(m + VM_FOLD_UNITS - 1) / VM_FOLD_UNITS, 64, LDS_FOLD, xs>>>(
          G - 1, c->vm_fold, c->vm_consts, Slab{g.p + (size_t)VM_G_F * 12 * g.cap + 1, g.cap}, Slab{nullptr, 0},
          region_F(c, slot, 0), nullptr);
    }
  }
  if (G > 1) CHK(fold_down(c, slot, xs, 1, &reg, &m, 1));
  CHK(enqueue_msm(c, fst, slot, N, dc));
  if (xs != fst) {
    HIPCHK(hipEventRecord(c->ev_x[3], xs));
    HIPCHK(hipStreamWaitEvent(fst, c->ev_x[3], 0));
  }
  int32_t* verdict = c->result + RES_BATCH + slot;
  {
    StageScope p(c, ST_FINAL, fst);
    k_vm_gfin<<<1, 64, LDS_GFIN, fst>>>(c->vm_gfin, c->vm_consts, G > 1 ? region_F(c, slot, reg) : Slab{nullptr, 0},
                                        head, hsel, P, gH, msm_S(c, slot), verdict);
  }
  {
    StageScope p(c, ST_FALLBACK, fst);
    if (T)
      k_vm_vote1h_b<true><<<T, 64, LDS_VOTE1H, fst>>>(T, 0, c->vm_vote_t1h, c->vm_consts, nullptr, tab, sigs, s, dc, gid,
                                                      gH, ghinf, verdict);
    if (N > T)
      k_vm_vote1h_b<false><<<N - T, 64, LDS_VOTE1H, fst>>>(N - T, T, c->vm_vote1h, c->vm_consts, pks, PkSrc{},
                                                           sigs + 96 * (size_t)T, s, dc, gid, gH, ghinf, verdict);
    k_vm_votefe<<<N, 64, LDS_FINAL1, fst>>>(N, c->vm_final1, c->vm_consts, s, dc, verdict);
  }
  HIPCHK(hipEventRecord(c->ev_back[slot], fst));
  HIPCHK(hipGetLastError());
  c->slot_n[slot] = N;
  c->last_n = 0;  // no (f, r sigma) state for ovh_batch_partial_device / the standard bisection
  ++c->sm_batches;
  c->sm_votes += n;
  c->sm_hashes += G;
  return 0;
}

// ovh_verify_batch on one device (caller holds c->mu): codes (host) of n votes. Table votes and
// the others run as two batches (each its own combined check) when a batch mixes them.
static int verify_host_locked(ovh_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* hashes, const uint8_t* pks,
                              int32_t* codes) {
  HIPCHK(hipSetDevice(c->device));
  // same-message batches: at least two votes per distinct hash on average (a round's votes)
  SameMsgPlan pl;
  std::vector<uint32_t> perm;
  std::vector<int32_t> tidx;
  const size_t t0 = table_split(c, n, pks, perm, tidx);
  (void)t0;
  bool same = false;
  if (n >= 2 && (c->samemsg >= 2 || (c->samemsg == 1 && n > c->small_max))) {
    samemsg_plan(n, hashes, perm, pl);
    same = 2 * (size_t)pl.G <= n;
  }
  pl.off = (n * (96 + 32 + 48 + 4 + 4) + 255) / 256 * 256;
  CHK(ensure_in(c, same ? pl.off + pl.bytes + 64 : n * (96 + 32 + 48 + 4 + 4) + 64));
  uint8_t* d;
  size_t t;
  CHK(stage_split(c, n, sigs, hashes, pks, &d, &t, perm));
  int32_t* dc = (int32_t*)(d + n * 176);
  if (same) {
    std::vector<uint8_t> h(pl.bytes);
    memcpy(h.data(), pl.gid.data(), 4 * n);
    memcpy(h.data() + 4 * n, pl.ghash.data(), 32 * (size_t)pl.G);
    memcpy(h.data() + 4 * n + 32 * (size_t)pl.G, pl.head.data(), 4 * (size_t)pl.G);
    if (!pl.pairs.empty()) memcpy(h.data() + 4 * n + 36 * (size_t)pl.G, pl.pairs.data(), 4 * pl.pairs.size());
    HIPCHK(hipMemcpyAsync(d + pl.off, h.data(), pl.bytes, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));  // the pageable copy of h completed before h dies
    const uint8_t* ex = d + pl.off;
    const uint32_t* head = (const uint32_t*)(ex + 4 * n + 32 * (size_t)pl.G);
    const SameMsgDev pd{pl.G, (const uint32_t*)ex, ex + 4 * n, head, head + pl.G, &pl.level_off};
    CHK(ensure_cap(c, n));
    int slot;
    CHK(take_slot(c, &slot));
    CHK(verify_samemsg_locked(c, slot, n, d, t, (const int32_t*)(d + n * 180), d + n * 128 + 48 * t, pd, dc));
  } else if (n == 1) {
    CHK(verify_one_locked(c, d, d + 96, staged_key(c, n, d, t, 0), dc, hashes));
  } else {
    for (int part = 0; part < 2; ++part) {  // table votes [0, t), then the others [t, n)
      const size_t lo = part ? t : 0, cnt = part ? n - t : t;
      if (!cnt) continue;
      CHK(verify_async_locked(c, cnt, d + 96 * lo, d + n * 96 + 32 * lo, staged_key(c, n, d, t, lo), dc + lo));
    }
  }
  CHK(sync_all(c));
  if (perm.empty()) {
    HIPCHK(hipMemcpyAsync(codes, dc, 4 * n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
  } else {
    std::vector<int32_t> pc(n);
    HIPCHK(hipMemcpyAsync(pc.data(), dc, 4 * n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    for (size_t j = 0; j < n; ++j) codes[perm[j]] = pc[j];
  }
  return 0;
}

// Per-shard partial of `slot` (f folded to one, S from the MSM) -> AoS at `out` (device), on
// the main stream.
static int shard_partial(ovh_ctx* c, int slot, uint32_t n, const int32_t* d_codes, uint32_t* out, hipStream_t wait_on) {
  uint32_t m;
  int reg;
  CHK(pool_join(c, slot, c->stream, &reg, &m));
  CHK(fold_down(c, slot, c->stream, VM_SLICES, &reg, &m, 1));
  CHK(enqueue_msm(c, c->stream, slot, n, d_codes));
  if (wait_on) {  // the caller's earlier work on its stream (e.g. a gather reading `out`) first
    HIPCHK(hipEventRecord(c->ev_x[0], wait_on));
    HIPCHK(hipStreamWaitEvent(c->stream, c->ev_x[0], 0));
  }
  k_pack_partial2<<<1, 64, 0, c->stream>>>(region_F(c, slot, reg), msm_S(c, slot), out);
  HIPCHK(hipGetLastError());
  return 0;
}

// ---- multi-device (ovh_create_multi)
static void shard_range(size_t n, size_t nd, size_t d, size_t* lo, size_t* cnt) {
  const size_t base = n / nd, extra = n % nd;
  *lo = d * base + (d < extra ? d : extra);
  *cnt = base + (d < extra ? 1 : 0);
}

static int drain_host(ovh_ctx* root);

static int verify_host_multi(ovh_ctx* root, size_t n, const uint8_t* sigs, const uint8_t* hashes, const uint8_t* pks,
                             int32_t* codes) {
  const size_t nd = root->sub.size();
  std::vector<std::unique_lock<std::mutex>> locks;  // root (gather scratch), then every device
  locks.emplace_back(root->mu);
  for (ovh_ctx* s : root->sub) locks.emplace_back(s->mu);
  ovh_ctx* s0 = root->sub[0];
  CHK(drain_host(root));  // pipelined batches first (they share the partial buffers)
  // per device: its shard, staged table-first (stage_split), as up to two parts (table votes,
  // other votes), each a batch with its own partial
  struct Part {
    int slot;
    size_t lo, cnt;
  };
  std::vector<std::vector<Part>> parts(nd);
  std::vector<int32_t*> dcodes(nd, nullptr);
  std::vector<std::vector<uint32_t>> perms(nd);
  size_t k = 0;
  for (size_t d = 0; d < nd; ++d) {
    ovh_ctx* s = root->sub[d];
    size_t lo, cnt;
    shard_range(n, nd, d, &lo, &cnt);
    if (!cnt) continue;
    HIPCHK(hipSetDevice(s->device));
    CHK(ensure_in(s, cnt * (96 + 32 + 48 + 4 + 4) + 64));
    uint8_t* in;
    size_t t;
    CHK(stage_split(s, cnt, sigs + lo * 96, hashes + lo * 32, pks + lo * 48, &in, &t, perms[d]));
    dcodes[d] = (int32_t*)(in + cnt * 176);
    CHK(ensure_cap(s, cnt));
    for (int part = 0; part < 2; ++part) {  // table votes [0, t), then the others [t, cnt)
      const size_t plo = part ? t : 0, pc = part ? cnt - t : t;
      if (!pc) continue;
      Part p{0, plo, pc};
      CHK(pool_take_slot(s, &p.slot));
      s->test_base = root->test_base + lo + plo;  // OVH_FLAG_TEST_RLC only: one global index per vote
      CHK(batch_front(s, p.slot, (uint32_t)pc, in + 96 * plo, in + cnt * 96 + 32 * plo, staged_key(s, cnt, in, t, plo),
                      dcodes[d] + plo, false, true, true));
      uint32_t* po = s->part_out + (size_t)(parts[d].size()) * (OVH_PARTIAL_BYTES / 4);
      CHK(shard_partial(s, p.slot, (uint32_t)pc, dcodes[d] + plo, po, nullptr));
      // partial -> devices[0] (peer copy over xGMI), ordered on this device's stream
      HIPCHK(hipMemcpyPeerAsync(root->gather + k * OVH_PARTIAL_BYTES, s0->device, po, s->device, OVH_PARTIAL_BYTES,
                                s->stream));
      parts[d].push_back(p);
      ++k;
    }
    HIPCHK(hipEventRecord(s->ev_x[1], s->stream));
  }
  if (!k) return 0;
  HIPCHK(hipSetDevice(s0->device));
  for (size_t d = 0; d < nd; ++d)
    if (dcodes[d]) HIPCHK(hipStreamWaitEvent(s0->fstream, root->sub[d]->ev_x[1], 0));
  Slab uF{root->mfin, 16}, uS{root->mfin + (size_t)12 * 12 * 16, 16};
  Slab F = uF, S = uS;
  uint32_t m = (uint32_t)k;
  k_unpack_partials<<<(uint32_t)((k * PART_PLANES + 63) / 64), 64, 0, s0->fstream>>>((uint32_t)k,
                                                                                   (const uint32_t*)root->gather, uF, uS);
  if (k > 4) {
    uint32_t* o = root->mfin + (size_t)PART_PLANES * 12 * 16;
    F = Slab{o, 4};
    S = Slab{o + (size_t)12 * 12 * 4, 4};
    k_vm_fold<VM_FOLD_UNITS><<<1, 64, LDS_FOLD, s0->fstream>>>((uint32_t)k, s0->vm_fold, s0->vm_consts, uF, uS, F,
                                                             nullptr);
    m = (uint32_t)((k + 3) / 4);
  }
  enqueue_final(s0, s0->fstream, F, S, m, s0->result + RES_MULTI);
  HIPCHK(hipGetLastError());
  int32_t verdict = 0;
  HIPCHK(hipMemcpyAsync(&verdict, s0->result + RES_MULTI, 4, hipMemcpyDeviceToHost, s0->fstream));
  HIPCHK(hipStreamSynchronize(s0->fstream));
  std::vector<std::vector<int32_t>> staged(nd);
  for (size_t d = 0; d < nd; ++d) {
    if (!dcodes[d]) continue;
    ovh_ctx* s = root->sub[d];
    size_t lo, cnt;
    shard_range(n, nd, d, &lo, &cnt);
    HIPCHK(hipSetDevice(s->device));
    if (!verdict)
      for (const Part& p : parts[d])
        enqueue_bisect(s, s->stream, p.slot, (uint32_t)p.cnt, dcodes[d] + p.lo, nullptr);
    int32_t* dst = codes + lo;
    if (!perms[d].empty()) {
      staged[d].resize(cnt);
      dst = staged[d].data();
    }
    HIPCHK(hipMemcpyAsync(dst, dcodes[d], 4 * cnt, hipMemcpyDeviceToHost, s->stream));
  }
  for (size_t d = 0; d < nd; ++d)
    if (dcodes[d]) {
      HIPCHK(hipSetDevice(root->sub[d]->device));
      HIPCHK(hipStreamSynchronize(root->sub[d]->stream));
      if (!perms[d].empty()) {
        size_t lo, cnt;
        shard_range(n, nd, d, &lo, &cnt);
        for (size_t j = 0; j < cnt; ++j) codes[lo + perms[d][j]] = staged[d][j];
      }
    }
  HIPCHK(hipSetDevice(root->device));  // the caller's thread back on devices[0]
  return 0;
}

static int stage_partials(ovh_ctx* c, hipStream_t st, size_t k, const uint8_t* d_partials, uint32_t* scratch, Slab* F,
                          Slab* S, uint32_t* m);

// ---- pipelined host batches (ovh_verify_batch_async) on single and multi-device contexts
static std::vector<ovh_ctx*> devices_of(ovh_ctx* c) {
  return c->sub.empty() ? std::vector<ovh_ctx*>{c} : c->sub;
}

// pinned host staging + its device copy for ring slot j (>= bytes)
static int ensure_hst(ovh_ctx* c, int j, size_t bytes) {
  if (bytes <= c->hst_cap[j] && c->hst_h[j]) return 0;
  size_t cap = 1 << 16;
  while (cap < bytes) cap <<= 1;
  CHK(sync_all(c));
  if (c->hst_h[j]) (void)hipHostFree(c->hst_h[j]);
  if (c->hst_d[j]) (void)hipFree(c->hst_d[j]);
  c->hst_h[j] = nullptr;
  c->hst_d[j] = nullptr;
  c->hst_cap[j] = 0;
  HIPCHK(hipHostMalloc((void**)&c->hst_h[j], cap, hipHostMallocDefault));
  HIPCHK(hipMalloc(&c->hst_d[j], cap));
  c->hst_cap[j] = cap;
  return 0;
}

// Stage one device's votes for ring slot j: table-first into the pinned buffer, then one H2D copy
// on the main stream (layout of stage_split: sigs | hashes | pks | codes | table indices).
static int stage_pinned(ovh_ctx* s, int j, size_t cnt, const uint8_t* sigs, const uint8_t* hashes, const uint8_t* pks,
                        size_t* t, std::vector<uint32_t>& perm) {
  std::vector<int32_t> idx;
  *t = table_split(s, cnt, pks, perm, idx);
  CHK(ensure_hst(s, j, cnt * 184 + 64));
  uint8_t* h = s->hst_h[j];
  if (perm.empty()) {
    memcpy(h, sigs, cnt * 96);
    memcpy(h + cnt * 96, hashes, cnt * 32);
    memcpy(h + cnt * 128, pks, cnt * 48);
  } else {
    for (size_t q = 0; q < cnt; ++q) {
      const size_t i = perm[q];
      memcpy(h + 96 * q, sigs + 96 * i, 96);
      memcpy(h + cnt * 96 + 32 * q, hashes + 32 * i, 32);
      memcpy(h + cnt * 128 + 48 * q, pks + 48 * i, 48);
    }
  }
  if (*t) memcpy(h + cnt * 180, idx.data(), *t * 4);
  HIPCHK(hipMemcpyAsync(s->hst_d[j], h, cnt * 176, hipMemcpyHostToDevice, s->stream));
  if (*t) HIPCHK(hipMemcpyAsync(s->hst_d[j] + cnt * 180, h + cnt * 180, *t * 4, hipMemcpyHostToDevice, s->stream));
  return 0;
}

// Oldest batch in flight: wait for its codes (pinned) and write them to the caller's array.
static int complete_front(ovh_ctx* root) {
  const std::vector<ovh_ctx*> devs = devices_of(root);
  HostBatch& hb = root->hq.front();
  for (const HostBatch::Dev& dv : hb.dev) {
    ovh_ctx* s = devs[dv.d];
    HIPCHK(hipSetDevice(s->device));
    HIPCHK(hipEventSynchronize(s->ev_m[hb.ring][3]));
    const int32_t* pc = (const int32_t*)(s->hst_h[hb.ring] + dv.cnt * 176);
    if (dv.perm.empty()) memcpy(hb.codes + dv.lo, pc, dv.cnt * 4);
    else
      for (size_t q = 0; q < dv.cnt; ++q) hb.codes[dv.lo + dv.perm[q]] = pc[q];
  }
  root->hq.pop_front();
  return 0;
}

static int drain_host(ovh_ctx* root) {
  while (!root->hq.empty()) CHK(complete_front(root));
  return 0;
}

// One context: the batch's parts (table votes, other votes) through the pipelined batch path
// (verify_async_locked), the codes read back on the last part's final stream. Caller holds c->mu.
static int submit_host_single(ovh_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* hashes, const uint8_t* pks,
                              int32_t* codes) {
  if (c->hq.size() >= OVH_BATCH_SLOTS) CHK(complete_front(c));
  const int j = (int)(c->hb_k++ % OVH_BATCH_SLOTS);
  HostBatch hb;
  hb.codes = codes;
  hb.n = n;
  hb.ring = j;
  hb.dev.push_back(HostBatch::Dev{0, 0, n, {}});
  size_t t;
  CHK(stage_pinned(c, j, n, sigs, hashes, pks, &t, hb.dev[0].perm));
  uint8_t* in = c->hst_d[j];
  int32_t* dc = (int32_t*)(in + n * 176);
  hipStream_t last = c->stream;
  if (n == 1) {
    CHK(verify_one_locked(c, in, in + 96, staged_key(c, n, in, t, 0), dc));
  } else {
    int prev = -1;
    for (int part = 0; part < 2; ++part) {  // table votes [0, t), then the others [t, n)
      const size_t lo = part ? t : 0, cnt = part ? n - t : t;
      if (!cnt) continue;
      CHK(verify_async_locked(c, cnt, in + 96 * lo, in + n * 96 + 32 * lo, staged_key(c, n, in, t, lo), dc + lo));
      if (prev >= 0) HIPCHK(hipStreamWaitEvent(c->fs[c->last_slot], c->ev_back[prev], 0));
      prev = c->last_slot;
      last = c->fs[c->last_slot];
    }
  }
  HIPCHK(hipMemcpyAsync(c->hst_h[j] + n * 176, dc, n * 4, hipMemcpyDeviceToHost, last));
  HIPCHK(hipEventRecord(c->ev_m[j][3], last));
  c->hq.push_back(std::move(hb));
  return 0;
}

// Several devices: per device its shard's parts through hash_to_field + the vote kernel (main
// stream) and the fold levels, MSM and packing (final stream), each packed partial peer-copied
// to this batch's final device -- devices[k mod ndev] for the k-th batch, so the combined checks
// rotate -- whose final stream runs the combined check and sends the verdict back to every
// device; each device then runs its device-gated bisection and reads its codes back. Nothing
// blocks the host: the next batch's per-vote work overlaps this batch's combined check on every
// device. Caller holds root->mu and every device's mu.
static int submit_host_multi(ovh_ctx* root, size_t n, const uint8_t* sigs, const uint8_t* hashes, const uint8_t* pks,
                             int32_t* codes) {
  const size_t nd = root->sub.size();
  if (root->hq.size() >= OVH_BATCH_SLOTS) CHK(complete_front(root));
  const int j = (int)(root->hb_k % OVH_BATCH_SLOTS);
  // the final device rotates over the devices with peer access to and from all others
  ovh_ctx* F = root->sub[root->fin_devs.empty() ? 0 : root->fin_devs[root->hb_k % root->fin_devs.size()]];
  ++root->hb_k;
  HostBatch hb;
  hb.codes = codes;
  hb.n = n;
  hb.ring = j;
  struct Part {
    ovh_ctx* s;
    int slot, pi;
    size_t plo, pc;
    int32_t* dcodes;
  };
  std::vector<Part> ps;
  std::vector<size_t> first;  // index into ps of each device's first part
  size_t k = 0;
  if (!F->mg) {
    HIPCHK(hipSetDevice(F->device));
    HIPCHK(hipMalloc(&F->mg, (size_t)OVH_BATCH_SLOTS * 16 * OVH_PARTIAL_BYTES));
  }
  uint8_t* gather = F->mg + (size_t)j * 16 * OVH_PARTIAL_BYTES;
  for (size_t d = 0; d < nd; ++d) {
    ovh_ctx* s = root->sub[d];
    size_t lo, cnt;
    shard_range(n, nd, d, &lo, &cnt);
    if (!cnt) continue;
    HIPCHK(hipSetDevice(s->device));
    hb.dev.push_back(HostBatch::Dev{d, lo, cnt, {}});
    size_t t;
    CHK(stage_pinned(s, j, cnt, sigs + lo * 96, hashes + lo * 32, pks + lo * 48, &t, hb.dev.back().perm));
    uint8_t* in = s->hst_d[j];
    int32_t* dcodes = (int32_t*)(in + cnt * 176);
    CHK(ensure_cap(s, cnt));
    first.push_back(ps.size());
    int pi = 0;
    for (int part = 0; part < 2; ++part) {  // table votes [0, t), then the others [t, cnt)
      const size_t plo = part ? t : 0, pc = part ? cnt - t : t;
      if (!pc) continue;
      int slot;
      CHK(pool_take_slot(s, &slot));
      s->test_base = root->test_base + lo + plo;  // OVH_FLAG_TEST_RLC only: one global index per vote
      CHK(batch_front(s, slot, (uint32_t)pc, in + 96 * plo, in + cnt * 96 + 32 * plo, staged_key(s, cnt, in, t, plo),
                      dcodes + plo, false, true, true));  // (peer copies of the partials: grids per batch)
      const hipStream_t fst = s->fs[slot];
      int reg;
      uint32_t m;
      CHK(side_front(s, slot, 1, &reg, &m));
      CHK(enqueue_msm(s, fst, slot, (uint32_t)pc, dcodes + plo));
      uint32_t* po = s->part_out + ((size_t)j * 2 + pi) * (OVH_PARTIAL_BYTES / 4);
      k_pack_partial2<<<1, 64, 0, fst>>>(region_F(s, slot, reg), msm_S(s, slot), po);
      HIPCHK(hipMemcpyPeerAsync(gather + k * OVH_PARTIAL_BYTES, F->device, po, s->device, OVH_PARTIAL_BYTES, fst));
      HIPCHK(hipEventRecord(s->ev_m[j][pi], fst));
      ps.push_back(Part{s, slot, pi, plo, pc, dcodes});
      ++k;
      ++pi;
    }
  }
  // the combined check on the batch's final device
  HIPCHK(hipSetDevice(F->device));
  // consecutive batches' combined checks alternate between the final device's two final streams
  const hipStream_t fin = (root->hb_k & 1) ? F->fstream2 : F->fstream;
  for (const Part& p : ps) HIPCHK(hipStreamWaitEvent(fin, p.s->ev_m[j][p.pi], 0));
  Slab PF, PS;
  uint32_t m;
  CHK(stage_partials(F, fin, k, gather, F->fin + (size_t)j * FIN_STRIDE, &PF, &PS, &m));
  int32_t* fv = F->result + RES_MULTI + 1 + j;
  enqueue_final(F, fin, PF, PS, m, fv);
  for (size_t q : first)
    if (ps[q].s != F)
      HIPCHK(hipMemcpyPeerAsync(ps[q].s->result + RES_MULTI + 1 + j, ps[q].s->device, fv, F->device, 4, fin));
  HIPCHK(hipEventRecord(F->ev_m[j][2], fin));
  // per device: device-gated bisection of its parts, then the codes into the pinned buffer
  for (size_t e = 0; e < first.size(); ++e) {
    const Part& p0 = ps[first[e]];
    ovh_ctx* s = p0.s;
    const size_t end = e + 1 < first.size() ? first[e + 1] : ps.size();
    const size_t cnt = hb.dev[e].cnt;
    HIPCHK(hipSetDevice(s->device));
    const hipStream_t bst = s->fs[p0.slot];
    HIPCHK(hipStreamWaitEvent(bst, F->ev_m[j][2], 0));
    for (size_t q = first[e]; q < end; ++q) {
      enqueue_bisect(s, bst, ps[q].slot, (uint32_t)ps[q].pc, ps[q].dcodes + ps[q].plo, s->result + RES_MULTI + 1 + j);
      HIPCHK(hipEventRecord(s->ev_back[ps[q].slot], bst));
    }
    HIPCHK(hipMemcpyAsync(s->hst_h[j] + cnt * 176, p0.dcodes, cnt * 4, hipMemcpyDeviceToHost, bst));
    HIPCHK(hipEventRecord(s->ev_m[j][3], bst));
  }
  HIPCHK(hipGetLastError());
  root->hq.push_back(std::move(hb));
  return 0;
}

static ovh_ctx* pick_sub(ovh_ctx* c) {
  if (c->sub.empty()) return c;
  return c->sub[c->rr.fetch_add(1) % c->sub.size()];
}

// ---- verdict cache
static std::string cache_key(const uint8_t* sig, const uint8_t* hash, const uint8_t* pk) {
  std::string k(176, '\0');
  memcpy(&k[0], sig, 96);
  memcpy(&k[96], hash, 32);
  memcpy(&k[128], pk, 48);
  return k;
}

static void cache_put(ovh_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* hashes, const uint8_t* pks,
                      const int32_t* codes) {
  std::lock_guard<std::mutex> g(c->cache.mu);
  if (!c->cache.cap) return;
  for (size_t i = 0; i < n; ++i) {
    std::string k = cache_key(sigs + 96 * i, hashes + 32 * i, pks + 48 * i);
    auto it = c->cache.map.find(k);
    if (it != c->cache.map.end()) {
      it->second = codes[i];
      continue;
    }
    while (c->cache.map.size() >= c->cache.cap && !c->cache.fifo.empty()) {
      c->cache.map.erase(c->cache.fifo.front());
      c->cache.fifo.pop_front();
    }
    c->cache.map.emplace(k, codes[i]);
    c->cache.fifo.push_back(std::move(k));
  }
}

static bool cache_get(ovh_ctx* c, const uint8_t* sig, const uint8_t* hash, const uint8_t* pk, int32_t* code) {
  std::lock_guard<std::mutex> g(c->cache.mu);
  if (!c->cache.cap) return false;
  auto it = c->cache.map.find(cache_key(sig, hash, pk));
  if (it == c->cache.map.end()) {
    ++c->cache.misses;
    return false;
  }
  ++c->cache.hits;
  *code = it->second;
  return true;
}

// ---- key parse
// a parsed secret scalar on the host stack, wiped when it goes out of scope
struct SecretBytes {
  uint8_t b[32];
  ~SecretBytes() { keygen::wipe(b, sizeof b); }
};

static int sk_parse(const ovh_ctx* c, const uint8_t* key, size_t len, uint8_t out[32]) {
  const bool ok = (c->flags & OVH_FLAG_SK_RAW) ? keygen::sk_raw(out, key, len) : keygen::key_gen(out, key, len);
  return ok ? 0 : BLST_BAD_ENCODING;
}

extern "C" {

static void destroy_one(ovh_ctx* c);

ovh_ctx* ovh_create(int device, const uint8_t* dst, size_t dst_len, uint32_t flags) {
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  ovh_ctx* c = new (std::nothrow) ovh_ctx();
  if (!c) return nullptr;
  c->device = device;
  c->flags = flags;
  // the two environment knobs (DESIGN.md sections 3.2, 3.3): the small-batch threshold and the
  // same-message routing
  if (const char* e = getenv("OVH_SMALL_MAX")) c->small_max = (uint32_t)atoi(e);
  if (const char* e = getenv("OVH_SAMEMSG")) c->samemsg = atoi(e);
  if (const char* e = getenv("OVH_SHARD_SPAN")) c->shard_span = (uint32_t)atoi(e);
  if (const char* e = getenv("OVH_SHARD_STREAMS")) c->shard_streams = atoi(e) == 3 ? 3u : 2u;
  if (const char* e = getenv("OVH_NFIN")) c->nfin = atoi(e) == 3 ? 3u : atoi(e) == 2 ? 2u : NFIN_STREAMS;
  int ncu = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || ncu <= 0) ncu = 256;
  // the pool: eight vote workgroups fit a CU (LDS); POOL_HOLES_PER_8CU of every eight CUs' 64
  // places are left to the final streams' kernels (fold, MSM, final, bisection) and the staging
  // and hash_to_field of the next batches, which would otherwise wait for the pool to drain. The
  // pool's places are split between the grids of the two pool streams (batch_front), which run
  // side by side: each grid holds half of them
  // OVH_FLAG_POOL_RESERVE: pool_rsv / 8 CUs of every XCC left free of the pool -- its workgroups
  // that land there leave at once (k_vm_pool; a CU mask on the pool streams made them blocking
  // streams on separate queues that ran one batch at a time, r06e-g); the grids keep their sizes,
  // so the dispatcher still deals them evenly. OVH_POOL_PER_CU (A/B): 8 = no holes on the others
  if (flags & OVH_FLAG_POOL_RESERVE) {
    c->pool_rsv = 8;
    if (const char* e = getenv("OVH_POOL_RESERVE")) c->pool_rsv = (uint32_t)atoi(e);
    if (c->pool_rsv % 8 || c->pool_rsv > 64 || (uint32_t)ncu <= 2 * c->pool_rsv) c->pool_rsv = 0;
  }
  const uint32_t pncu = (uint32_t)ncu - c->pool_rsv;
  uint32_t holes = POOL_HOLES_PER_8CU;
  if (const char* e = c->pool_rsv ? getenv("OVH_POOL_PER_CU") : nullptr) holes = atoi(e) == 8 ? 0u : holes;
  c->pool_wgs = ((uint32_t)ncu * 8 - (uint32_t)ncu * holes / 8) / 2;
  if (c->pool_wgs > POOL_MAX_WGS) c->pool_wgs = POOL_MAX_WGS;
  // the two grids as 4 + 3 workgroups per CU rather than 3.5 + 3.5: a grid of a whole number of
  // workgroups per CU is dealt evenly (one per SIMD), so every SIMD holds a pool wave -- with two
  // half-pools some CUs got 8 and others 6, some SIMDs none, and a lone batch's quads doubled up
  // on ~90 SIMDs (5.6 ms against 3.8 for a quad alone, r05az)
  c->pool_grid0 = std::min(4u * (uint32_t)ncu, 2 * c->pool_wgs - 1);
  c->ncu = (uint32_t)ncu;
  c->pool_ncu = pncu;
  if (!dst) {
    dst = DEFAULT_DST;
    dst_len = 43;
  }
  int lo = 0, hi = 0;
  (void)hipDeviceGetStreamPriorityRange(&lo, &hi);  // lo = numerically largest = lowest priority
  // streams: ovh_stream (normal priority), three final streams (lowest), the two pool streams
  // (highest; created with the context, so each holds a hardware queue of its own)
  bool ok = xmd_build_templates(c->xmd, dst, (uint32_t)dst_len) &&
            stream_new(&c->stream, 0) == hipSuccess &&
            stream_new(&c->fstream, lo) == hipSuccess &&
            stream_new(&c->fstream2, lo) == hipSuccess &&
            stream_new(&c->fstream3, lo) == hipSuccess &&
            (c->nfin < 4 || stream_new(&c->fstream4, lo) == hipSuccess) &&
            stream_new(&c->pool_st[0], hi) == hipSuccess &&
            stream_new(&c->pool_st[1], hi) == hipSuccess &&
            (c->shard_streams < 3 || stream_new(&c->pool_st[2], hi) == hipSuccess) &&
            hipMalloc(&c->part_out, (size_t)OVH_BATCH_SLOTS * 2 * 216 * 4) == hipSuccess && hipMalloc(&c->result, RES_WORDS * 4) == hipSuccess &&
            hipMemset(c->result, 0, RES_WORDS * 4) == hipSuccess &&
            hipMalloc(&c->pool_q, (size_t)PQ_WORDS * 8) == hipSuccess && hipMemset(c->pool_q, 0, (size_t)PQ_WORDS * 8) == hipSuccess &&
            hipMalloc(&c->pool_desc, sizeof(PoolBatch) * OVH_BATCH_SLOTS) == hipSuccess &&
            hipMemset(c->pool_desc, 0, sizeof(PoolBatch) * OVH_BATCH_SLOTS) == hipSuccess &&
            hipMalloc(&c->pool_scr, (size_t)2 * c->shard_streams * c->pool_wgs * VM_SLICES * VOTE_NSCR * 48) == hipSuccess &&
            hipHostMalloc((void**)&c->pool_err, 64, hipHostMallocCoherent | hipHostMallocMapped) == hipSuccess &&
            hipMalloc(&c->fin, (size_t)OVH_BATCH_SLOTS * FIN_STRIDE * 4) == hipSuccess && vm_init(c) == 0;
  if (ok) *c->pool_err = 0;
  if (ok && (flags & OVH_FLAG_VM_CLOCK))
    ok = hipMalloc(&c->plog, PLOG_TOTAL * 8) == hipSuccess && hipMemset(c->plog, 0, PLOG_TOTAL * 8) == hipSuccess;
  ok = ok && hipDeviceSynchronize() == hipSuccess;  // the memsets above are done before any batch
  // NFIN_STREAMS finals in flight at most (the pool's holes hold them; r02i ran one final stream
  // per slot and lost 2.4 ms in every third vote kernel to a workgroup that found no LDS beside
  // them)
  for (int k = 0; ok && k < OVH_BATCH_SLOTS; ++k) c->fs[k] = c->fstream;
  for (int k = 0; ok && k < OVH_BATCH_SLOTS; ++k)
    ok = hipEventCreateWithFlags(&c->ev_front[k], hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&c->ev_back[k], hipEventDisableTiming) == hipSuccess;
  for (int k = 0; ok && k < 4; ++k) ok = hipEventCreateWithFlags(&c->ev_x[k], hipEventDisableTiming) == hipSuccess;
  for (int k = 0; ok && k < OVH_BATCH_SLOTS; ++k)
    for (int q = 0; ok && q < 4; ++q) ok = hipEventCreateWithFlags(&c->ev_m[k][q], hipEventDisableTiming) == hipSuccess;
  if (ok && (flags & OVH_FLAG_PROFILE)) {
    for (int k = 0; ok && k < OVH_NSTAGES; ++k)
      ok = hipEventCreate(&c->ev0[k]) == hipSuccess && hipEventCreate(&c->ev1[k]) == hipSuccess;
    for (uint32_t k = 0; ok && k < ovh_ctx::VEV_CAP; ++k)
      ok = hipEventCreate(&c->vev0[k]) == hipSuccess && hipEventCreate(&c->vev1[k]) == hipSuccess;
  }
  if (!ok) {
    destroy_one(c);
    return nullptr;
  }
  return c;
}

ovh_ctx* ovh_create_multi(const int* devices, int ndev, const uint8_t* dst, size_t dst_len, uint32_t flags) {
  // up to 8 devices (one node): two partials per device (table / other votes) fill the 16-entry
  // gather buffer and one fold level
  if (!devices || ndev < 1 || ndev > 8) return nullptr;
  ovh_ctx* root = new (std::nothrow) ovh_ctx();
  if (!root) return nullptr;
  root->device = devices[0];
  root->flags = flags;
  for (int d = 0; d < ndev; ++d) {
    ovh_ctx* s = ovh_create(devices[d], dst, dst_len, flags);
    if (!s) {
      ovh_destroy(root);
      return nullptr;
    }
    root->sub.push_back(s);
  }
  // Peer access (xGMI) for every ordered pair of distinct devices: the partials go from every
  // device to the batch's final device, which rotates, and its verdict word back. peer[a][b] = 1
  // when device a's kernels / copies reach b's memory directly (or a and b are one device); a
  // pair without it still works (hipMemcpyPeerAsync stages through the host) but is not xGMI.
  // The final rotates only over devices that reach, and are reached by, every other device.
  root->peer.assign((size_t)ndev * ndev, 0);
  for (int a = 0; a < ndev; ++a)
    for (int b = 0; b < ndev; ++b) {
      uint8_t ok = 1;
      if (devices[a] != devices[b]) {
        int can = 0;
        ok = 0;
        if (hipDeviceCanAccessPeer(&can, devices[a], devices[b]) == hipSuccess && can) {
          (void)hipSetDevice(devices[a]);
          const hipError_t e = hipDeviceEnablePeerAccess(devices[b], 0);
          ok = (e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled) ? 1 : 0;
        }
      }
      root->peer[(size_t)a * ndev + b] = ok;
    }
  (void)hipGetLastError();
  for (int d = 0; d < ndev; ++d) {
    bool all = true;
    for (int e = 0; e < ndev; ++e) all = all && root->peer[(size_t)d * ndev + e] && root->peer[(size_t)e * ndev + d];
    if (all) root->fin_devs.push_back(d);
  }
  if (root->fin_devs.empty()) root->fin_devs.push_back(0);
  if (hipSetDevice(devices[0]) != hipSuccess || hipMalloc(&root->gather, (size_t)16 * OVH_PARTIAL_BYTES) != hipSuccess ||
      hipMalloc(&root->mfin, FIN_STRIDE * 4) != hipSuccess) {
    ovh_destroy(root);
    return nullptr;
  }
  return root;
}

int ovh_multi_peer_matrix(ovh_ctx* c, uint8_t* out, size_t cap) {
  if (!c || !out) return OVH_ERR_ARG;
  const size_t nd = c->sub.empty() ? 1 : c->sub.size();
  if (cap < nd * nd) return OVH_ERR_ARG;
  if (c->sub.empty()) {
    out[0] = 1;
    return 1;
  }
  memcpy(out, c->peer.data(), nd * nd);
  return (int)nd;
}

static void destroy_one(ovh_ctx* c) {
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (hipStream_t s : {c->fstream, c->fstream2, c->fstream3, c->fstream4, c->xstream, c->vstream[0], c->vstream[1], c->vstream[2], c->pool_st[0],
                        c->pool_st[1], c->pool_st[2], c->hstream[1], c->hstream[2], c->hstream[3]})
    if (s) (void)hipStreamSynchronize(s);
  for (int k = 0; k < OVH_BATCH_SLOTS; ++k)
    for (void* p : {(void*)c->grp_ok[k], (void*)c->msm_buf[k], (void*)c->gslab[k]})
      if (p) (void)hipFree(p);
  for (void* p : {(void*)c->state_all, (void*)c->red_all, (void*)c->pstage_all})
    if (p) (void)hipFree(p);
  for (void* p : {(void*)c->in_buf, (void*)c->part_out, (void*)c->result, (void*)c->pool_q, (void*)c->pool_desc,
                  (void*)c->pool_scr, (void*)c->plog, (void*)c->vm_consts,
                  (void*)c->fin, (void*)c->scr, (void*)c->scr_pk, (void*)c->scr_sig, (void*)c->comb,
                  (void*)c->tab.planes, (void*)c->tab.flags, (void*)c->qc_buf, (void*)c->qt_buf, (void*)c->hc_planes, (void*)c->hc_inf, (void*)c->gather,
                  (void*)c->mfin, (void*)c->sm1_plan, (void*)c->sm1_hash})
    if (p) (void)hipFree(p);
  for (void* p : c->vm_bufs) (void)hipFree(p);
  for (int k = 0; k < OVH_BATCH_SLOTS; ++k)
    for (hipEvent_t e : {c->ev_front[k], c->ev_back[k]})
      if (e) (void)hipEventDestroy(e);
  for (int k = 0; k < 4; ++k)
    if (c->ev_x[k]) (void)hipEventDestroy(c->ev_x[k]);
  for (int k = 0; k < OVH_BATCH_SLOTS; ++k) {
    for (int q = 0; q < 4; ++q)
      if (c->ev_m[k][q]) (void)hipEventDestroy(c->ev_m[k][q]);
    if (c->hst_h[k]) (void)hipHostFree(c->hst_h[k]);
    if (c->hst_d[k]) (void)hipFree(c->hst_d[k]);
  }
  if (c->mg) (void)hipFree(c->mg);
  for (int k = 0; k < OVH_NSTAGES; ++k) {
    if (c->ev0[k]) (void)hipEventDestroy(c->ev0[k]);
    if (c->ev1[k]) (void)hipEventDestroy(c->ev1[k]);
  }
  for (uint32_t k = 0; k < ovh_ctx::VEV_CAP; ++k) {
    if (c->vev0[k]) (void)hipEventDestroy(c->vev0[k]);
    if (c->vev1[k]) (void)hipEventDestroy(c->vev1[k]);
  }
  // the streams are parked, not destroyed (stream_new)
  for (hipStream_t s : {c->stream, c->fstream, c->fstream2, c->fstream3, c->fstream4, c->xstream, c->vstream[0], c->vstream[1], c->vstream[2],
                        c->pool_st[0], c->pool_st[1], c->pool_st[2], c->hstream[1], c->hstream[2], c->hstream[3]})
    stream_park(c->device, s);
  if (c->pool_err) (void)hipHostFree(c->pool_err);
  delete c;
}

void ovh_destroy(ovh_ctx* c) {
  if (!c) return;
  for (ovh_ctx* s : c->sub) destroy_one(s);
  c->sub.clear();
  destroy_one(c);
}

int ovh_device_count(ovh_ctx* c) { return !c ? 0 : c->sub.empty() ? 1 : (int)c->sub.size(); }

// Diagnostics. prog 0: occupancy A/B of the vsame program -- `reps`
// launches over n votes of zeros (the programs are branch-free: the input values do not change
// the work), all on the main stream (streams = 1) or alternating over the main and the side
// stream (streams = 2: two launches co-resident). prog 1: the vote pool alone -- `reps` batches
// of n zero votes published back to back (staging, hash_to_field, publication; a slot is reused
// once the pool finished its previous batch), no final-stream work; `streams` is ignored.
// *ms = the wall time of the whole sequence (HIP events).
int ovh_diag_vm_occupancy(ovh_ctx* c, int prog, size_t n, int reps, int streams, float* ms) {
  if (!c || !ms || n == 0 || n > (1u << 20) || reps < 1 || streams < 1 || streams > 2 || prog < 0 || prog > 2 ||
      (prog == 2 && reps > OVH_BATCH_SLOTS))
    return OVH_ERR_ARG;
  if (!c->sub.empty()) c = c->sub[0];
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  CHK(ensure_cap(c, n));
  CHK(ensure_in(c, n * 180 + 64));
  CHK(sync_all(c));
  if (!c->xstream) HIPCHK(stream_new(&c->xstream, 0));
  HIPCHK(hipMemsetAsync(c->in_buf, 0, n * 180, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  const Slab s{c->state_slot[0], c->cap};
  int32_t* dc = (int32_t*)(c->in_buf + n * 176);
  const uint32_t N = (uint32_t)n;
  hipEvent_t e0, e1;
  HIPCHK(hipEventCreate(&e0));
  HIPCHK(hipEventCreate(&e1));
  HIPCHK(hipEventRecord(e0, c->stream));
  HIPCHK(hipStreamWaitEvent(c->xstream, e0, 0));
  for (int r = 0; r < reps; ++r) {
    if (prog == 0) {
      hipStream_t st = (streams == 2 && (r & 1)) ? c->xstream : c->stream;
      k_vm_vsame<false><<<(N + VM_SLICES - 1) / VM_SLICES, 64, LDS_VSAME, st>>>(N, 0, c->vm_vsame, c->vm_consts,
                                                                               c->in_buf + n * 128, PkSrc{}, c->in_buf,
                                                                               s, 1, 0, dc);
    } else {
      // prog 2: every batch published before the pool's grids start (one pair, after the last):
      // the pool runs without a gap, so under rocprofv3's serialised dispatches (PMC passes) its
      // counters cover the reps batches and no idle wait for a publication
      const int slot = r % OVH_BATCH_SLOTS;
      k_pool_announce<<<1, 64, 0, c->stream>>>(c->pool_q, c->pool_seq + 1);
      if (r >= OVH_BATCH_SLOTS)
        k_pool_wait<<<1, 64, 0, c->stream>>>(c->pool_q, (uint32_t)slot, (N + VM_SLICES - 1) / VM_SLICES,
                                             pool_wait_ticks(N), c->pool_err);
      CHK(batch_front(c, slot, N, c->in_buf, c->in_buf + n * 96, KeySrc{c->in_buf + n * 128, PkSrc{}}, dc, false,
                      prog == 1 || r == reps - 1));
    }
  }
  HIPCHK(hipGetLastError());
  if (prog >= 1) c->clk_wgs = c->pool_wgs < VM_CLOCK_WGS ? c->pool_wgs : VM_CLOCK_WGS;
  for (hipStream_t p : {c->xstream, c->pool_st[0], c->pool_st[1]}) {
    HIPCHK(hipEventRecord(e1, p));
    HIPCHK(hipStreamWaitEvent(c->stream, e1, 0));
  }
  HIPCHK(hipEventRecord(e1, c->stream));
  HIPCHK(hipEventSynchronize(e1));
  HIPCHK(hipEventElapsedTime(ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return 0;
}

int ovh_vm_trace(ovh_ctx* c, int prog, uint64_t* stamps, size_t max) {
  if (!c || prog < 0 || prog > 3 || (max && !stamps)) return -OVH_ERR_ARG;
  if (!c->sub.empty()) c = c->sub[0];
  if (!(c->flags & OVH_FLAG_VM_TRACE)) return 0;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return -OVH_ERR_DEVICE;
  const VmDev* d = prog == 0 ? &c->vm_vote : prog == 1 ? &c->vm_fold : prog == 2 ? &c->vm_final : &c->vm_vote_t;
  const size_t n = (size_t)d->nphases + 1, k = max < n ? max : n;
  if (sync_all(c) || (k && hipMemcpy(stamps, d->trace, k * 8, hipMemcpyDeviceToHost) != hipSuccess))
    return -OVH_ERR_DEVICE;
  return (int)n;
}

int ovh_vm_clock(ovh_ctx* c, uint64_t* stamps, size_t max) {
  if (!c || (max && !stamps)) return -OVH_ERR_ARG;
  if (!c->sub.empty()) c = c->sub[0];
  if (!(c->flags & OVH_FLAG_VM_CLOCK)) return 0;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess || sync_all(c)) return -OVH_ERR_DEVICE;
  const VmDev* d = c->clk_table ? &c->vm_vote_t : &c->vm_vote;
  const size_t n = (size_t)2 * c->clk_wgs, k = max < n ? max : n;
  if (k && hipMemcpy(stamps, d->clk, k * 8, hipMemcpyDeviceToHost) != hipSuccess) return -OVH_ERR_DEVICE;
  return (int)n;
}

int ovh_pool_log(ovh_ctx* c, uint64_t* words, size_t max) {
  if (!c || (max && !words)) return -OVH_ERR_ARG;
  if (!c->sub.empty()) c = c->sub[0];
  if (!c->plog) return 0;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess || sync_all(c)) return -OVH_ERR_DEVICE;
  const size_t n = PLOG_TOTAL, k = max < n ? max : n;
  if (k && hipMemcpy(words, c->plog, k * 8, hipMemcpyDeviceToHost) != hipSuccess) return -OVH_ERR_DEVICE;
  return (int)n;
}

int ovh_stage_times(ovh_ctx* c, float* ms, size_t max) {
  if (!c || (!ms && max)) return -OVH_ERR_ARG;
  if (!c->sub.empty()) c = c->sub[0];
  if (!(c->flags & OVH_FLAG_PROFILE)) return 0;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess || sync_all(c)) return -OVH_ERR_DEVICE;
  const size_t n = max < OVH_NSTAGES ? max : OVH_NSTAGES;
  for (size_t k = 0; k < n; ++k) {
    ms[k] = 0.f;
    if (c->ev_mask & (1u << k))
      if (hipEventElapsedTime(&ms[k], c->ev0[k], c->ev1[k]) != hipSuccess) return -OVH_ERR_DEVICE;
  }
  return (int)n;
}

int ovh_vote_spans(ovh_ctx* c, float* ms, size_t max) {
  if (!c || (!ms && max)) return -OVH_ERR_ARG;
  if (!c->sub.empty()) c = c->sub[0];
  if (!(c->flags & OVH_FLAG_PROFILE)) return 0;
  std::lock_guard<std::mutex> g(c->mu);
  if (max == 0) {  // reset
    c->vev_n = 0;
    return 0;
  }
  if (hipSetDevice(c->device) != hipSuccess || sync_all(c)) return -OVH_ERR_DEVICE;
  const uint32_t n = c->vev_n < ovh_ctx::VEV_CAP ? c->vev_n : ovh_ctx::VEV_CAP;
  const uint32_t first = c->vev_n - n;  // the oldest kept batch
  size_t k = 0;
  for (uint32_t j = 0; j < n && 2 * k + 1 < max; ++j, ++k) {
    const uint32_t e = (first + j) % ovh_ctx::VEV_CAP, e0 = first % ovh_ctx::VEV_CAP;
    if (hipEventElapsedTime(&ms[2 * k], c->vev0[e0], c->vev0[e]) != hipSuccess ||
        hipEventElapsedTime(&ms[2 * k + 1], c->vev0[e0], c->vev1[e]) != hipSuccess)
      return -OVH_ERR_DEVICE;
  }
  return (int)k;
}

const char* ovh_stage_name(int k) { return (k >= 0 && k < OVH_NSTAGES) ? STAGE_NAMES[k] : nullptr; }

void* ovh_stream(ovh_ctx* c) {
  if (!c) return nullptr;
  if (!c->sub.empty()) c = c->sub[0];
  return (void*)c->stream;
}

int ovh_sm3(const uint8_t* msg, size_t len, uint8_t out[32]) {
  if ((!msg && len) || !out) return OVH_ERR_ARG;
  sm3_digest(msg, len, out);
  return 0;
}

static_assert(OVH_VOTE_HASH_MAX == VOTE_HASH_MAX, "vote hash stride");

int ovh_vote_digests_device(ovh_ctx* c, size_t n, const uint64_t* heights, const uint64_t* rounds,
                            const uint8_t* vote_types, const uint8_t* block_hashes, const uint8_t* hash_lens,
                            uint8_t* digests) {
  if (!c || n > (1u << 24) || (n && (!heights || !rounds || !vote_types || !block_hashes || !hash_lens || !digests)))
    return OVH_ERR_ARG;
  if (n == 0) return 0;
  ovh_ctx* s = c->sub.empty() ? c : c->sub[0];
  std::lock_guard<std::mutex> g(s->mu);
  HIPCHK(hipSetDevice(s->device));
  k_vote_digest<<<nblk(n), WG, 0, s->stream>>>((uint32_t)n, heights, rounds, vote_types, block_hashes, hash_lens,
                                               digests);
  HIPCHK(hipGetLastError());
  return 0;
}

int ovh_vote_digests(ovh_ctx* c, size_t n, const uint64_t* heights, const uint64_t* rounds, const uint8_t* vote_types,
                     const uint8_t* block_hashes, const uint8_t* hash_lens, uint8_t* digests) {
  if (!c || n > (1u << 24) || (n && (!heights || !rounds || !vote_types || !block_hashes || !hash_lens || !digests)))
    return OVH_ERR_ARG;
  if (n == 0) return 0;
  for (size_t i = 0; i < n; ++i)
    if (hash_lens[i] > OVH_VOTE_HASH_MAX) return OVH_ERR_ARG;
  ovh_ctx* s = pick_sub(c);
  std::lock_guard<std::mutex> g(s->mu);
  HIPCHK(hipSetDevice(s->device));
  // staging: heights, rounds (8 B), types, lens (1 B), hashes (64 B), digests (32 B) per vote
  const size_t per = 8 + 8 + 1 + 1 + OVH_VOTE_HASH_MAX + 32;
  CHK(ensure_in(s, n * per + 256));
  uint8_t* d = s->in_buf;
  uint64_t* dh = (uint64_t*)d;
  uint64_t* dr = dh + n;
  uint8_t* dt = (uint8_t*)(dr + n);
  uint8_t* dl = dt + n;
  uint8_t* db = dl + n;
  uint8_t* dd = db + n * OVH_VOTE_HASH_MAX;
  HIPCHK(hipMemcpyAsync(dh, heights, n * 8, hipMemcpyHostToDevice, s->stream));
  HIPCHK(hipMemcpyAsync(dr, rounds, n * 8, hipMemcpyHostToDevice, s->stream));
  HIPCHK(hipMemcpyAsync(dt, vote_types, n, hipMemcpyHostToDevice, s->stream));
  HIPCHK(hipMemcpyAsync(dl, hash_lens, n, hipMemcpyHostToDevice, s->stream));
  HIPCHK(hipMemcpyAsync(db, block_hashes, n * OVH_VOTE_HASH_MAX, hipMemcpyHostToDevice, s->stream));
  k_vote_digest<<<nblk(n), WG, 0, s->stream>>>((uint32_t)n, dh, dr, dt, db, dl, dd);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(digests, dd, n * 32, hipMemcpyDeviceToHost, s->stream));
  HIPCHK(hipStreamSynchronize(s->stream));
  return 0;
}

int ovh_sk_parse(ovh_ctx* c, const uint8_t* key, size_t key_len, uint8_t out_scalar[32]) {
  if (!c || !out_scalar) return OVH_ERR_ARG;
  return sk_parse(c, key, key_len, out_scalar);
}

// Blinding factors for the one-lane compressions of k_vm_pkgen / k_vm_signg (their
// inversion runs variable-time divsteps on a secret-dependent Z): `planes` Fp planes of n
// uniform nonzero elements below p (getrandom, rejection sampling), uploaded on c->stream into
// scr planes first..first + planes - 1. Caller holds c->mu and has sized scr for n; the host
// copy lives in the context until the next call (every caller synchronises before returning).
static int upload_blinds(ovh_ctx* c, size_t n, uint32_t first, uint32_t planes, Slab* out) {
  const size_t cap = c->scr_cap;
  c->blind_h.assign((size_t)planes * 12 * cap, 0u);
  for (size_t i = 0; i < n; ++i)
    for (uint32_t j = 0; j < planes; ++j) {
      uint32_t v[12];
      for (;;) {
        size_t got = 0;
        while (got < sizeof v) {
          const ssize_t r = getrandom((uint8_t*)v + got, sizeof v - got, 0);
          if (r < 0) {
            if (errno == EINTR) continue;
            return OVH_ERR_RNG;
          }
          got += (size_t)r;
        }
        v[11] &= 0x1FFFFFFFu;  // p < 2^381: below 2^381, then reject >= p and 0
        uint32_t z = 0;
        for (int k = 0; k < 12; ++k) z |= v[k];
        if (z && limbs_lt_p(v)) break;
      }
      for (int k = 0; k < 12; ++k) c->blind_h[((size_t)j * 12 + k) * cap + i] = v[k];
    }
  uint32_t* d = c->scr + (size_t)first * 12 * cap;
  HIPCHK(hipMemcpyAsync(d, c->blind_h.data(), c->blind_h.size() * 4, hipMemcpyHostToDevice, c->stream));
  *out = Slab{d, (uint32_t)cap};
  return 0;
}

// n signatures on c->stream: hash_to_field per hash (k_h2f, u planes in scr), then the VM
// (k_vm_sign). Caller holds c->mu and has sized scr for n.
static int enqueue_sign(ovh_ctx* c, size_t n, const uint8_t* d_sks, const uint8_t* d_hashes, uint8_t* d_sigs) {
  Slab u{c->scr, c->scr_cap}, bl;
  static_assert(S_U + 4 <= 6, "u planes below the blinding planes");
  CHK(upload_blinds(c, n, 6, 2, &bl));
  k_h2f<<<nblk(n), WG, 0, c->stream>>>((uint32_t)n, d_hashes, c->xmd, u);
  constexpr uint32_t SL = 64 / VM_SIGNG0_W;
  k_vm_signg<<<(uint32_t)((n + SL - 1) / SL), 64, LDS_SIGNG, c->stream>>>((uint32_t)n, c->vm_signg0, c->vm_signg1,
                                                                          c->vm_consts, d_sks, u, d_sigs, bl);
  HIPCHK(hipGetLastError());
  return 0;
}

int ovh_sign(ovh_ctx* c, const uint8_t* key, size_t key_len, const uint8_t* hash, size_t hash_len, uint8_t out[96]) {
  if (!c || !out) return OVH_ERR_ARG;
  if (hash_len != 32 || !hash) return OVH_ERR_HASH_LEN;
  SecretBytes sk;
  CHK(sk_parse(c, key, key_len, sk.b));
  c = pick_sub(c);
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  CHK(ensure_in(c, 256));
  CHK(ensure_scr(c, 1));
  HIPCHK(hipMemcpyAsync(c->in_buf, sk.b, 32, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->in_buf + 32, hash, 32, hipMemcpyHostToDevice, c->stream));
  CHK(enqueue_sign(c, 1, c->in_buf, c->in_buf + 32, c->in_buf + 64));
  // the scalar does not outlive the call: staging bytes zeroed after the kernel, host copy wiped
  HIPCHK(hipMemsetAsync(c->in_buf, 0, 32, c->stream));
  HIPCHK(hipMemcpyAsync(out, c->in_buf + 64, 96, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int ovh_sk_to_pk(ovh_ctx* c, const uint8_t* key, size_t key_len, uint8_t out[48]) {
  if (!c || !out) return OVH_ERR_ARG;
  SecretBytes sk;
  CHK(sk_parse(c, key, key_len, sk.b));
  c = pick_sub(c);
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  CHK(ensure_in(c, 128));
  CHK(ensure_scr(c, 1));
  Slab bl;
  CHK(upload_blinds(c, 1, 0, 1, &bl));
  HIPCHK(hipMemcpyAsync(c->in_buf, sk.b, 32, hipMemcpyHostToDevice, c->stream));
  k_vm_pkgen<<<1, 64, LDS_PKGEN, c->stream>>>(1, c->vm_pkgen, c->vm_consts, c->in_buf, c->in_buf + 32, bl);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemsetAsync(c->in_buf, 0, 32, c->stream));
  HIPCHK(hipMemcpyAsync(out, c->in_buf + 32, 48, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int ovh_verify(ovh_ctx* c, const uint8_t* sig, size_t sig_len, const uint8_t* hash, size_t hash_len, const uint8_t* pk,
               size_t pk_len) {
  if (!c) return OVH_ERR_ARG;
  if (hash_len != 32 || !hash) return OVH_ERR_HASH_LEN;
  if ((sig_len && !sig) || (pk_len && !pk)) return OVH_ERR_ARG;
  // consensus.rs:406-410 order: an encoding of any other length never parses; an over-long one
  // is passed on as empty, so the kernel answers with the reference's precedence (key first: 102)
  if (pk_len > 4096) pk_len = 0;
  if (sig_len > 4096) sig_len = 0;
  const bool fixed = sig_len == 96 && pk_len == 48;
  int32_t code;
  if (fixed && cache_get(c, sig, hash, pk, &code)) return code;
  ovh_ctx* s = pick_sub(c);
  std::lock_guard<std::mutex> g(s->mu);
  HIPCHK(hipSetDevice(s->device));
  if (fixed) {
    // one standalone vote (vote1 / vote_t1 + final1): the vote's own pairing check; a failed
    // check with a clean parse is VERIFY_FAIL (set by k_vm_final1)
    uint8_t* d;
    size_t t;
    std::vector<uint32_t> perm;
    CHK(stage_split(s, 1, sig, hash, pk, &d, &t, perm));
    int32_t* dc = (int32_t*)(d + 176);
    CHK(verify_one_locked(s, d, d + 96, staged_key(s, 1, d, t, 0), dc, hash));
    int32_t out = -1;
    HIPCHK(hipMemcpyAsync(&out, dc, 4, hipMemcpyDeviceToHost, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    return out;
  }
  // other encodings (uncompressed keys / signatures, other lengths): k_canon_one turns them into
  // one staged compressed vote (sig [0, 96), hash [96, 128), key [128, 176), code at 176; the
  // raw bytes from 256), which takes the fixed-size path above
  CHK(ensure_in(s, 256 + sig_len + pk_len + 64));
  uint8_t* d = s->in_buf;
  uint8_t* raw = d + 256;
  HIPCHK(hipMemcpyAsync(d + 96, hash, 32, hipMemcpyHostToDevice, s->stream));
  if (sig_len) HIPCHK(hipMemcpyAsync(raw, sig, sig_len, hipMemcpyHostToDevice, s->stream));
  if (pk_len) HIPCHK(hipMemcpyAsync(raw + sig_len, pk, pk_len, hipMemcpyHostToDevice, s->stream));
  k_canon_one<<<1, 64, 0, s->stream>>>(raw, (uint32_t)sig_len, raw + sig_len, (uint32_t)pk_len, d, d + 128);
  HIPCHK(hipGetLastError());
  int32_t* dc = (int32_t*)(d + 176);
  CHK(verify_one_locked(s, d, d + 96, KeySrc{d + 128, PkSrc{}}, dc, hash));
  int32_t r = -1;
  HIPCHK(hipMemcpyAsync(&r, dc, 4, hipMemcpyDeviceToHost, s->stream));
  HIPCHK(hipStreamSynchronize(s->stream));
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
  if (need > c->in_cap) return OVH_ERR_ARG;  // callers size the staging buffer first
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

static size_t list_bytes(const size_t* lens, size_t n) {
  size_t t = 0;
  for (size_t i = 0; i < n; ++i) t += lens[i];
  return t;
}

int ovh_aggregate_sigs(ovh_ctx* c, const uint8_t* sigs, const size_t* sig_lens, size_t n_sigs, const uint8_t* pks,
                       const size_t* pk_lens, size_t n_pks, uint8_t out[96]) {
  if (!c || !out) return OVH_ERR_ARG;
  if (n_sigs != n_pks) return OVH_ERR_LEN_MISMATCH;
  const size_t n = n_sigs;
  if (n && (!sig_lens || !pk_lens)) return OVH_ERR_ARG;
  c = pick_sub(c);
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  // the signatures go through the VM (k_vm_sigchk + a padd tree, planes [0, 2n) of scr); a list
  // with other encodings (uncompressed, other lengths) is re-encoded first (k_canon_sig_list:
  // every item as 96 compressed bytes that parse to the same point or fail with the same code)
  bool compressed = true;
  for (size_t i = 0; i < n; ++i) compressed = compressed && sig_lens[i] == 96;
  const size_t canon_bytes = compressed ? 0 : (size_t)104 * n + 64;
  CHK(ensure_scr(c, n > 0 ? 2 * n : 1));
  CHK(ensure_in(c, list_bytes(sig_lens, n) + list_bytes(pk_lens, n) + 512 + 32 * (n + 1) + canon_bytes));
  uint8_t *ds, *dp;
  uint64_t *so, *sl, *po, *pl;
  size_t used1 = 0, used2 = 0;
  CHK(stage_list(c, sigs, sig_lens, n, 0, &ds, &so, &sl, &used1));
  CHK(stage_list(c, pks, pk_lens, n, used1, &dp, &po, &pl, &used2));
  if (n && !compressed) {
    uint8_t* cs = c->in_buf + ((used2 + 15) & ~(size_t)15);
    uint64_t* co = (uint64_t*)(cs + (size_t)96 * n);
    k_canon_sig_list<<<nblk(n), WG, 0, c->stream>>>((uint32_t)n, ds, so, sl, cs, co);
    HIPCHK(hipGetLastError());
    ds = cs;
    so = co;
    used2 = (size_t)((uint8_t*)(co + n) - c->in_buf);
  }
  Slab pts{c->scr, c->scr_cap};
  Slab ppts{c->scr + (size_t)6 * 12 * c->scr_cap, c->scr_cap};
  if (n) {
    // the keys parse on the side stream while the signatures run through the VM
    HIPCHK(hipEventRecord(c->ev_x[2], c->stream));  // staged inputs
    // created on first use: a context that only verifies batches keeps to three streams, which
    // map onto distinct hardware queues at HIP's default of four (GPU_MAX_HW_QUEUES)
    if (!c->xstream) HIPCHK(stream_new(&c->xstream, 0));
    HIPCHK(hipStreamWaitEvent(c->xstream, c->ev_x[2], 0));
    bool keys48 = true;
    for (size_t i = 0; i < n; ++i) keys48 = keys48 && pk_lens[i] == 48;
    if (keys48) {  // compressed keys: the decompression on the VM (r04; was one lane per key)
      constexpr uint32_t KSL = 64 / VM_PKDEC_W;
      k_vm_pkdec<<<(uint32_t)((n + KSL - 1) / KSL), 64, LDS_PKDEC, c->xstream>>>((uint32_t)n, c->vm_pkdec,
                                                                                c->vm_consts, dp, po, c->scr_pk);
    } else {  // other encodings (uncompressed keys: an on-curve check, no square root)
      k_parse_pk_list<<<nblk(n), WG, 0, c->xstream>>>((uint32_t)n, dp, po, pl, c->scr_pk, ppts);
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(c->ev_x[3], c->xstream));
    const int gc = (c->flags & OVH_FLAG_AGG_NO_GROUPCHECK) ? 0 : 1;
    constexpr uint32_t SL = 64 / VM_SIGCHK_W;
    k_vm_sigchk<<<(uint32_t)((n + SL - 1) / SL), 64, LDS_SIGCHK, c->stream>>>((uint32_t)n, c->vm_sigchk, c->vm_consts,
                                                                              ds, so, gc, c->scr_sig, pts);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamWaitEvent(c->stream, c->ev_x[3], 0));
  }
  std::vector<int32_t> cs(n), cp(n);
  if (n) {
    HIPCHK(hipMemcpyAsync(cs.data(), c->scr_sig, 4 * n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(cp.data(), c->scr_pk, 4 * n, hipMemcpyDeviceToHost, c->stream));
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
  {
    constexpr uint32_t SL = 64 / VM_PADD_W;
    uint32_t m = (uint32_t)n, base = 0;
    while (m > 1) {
      const uint32_t half = (m + 1) / 2, dst = base ? 0 : (uint32_t)n;
      k_vm_g2tree<<<(half + SL - 1) / SL, 64, LDS_MSM8, c->stream>>>(m, c->vm_padd, MSM8_STRIDE_W, c->vm_consts,
                                                                     Slab{pts.p + base, pts.cap}, Slab{pts.p + dst, pts.cap});
      m = half;
      base = dst;
    }
    k_g2p_compress<<<1, 64, 0, c->stream>>>(Slab{pts.p + base, pts.cap}, c->in_buf + used2);
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out, c->in_buf + used2, 96, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

// Parses + sums a pk list on the device; the Jacobian sum (36 words) stays at *d_sum (in the
// staging buffer, after `reserve` bytes kept free for the caller). Caller holds c->mu.
static int sum_pks(ovh_ctx* c, const uint8_t* pks, const size_t* pk_lens, size_t n, size_t reserve, uint8_t* out48,
                   uint32_t** d_sum) {
  if (n && !pk_lens) return OVH_ERR_ARG;
  CHK(ensure_scr(c, n > 0 ? n : 1));
  CHK(ensure_in(c, list_bytes(pk_lens, n) + 16 * (n + 1) + 512 + reserve));
  uint8_t* dp;
  uint64_t *po, *pl;
  size_t used = 0;
  CHK(stage_list(c, pks, pk_lens, n, 0, &dp, &po, &pl, &used));
  Slab ppts{c->scr, c->scr_cap};
  if (n) {
    k_parse_pk_list<<<nblk(n), WG, 0, c->stream>>>((uint32_t)n, dp, po, pl, c->scr_pk, ppts);
    HIPCHK(hipGetLastError());
  }
  std::vector<int32_t> cp(n);
  if (n) HIPCHK(hipMemcpyAsync(cp.data(), c->scr_pk, 4 * n, hipMemcpyDeviceToHost, c->stream));
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

// One homogeneous projective G1 point (planes X, Y, Z at index u) -> 48-byte compressed encoding.
__global__ __launch_bounds__(64) void k_g1p_compress(Slab pts, uint32_t u, uint8_t* __restrict__ out) {
  if (threadIdx.x != 0) return;
  Fp X, Y, Z, zz;
  pts.ld(X, 0, u);
  pts.ld(Y, 1, u);
  pts.ld(Z, 2, u);
  G1J j;  // (X : Y : Z) homogeneous = (X Z : Y Z^2 : Z) Jacobian
  fp_mul(j.X, X, Z);
  fp_sqr(zz, Z);
  fp_mul(j.Y, Y, zz);
  j.Z = Z;
  g1_compress(out, j);
}

// BlsPublicKey::aggregate (consensus.rs:371, 441-443) over compressed keys on the VM: every key
// decoded by k_vm_pkchk (a key that does not parse -> "lose public key"; the aggregate, like the
// one-lane path, does not require the subgroup), summed by a g1padd tree, compressed. Returns 1
// when the one-lane path must decide (other encodings, no keys).
static int aggregate_pks_vm(ovh_ctx* c, const uint8_t* pks, const size_t* pk_lens, size_t n, uint8_t* out48) {
  if (n == 0) return 1;
  for (size_t i = 0; i < n; ++i)
    if (pk_lens[i] != 48) return 1;
  if (2 * n > c->qt_cap || !c->qt_buf) {  // keys in [0, n), the tree's levels ping-pong over [0, 2n)
    if (c->qt_buf) (void)hipFree(c->qt_buf);
    c->qt_buf = nullptr;
    c->qt_cap = 0;
    uint32_t cap = 64;
    while (cap < 2 * n) cap <<= 1;
    HIPCHK(hipMalloc(&c->qt_buf, (size_t)(3 * 12 + 1) * cap * 4));
    c->qt_cap = cap;
  }
  CHK(ensure_in(c, n * 48 + 64));
  uint8_t* d = c->in_buf;  // keys | compressed sum
  HIPCHK(hipMemcpyAsync(d, pks, n * 48, hipMemcpyHostToDevice, c->stream));
  uint32_t* kflags = c->qt_buf + (size_t)3 * 12 * c->qt_cap;
  constexpr uint32_t PK_SL = 64 / VM_PKCHK_W;
  k_vm_pkchk<<<(uint32_t)((n + PK_SL - 1) / PK_SL), 64, LDS_PKCHK, c->stream>>>((uint32_t)n, c->vm_pkchk, c->vm_consts, d,
                                                                               Slab{c->qt_buf, c->qt_cap}, kflags);
  HIPCHK(hipGetLastError());
  std::vector<uint32_t> hf(n);
  HIPCHK(hipMemcpyAsync(hf.data(), kflags, n * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  for (size_t i = 0; i < n; ++i)
    if (hf[i] & PKF_PARSE) return OVH_ERR_PUBKEY;
  constexpr uint32_t SL = 64 / VM_G1PADD_W;
  uint32_t m = (uint32_t)n, base = 0;
  while (m > 1) {
    const uint32_t half = (m + 1) / 2, dst = base ? 0 : (uint32_t)n;
    k_vm_g1tree<<<(half + SL - 1) / SL, 64, LDS_G1PADD, c->stream>>>(m, c->vm_g1padd, G1PADD_STRIDE_W, c->vm_consts,
                                                                     Slab{c->qt_buf + base, c->qt_cap},
                                                                     Slab{c->qt_buf + dst, c->qt_cap});
    m = half;
    base = dst;
  }
  uint8_t* o48 = d + ((n * 48 + 15) & ~(size_t)15);
  k_g1p_compress<<<1, 64, 0, c->stream>>>(Slab{c->qt_buf + base, c->qt_cap}, 0, o48);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out48, o48, 48, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int ovh_aggregate_pks(ovh_ctx* c, const uint8_t* pks, const size_t* pk_lens, size_t n, uint8_t out[48]) {
  if (!c || !out || (n && (!pks || !pk_lens))) return OVH_ERR_ARG;
  c = pick_sub(c);
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  const int r = aggregate_pks_vm(c, pks, pk_lens, n, out);
  if (r != 1) return r;
  uint32_t* sum = nullptr;
  return sum_pks(c, pks, pk_lens, n, 0, out, &sum);
}

static int ensure_qc_buf(ovh_ctx* c, size_t nd) {
  if (nd <= c->qc_cap && c->qc_buf) return 0;
  if (c->qc_buf) (void)hipFree(c->qc_buf);
  c->qc_buf = nullptr;
  c->qc_cap = 0;
  uint32_t cap = 64;
  while (cap < nd) cap <<= 1;
  HIPCHK(hipMalloc(&c->qc_buf, (size_t)(3 * 12 + 1) * cap * 4));
  c->qc_cap = cap;
  return 0;
}

// verify_aggregated_signature (consensus.rs:365-382) on the batch kernels: the keys decoded and
// group-checked on the VM (k_vm_pkchk), their sum (a g1padd tree), then the vote_t program and
// the final check for the one (sig, hash, apk). Returns 1 when the exact one-lane path must
// decide instead (a key outside G1: the sum's own group check decides). Other encodings
// (uncompressed, other lengths) are re-encoded first (k_canon_qc, as k_canon_one).
static int verify_aggregated_vm(ovh_ctx* c, const uint8_t* agg_sig, size_t agg_len, const uint8_t* hash,
                                size_t hash_len, const uint8_t* pks, const size_t* pk_lens, size_t n, int* code) {
  if (n == 0 || !hash || hash_len != 32 || agg_len > 4096) return 1;
  bool fixed = agg_len == 96;
  for (size_t i = 0; i < n; ++i) fixed = fixed && pk_lens[i] == 48;
  if (2 * n > c->qt_cap || !c->qt_buf) {  // keys in [0, n), the tree's levels ping-pong over [0, 2n)
    if (c->qt_buf) (void)hipFree(c->qt_buf);
    c->qt_buf = nullptr;
    c->qt_cap = 0;
    uint32_t cap = 64;
    while (cap < 2 * n) cap <<= 1;
    HIPCHK(hipMalloc(&c->qt_buf, (size_t)(3 * 12 + 1) * cap * 4));
    c->qt_cap = cap;
  }
  CHK(ensure_qc_buf(c, 1));
  CHK(ensure_cap(c, 2));
  const size_t raw_base = ((n * 48 + 128 + 15) & ~(size_t)15) + 256;
  CHK(ensure_in(c, fixed ? n * 48 + 96 + 32 + 64 : raw_base + list_bytes(pk_lens, n) + 16 * (n + 1) + agg_len + 64));
  uint8_t* d = c->in_buf;  // keys | sig | hash | code, qcpre flags
  int32_t* dc = (int32_t*)(d + ((n * 48 + 128 + 15) & ~(size_t)15));
  uint32_t* qpf = (uint32_t*)(dc + 1);
  if (fixed) {
    HIPCHK(hipMemcpyAsync(d, pks, n * 48, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(d + n * 48, agg_sig, 96, hipMemcpyHostToDevice, c->stream));
  } else {
    uint8_t* dp;
    uint64_t *po, *pl;
    size_t used = 0;
    CHK(stage_list(c, pks, pk_lens, n, raw_base, &dp, &po, &pl, &used));
    uint8_t* rs = c->in_buf + used;
    if (agg_len) HIPCHK(hipMemcpyAsync(rs, agg_sig, agg_len, hipMemcpyHostToDevice, c->stream));
    k_canon_qc<<<nblk(n + 1), WG, 0, c->stream>>>((uint32_t)n, dp, po, pl, rs, (uint32_t)agg_len, d);
    HIPCHK(hipGetLastError());
  }
  HIPCHK(hipMemcpyAsync(d + n * 48 + 96, hash, 32, hipMemcpyHostToDevice, c->stream));
  // the signature's checks, H(m) and Miller(-G1, sigma) on the side stream, beside the keys
  int slot;
  CHK(take_slot(c, &slot));
  c->last_n = 0;
  Slab s{c->state_slot[slot], c->cap};
  HIPCHK(hipEventRecord(c->ev_x[2], c->stream));  // staged inputs
  if (!c->xstream) HIPCHK(stream_new(&c->xstream, 0));
  HIPCHK(hipStreamWaitEvent(c->xstream, c->ev_x[2], 0));
  k_h2f<<<1, WG, 0, c->xstream>>>(1, d + n * 48 + 96, c->xmd, s);
  k_vm_qcpre<<<1, 64, LDS_QCPRE, c->xstream>>>(c->vm_qcpre, c->vm_consts, d + n * 48, s, qpf);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(c->ev_x[3], c->xstream));
  uint32_t* kflags = c->qt_buf + (size_t)3 * 12 * c->qt_cap;
  constexpr uint32_t PK_SL = 64 / VM_PKCHK_W;
  k_vm_pkchk<<<(uint32_t)((n + PK_SL - 1) / PK_SL), 64, LDS_PKCHK, c->stream>>>((uint32_t)n, c->vm_pkchk, c->vm_consts, d,
                                                                               Slab{c->qt_buf, c->qt_cap}, kflags);
  HIPCHK(hipGetLastError());
  std::vector<uint32_t> hf(n);
  HIPCHK(hipMemcpyAsync(hf.data(), kflags, n * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  uint32_t fl = 0;
  for (size_t i = 0; i < n; ++i) fl |= hf[i];
  // consensus.rs:454-458 order as sum_pks: any unparsable key -> "lose public key"
  if (fl & (PKF_PARSE | PKF_GRP)) HIPCHK(hipStreamSynchronize(c->xstream));  // qcpre's buffers
  if (fl & PKF_PARSE) {
    *code = OVH_ERR_PUBKEY;
    return 0;
  }
  // a key outside G1 (r04: on the VM; was the one-lane k_verify_agg): the sum is group-checked
  // below (k_vm_g1grp), as blst's verify checks the aggregated key
  uint32_t* qflags = c->qc_buf + (size_t)3 * 12 * c->qc_cap;
  {
    constexpr uint32_t SL = 64 / VM_G1PADD_W;
    uint32_t m = (uint32_t)n, base = 0;
    while (m > 1) {
      const uint32_t half = (m + 1) / 2, dst = base ? 0 : (uint32_t)n;
      k_vm_g1tree<<<(half + SL - 1) / SL, 64, LDS_G1PADD, c->stream>>>(m, c->vm_g1padd, G1PADD_STRIDE_W, c->vm_consts,
                                                                       Slab{c->qt_buf + base, c->qt_cap},
                                                                       Slab{c->qt_buf + dst, c->qt_cap});
      m = half;
      base = dst;
    }
    k_apk_finish<<<1, 64, 0, c->stream>>>(Slab{c->qt_buf + base, c->qt_cap}, Slab{c->qc_buf, c->qc_cap}, qflags);
    if (fl & PKF_GRP)
      k_vm_g1grp<<<1, 64, LDS_G1GRP, c->stream>>>(c->vm_g1grp, c->vm_consts, Slab{c->qc_buf, c->qc_cap}, qflags);
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamWaitEvent(c->stream, c->ev_x[3], 0));
  k_vm_qcmil<<<1, 64, LDS_QCMIL, c->stream>>>(c->vm_qcmil, c->vm_consts, PkSrc{c->qc_buf, c->qc_cap, qflags, nullptr}, s,
                                              qpf, dc);
  k_vm_final1<<<1, 64, LDS_FINAL1, c->stream>>>(c->vm_final1, c->vm_consts,
                                                Slab{s.p + (size_t)S_F * 12 * s.cap + 1, s.cap}, dc,
                                                c->result + RES_BATCH + slot);
  HIPCHK(hipEventRecord(c->ev_back[slot], c->stream));
  HIPCHK(hipGetLastError());
  CHK(sync_all(c));
  int32_t r = -1;
  HIPCHK(hipMemcpyAsync(&r, dc, 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  *code = r;
  return 0;
}

static int verify_aggregated_locked(ovh_ctx* c, const uint8_t* agg_sig, size_t agg_len, const uint8_t* hash,
                                    size_t hash_len, const uint8_t* pks, const size_t* pk_lens, size_t n,
                                    bool exact = false) {
  HIPCHK(hipSetDevice(c->device));
  if (!exact) {
    int code = 0;
    const int r = verify_aggregated_vm(c, agg_sig, agg_len, hash, hash_len, pks, pk_lens, n, &code);
    if (r < 0 || r >= OVH_ERR_ARG) return r;
    if (r == 0) return code;
  }
  uint32_t* sum = nullptr;
  CHK(sum_pks(c, pks, pk_lens, n, 1024 + agg_len, nullptr, &sum));
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

int ovh_verify_aggregated(ovh_ctx* c, const uint8_t* agg_sig, size_t agg_len, const uint8_t* hash, size_t hash_len,
                          const uint8_t* pks, const size_t* pk_lens, size_t n) {
  if (!c) return OVH_ERR_ARG;
  if (agg_len > 4096 || (agg_len && !agg_sig)) return OVH_ERR_ARG;
  if (n && !pk_lens) return OVH_ERR_ARG;
  c = pick_sub(c);
  std::lock_guard<std::mutex> g(c->mu);
  return verify_aggregated_locked(c, agg_sig, agg_len, hash, hash_len, pks, pk_lens, n);
}

static int set_validators_locked(ovh_ctx* c, const uint8_t* pks, size_t n) {
  HIPCHK(hipSetDevice(c->device));
  CHK(sync_all(c));
  ValidatorTable& t = c->tab;
  uint32_t cap = 64;
  while (cap < n) cap <<= 1;
  if (cap > t.cap || !t.planes) {
    for (void* p : {(void*)t.planes, (void*)t.flags})
      if (p) (void)hipFree(p);
    t.planes = nullptr;
    t.flags = nullptr;
    t.cap = 0;
    HIPCHK(hipMalloc(&t.planes, (size_t)3 * 12 * cap * 4));
    HIPCHK(hipMalloc(&t.flags, (size_t)cap * 4));
    t.cap = cap;
  }
  t.n = 0;
  t.keys.clear();
  t.index.clear();
  t.sorted.clear();
  t.hflags.assign(n, 0);
  if (n) {
    CHK(ensure_in(c, n * 48 + 64));
    HIPCHK(hipMemcpyAsync(c->in_buf, pks, n * 48, hipMemcpyHostToDevice, c->stream));
    constexpr uint32_t PK_SL = 64 / VM_PKCHK_W;
    k_vm_pkchk<<<(uint32_t)((n + PK_SL - 1) / PK_SL), 64, LDS_PKCHK, c->stream>>>((uint32_t)n, c->vm_pkchk, c->vm_consts,
                                                                                 c->in_buf, Slab{t.planes, t.cap}, t.flags);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(t.hflags.data(), t.flags, n * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
  }
  for (size_t i = 0; i < n; ++i) {
    t.keys.emplace_back((const char*)pks + 48 * i, 48);
    t.index.emplace(t.keys.back(), (uint32_t)i);  // keeps the first of duplicate keys
    t.sorted.push_back((uint32_t)i);
  }
  std::stable_sort(t.sorted.begin(), t.sorted.end(), [&](uint32_t a, uint32_t b) { return t.keys[a] < t.keys[b]; });
  t.n = (uint32_t)n;
  return 0;
}

int ovh_set_validators(ovh_ctx* c, const uint8_t* pks, size_t n) {
  if (!c || (n && !pks) || n > (1u << 20)) return OVH_ERR_ARG;
  if (!c->sub.empty()) {
    for (ovh_ctx* s : c->sub) {
      std::lock_guard<std::mutex> g(s->mu);
      CHK(set_validators_locked(s, pks, n));
    }
    std::lock_guard<std::mutex> g(c->mu);
    c->tab.n = (uint32_t)n;
    c->tab.keys = c->sub[0]->tab.keys;
    c->tab.hflags = c->sub[0]->tab.hflags;
    c->tab.sorted = c->sub[0]->tab.sorted;
    return 0;
  }
  std::lock_guard<std::mutex> g(c->mu);
  return set_validators_locked(c, pks, n);
}

int ovh_verify_batch(ovh_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* hashes, const uint8_t* pks,
                     int32_t* codes) {
  if (!c || (n && (!sigs || !hashes || !pks || !codes))) return OVH_ERR_ARG;
  if (n == 0) return 0;
  if (n > (1u << 24)) return OVH_ERR_ARG;
  if (!c->sub.empty()) return verify_host_multi(c, n, sigs, hashes, pks, codes);
  std::lock_guard<std::mutex> g(c->mu);
  return verify_host_locked(c, n, sigs, hashes, pks, codes);
}

int ovh_prefetch(ovh_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* hashes, const uint8_t* pks) {
  if (!c || (n && (!sigs || !hashes || !pks))) return OVH_ERR_ARG;
  if (n == 0) return 0;
  std::vector<int32_t> codes(n);
  CHK(ovh_verify_batch(c, n, sigs, hashes, pks, codes.data()));
  cache_put(c, n, sigs, hashes, pks, codes.data());
  return 0;
}

int ovh_cache_config(ovh_ctx* c, size_t capacity) {
  if (!c) return OVH_ERR_ARG;
  std::lock_guard<std::mutex> g(c->cache.mu);
  c->cache.cap = capacity;
  while (c->cache.map.size() > capacity && !c->cache.fifo.empty()) {
    c->cache.map.erase(c->cache.fifo.front());
    c->cache.fifo.pop_front();
  }
  return 0;
}

int ovh_cache_stats(ovh_ctx* c, uint64_t stats[3]) {
  if (!c || !stats) return OVH_ERR_ARG;
  std::lock_guard<std::mutex> g(c->cache.mu);
  stats[0] = c->cache.hits;
  stats[1] = c->cache.misses;
  stats[2] = c->cache.map.size();
  return 0;
}

int ovh_samemsg_stats(ovh_ctx* c, uint64_t stats[3]) {
  if (!c || !stats) return OVH_ERR_ARG;
  stats[0] = stats[1] = stats[2] = 0;
  for (ovh_ctx* s : devices_of(c)) {
    std::lock_guard<std::mutex> g(s->mu);
    stats[0] += s->sm_batches;
    stats[1] += s->sm_votes;
    stats[2] += s->sm_hashes;
  }
  return 0;
}

int ovh_msg_cache_stats(ovh_ctx* c, uint64_t stats[2]) {
  if (!c || !stats) return OVH_ERR_ARG;
  stats[0] = stats[1] = 0;
  for (ovh_ctx* s : devices_of(c)) {
    std::lock_guard<std::mutex> g(s->mu);
    stats[0] += s->hc_hits;
    stats[1] += s->hc_misses;
  }
  return 0;
}

static int qc_batch_locked(ovh_ctx* c, size_t nq, const uint8_t* sigs, const uint8_t* hashes, const uint8_t* bitmaps,
                           size_t bitmap_len, int32_t* codes) {
  HIPCHK(hipSetDevice(c->device));
  const ValidatorTable& t = c->tab;
  // voters per QC (extract_voters: bit k MSB-first <-> k-th key in sorted order; zip truncates)
  const size_t nbits = bitmap_len * 8 < t.n ? bitmap_len * 8 : t.n;
  std::vector<uint32_t> off(1, 0), ent;
  std::vector<size_t> dev;  // QCs that go to the device batch
  for (size_t q = 0; q < nq; ++q) {
    const uint8_t* bm = bitmaps + q * bitmap_len;
    uint32_t fl = 0, cnt = 0;
    const size_t start = ent.size();
    for (size_t k = 0; k < nbits; ++k)
      if ((bm[k / 8] >> (7 - k % 8)) & 1) {
        const uint32_t e = t.sorted[k];
        ent.push_back(e);
        fl |= t.hflags[e];
        ++cnt;
      }
    // consensus.rs:454-458 (key parse) -> :371 (empty aggregate) -> ...
    if (fl & PKF_PARSE) {
      codes[q] = OVH_ERR_PUBKEY;
      ent.resize(start);
    } else if (!cnt) {
      codes[q] = BLST_AGGR_TYPE_MISMATCH;
    } else if (fl & PKF_GRP) {
      // a key outside G1: the sum's own group check decides -> the single-QC path (k_vm_g1grp)
      std::vector<uint8_t> cat;
      std::vector<size_t> lens;
      for (size_t k = start; k < ent.size(); ++k) {
        cat.insert(cat.end(), t.keys[ent[k]].begin(), t.keys[ent[k]].end());
        lens.push_back(48);
      }
      ent.resize(start);
      const int r =
          verify_aggregated_locked(c, sigs + 96 * q, 96, hashes + 32 * q, 32, cat.data(), lens.data(), cnt);
      if (r >= OVH_ERR_ARG) return r;
      codes[q] = r;
    } else {
      dev.push_back(q);
      off.push_back((uint32_t)ent.size());
    }
  }
  const size_t nd = dev.size();
  if (!nd) return 0;
  // device batch: apk per QC -> vote_t over (sig, hash, apk)
  CHK(ensure_qc_buf(c, nd));
  const size_t bytes = nd * (96 + 32 + 4) + off.size() * 4 + ent.size() * 4 + 256;
  CHK(ensure_in(c, bytes));
  uint8_t* d = c->in_buf;
  std::vector<uint8_t> hs(nd * 96), hh(nd * 32);
  for (size_t j = 0; j < nd; ++j) {
    memcpy(&hs[96 * j], sigs + 96 * dev[j], 96);
    memcpy(&hh[32 * j], hashes + 32 * dev[j], 32);
  }
  int32_t* dc = (int32_t*)(d + nd * 128);
  uint32_t* doff = (uint32_t*)(dc + nd);
  uint32_t* dent = doff + off.size();
  HIPCHK(hipMemcpyAsync(d, hs.data(), nd * 96, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(d + nd * 96, hh.data(), nd * 32, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(doff, off.data(), off.size() * 4, hipMemcpyHostToDevice, c->stream));
  if (!ent.empty()) HIPCHK(hipMemcpyAsync(dent, ent.data(), ent.size() * 4, hipMemcpyHostToDevice, c->stream));
  uint32_t* qflags = c->qc_buf + (size_t)3 * 12 * c->qc_cap;
  k_qc_apk<<<(uint32_t)nd, 64, 0, c->stream>>>((uint32_t)nd, doff, dent, Slab{t.planes, t.cap},
                                          Slab{c->qc_buf, c->qc_cap}, qflags);
  HIPCHK(hipGetLastError());
  const KeySrc qk{nullptr, PkSrc{c->qc_buf, c->qc_cap, qflags, nullptr}};
  if (nd == 1) CHK(verify_one_locked(c, d, d + 96, qk, dc));
  else CHK(verify_async_locked(c, nd, d, d + nd * 96, qk, dc));
  CHK(sync_all(c));
  std::vector<int32_t> dcodes(nd);
  HIPCHK(hipMemcpyAsync(dcodes.data(), dc, 4 * nd, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  for (size_t j = 0; j < nd; ++j) codes[dev[j]] = dcodes[j];
  return 0;
}

int ovh_verify_qc_batch(ovh_ctx* c, size_t nq, const uint8_t* sigs, const uint8_t* hashes, const uint8_t* bitmaps,
                        size_t bitmap_len, int32_t* codes) {
  if (!c || (nq && (!sigs || !hashes || !codes || (bitmap_len && !bitmaps)))) return OVH_ERR_ARG;
  if (nq == 0) return 0;
  if (nq > (1u << 20)) return OVH_ERR_ARG;
  ovh_ctx* s = c->sub.empty() ? c : c->sub[0];
  std::lock_guard<std::mutex> g(s->mu);
  if (!s->tab.n) return OVH_ERR_ARG;
  return qc_batch_locked(s, nq, sigs, hashes, bitmaps, bitmap_len, codes);
}

int ovh_set_test_rlc(ovh_ctx* c, uint64_t seed, uint64_t index_base) {
  if (!c || !(c->flags & OVH_FLAG_TEST_RLC)) return OVH_ERR_ARG;
  for (ovh_ctx* s : c->sub) {
    std::lock_guard<std::mutex> g(s->mu);
    s->test_seed = seed;
    s->test_base = index_base;
  }
  std::lock_guard<std::mutex> g(c->mu);
  c->test_seed = seed;
  c->test_base = index_base;
  return 0;
}

int ovh_verify_batch_device_async(ovh_ctx* c, size_t n, const uint8_t* d_sigs, const uint8_t* d_hashes,
                                  const uint8_t* d_pks, int32_t* d_codes) {
  if (!c || !c->sub.empty() || (n && (!d_sigs || !d_hashes || !d_pks || !d_codes))) return OVH_ERR_ARG;
  if (n == 0) return 0;
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  return verify_async_locked(c, n, d_sigs, d_hashes, KeySrc{d_pks, PkSrc{}}, d_codes);
}

int ovh_verify_samemsg_device_async(ovh_ctx* c, size_t n, const uint8_t* d_sigs, const uint8_t* hash,
                                    const uint8_t* d_pks, int32_t* d_codes) {
  if (!c || !c->sub.empty() || (n && (!d_sigs || !hash || !d_pks || !d_codes))) return OVH_ERR_ARG;
  if (n == 0) return 0;
  if (n > (1u << 24)) return OVH_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  CHK(ensure_cap(c, n));
  if (n != c->sm1_n) {  // the plan of one group of n votes; batches in flight may read the old one
    CHK(sync_all(c));
    if (c->sm1_plan) (void)hipFree(c->sm1_plan);
    c->sm1_plan = nullptr;
    c->sm1_n = 0;
    SameMsgPlan pl;
    std::vector<uint8_t> one(32 * n, 0);
    samemsg_plan(n, one.data(), {}, pl);
    std::vector<uint32_t> h(n + 1 + pl.pairs.size(), 0);
    std::copy(pl.pairs.begin(), pl.pairs.end(), h.begin() + n + 1);
    HIPCHK(hipMalloc(&c->sm1_plan, h.size() * 4));
    HIPCHK(hipMemcpy(c->sm1_plan, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    if (!c->sm1_hash) HIPCHK(hipMalloc(&c->sm1_hash, 32 * OVH_BATCH_SLOTS));
    c->sm1_lo = pl.level_off;
    c->sm1_n = n;
  }
  int slot;
  CHK(take_slot(c, &slot));
  Hash32 hv;
  memcpy(hv.w, hash, 32);
  const SameMsgDev pd{1, c->sm1_plan, c->sm1_hash + 32 * slot, c->sm1_plan + n, c->sm1_plan + n + 1, &c->sm1_lo};
  return verify_samemsg_locked(c, slot, n, d_sigs, 0, nullptr, d_pks, pd, d_codes, &hv);
}

// every device's lock, root first (the multi-device entry points)
static std::vector<std::unique_lock<std::mutex>> lock_all(ovh_ctx* c) {
  std::vector<std::unique_lock<std::mutex>> locks;
  locks.emplace_back(c->mu);
  for (ovh_ctx* s : c->sub) locks.emplace_back(s->mu);
  return locks;
}

// restores the caller thread's current HIP device when it goes out of scope
struct DeviceGuard {
  int dev = -1;
  DeviceGuard() { (void)hipGetDevice(&dev); }
  ~DeviceGuard() {
    if (dev >= 0) (void)hipSetDevice(dev);
  }
};

int ovh_verify_batch_async(ovh_ctx* c, size_t n, const uint8_t* sigs, const uint8_t* hashes, const uint8_t* pks,
                           int32_t* codes) {
  if (!c || (n && (!sigs || !hashes || !pks || !codes))) return OVH_ERR_ARG;
  if (n == 0) return 0;
  if (n > (1u << 24)) return OVH_ERR_ARG;
  DeviceGuard dg;
  auto locks = lock_all(c);
  if (c->sub.empty()) {
    HIPCHK(hipSetDevice(c->device));
    return submit_host_single(c, n, sigs, hashes, pks, codes);
  }
  return submit_host_multi(c, n, sigs, hashes, pks, codes);
}

int ovh_batch_wait(ovh_ctx* c) {
  if (!c) return OVH_ERR_ARG;
  DeviceGuard dg;
  auto locks = lock_all(c);
  CHK(drain_host(c));
  for (ovh_ctx* s : devices_of(c)) {
    HIPCHK(hipSetDevice(s->device));
    CHK(sync_all(s));
  }
  return 0;
}

int ovh_verify_batch_device(ovh_ctx* c, size_t n, const uint8_t* d_sigs, const uint8_t* d_hashes, const uint8_t* d_pks,
                            int32_t* d_codes) {
  if (!c || !c->sub.empty() || (n && (!d_sigs || !d_hashes || !d_pks || !d_codes))) return OVH_ERR_ARG;
  if (n == 0) return 0;
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  CHK(verify_async_locked(c, n, d_sigs, d_hashes, KeySrc{d_pks, PkSrc{}}, d_codes));
  return sync_all(c);
}

int ovh_batch_partial_device(ovh_ctx* c, size_t n, const uint8_t* d_sigs, const uint8_t* d_hashes, const uint8_t* d_pks,
                             int32_t* d_codes, uint8_t* d_partial, void* stream) {
  if (!c || !c->sub.empty() || !d_codes || !d_partial || (n && (!d_sigs || !d_hashes || !d_pks))) return OVH_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  if (n == 0) {
    // neutral partial: F = 1, S = O = (0 : 1 : 0)
    static uint32_t neutral[216];
    for (int k = 0; k < 12; ++k) neutral[k] = ONE_M[k];
    for (int k = 0; k < 12; ++k) neutral[144 + 24 + k] = ONE_M[k];  // Y.c0 = 1
    if (st) {
      HIPCHK(hipEventRecord(c->ev_x[0], st));
      HIPCHK(hipStreamWaitEvent(c->stream, c->ev_x[0], 0));
    }
    HIPCHK(hipMemcpyAsync(d_partial, neutral, 864, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->last_n = 0;
    return 0;
  }
  CHK(ensure_cap(c, n));
  int slot;
  CHK(pool_take_slot(c, &slot));
  if (!st) {
    CHK(batch_front(c, slot, (uint32_t)n, d_sigs, d_hashes, KeySrc{d_pks, PkSrc{}}, d_codes));
    CHK(shard_partial(c, slot, (uint32_t)n, d_codes, (uint32_t*)d_partial, nullptr));
    HIPCHK(hipStreamSynchronize(c->stream));
    return pool_failed(c);  // (the partial of a timed-out pool wait is stale)
  }
  // pipelined: only the staging, hash_to_field and the publication on the main stream (the votes
  // in the pool); the fold levels, the MSM and the packing on the slot's final stream, which the
  // caller's stream then waits for (its all-gather, then ovh_combine_partials_device_async). The
  // inputs are read in ovh_stream order (include/ovhip.h): waiting on `stream` here would also
  // wait for the previous batch's gather and combine queued there and serialise the pipeline
  // (r03b: 1,062k -> 796k verifs/s at one rank).
  CHK(batch_front(c, slot, (uint32_t)n, d_sigs, d_hashes, KeySrc{d_pks, PkSrc{}}, d_codes, false, true, true));
  hipStream_t fst = c->fs[slot];
  int reg;
  uint32_t m;
  CHK(side_front(c, slot, 1, &reg, &m));
  plog_stamp(c, slot, PLOG_EV_FOLD, fst);
  CHK(enqueue_msm(c, fst, slot, (uint32_t)n, d_codes));
  plog_stamp(c, slot, PLOG_EV_MSM, fst);
  HIPCHK(hipEventRecord(c->ev_x[0], st));  // the caller's earlier work (a gather out of d_partial)
  HIPCHK(hipStreamWaitEvent(fst, c->ev_x[0], 0));
  k_pack_partial2<<<1, 64, 0, fst>>>(region_F(c, slot, reg), msm_S(c, slot), (uint32_t*)d_partial);
  plog_stamp(c, slot, PLOG_EV_FINAL, fst);  // (here: the packed partial)
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(c->ev_x[1], fst));
  HIPCHK(hipStreamWaitEvent(st, c->ev_x[1], 0));
  HIPCHK(hipEventRecord(c->ev_back[slot], fst));  // (ovh_batch_fallback_device waits for it)
  return 0;
}

// AoS partials (k <= 16) -> <= 4 partials as planes in `scratch` (unpack, and one fold level
// when k > 4), on stream st.
static int stage_partials(ovh_ctx* c, hipStream_t st, size_t k, const uint8_t* d_partials, uint32_t* scratch, Slab* F,
                          Slab* S, uint32_t* m) {
  Slab uF{scratch, 16}, uS{scratch + (size_t)12 * 12 * 16, 16};
  k_unpack_partials<<<(uint32_t)((k * PART_PLANES + 63) / 64), 64, 0, st>>>((uint32_t)k, (const uint32_t*)d_partials,
                                                                           uF, uS);
  if (k <= 4) {
    *F = uF;
    *S = uS;
    *m = (uint32_t)k;
  } else {
    uint32_t* o = scratch + (size_t)PART_PLANES * 12 * 16;
    *F = Slab{o, 4};
    *S = Slab{o + (size_t)12 * 12 * 4, 4};
    k_vm_fold<VM_FOLD_UNITS><<<1, 64, LDS_FOLD, st>>>((uint32_t)k, c->vm_fold, c->vm_consts, uF, uS, *F, nullptr);
    *m = (uint32_t)((k + 3) / 4);
  }
  return hipGetLastError() == hipSuccess ? 0 : OVH_ERR_DEVICE;
}

int ovh_combine_partials_device(ovh_ctx* c, size_t k, const uint8_t* d_partials, int32_t* verdict) {
  if (!c || !c->sub.empty() || !d_partials || !verdict || k == 0 || k > 4096) return OVH_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  // own scratch (never the batch slots): U = k partials, then two ping-pong regions of k / 4
  const uint32_t kc = (uint32_t)((k + 15) & ~(size_t)15);
  if (kc > c->comb_cap || !c->comb) {
    HIPCHK(hipStreamSynchronize(c->stream));
    if (c->comb) (void)hipFree(c->comb);
    c->comb = nullptr;
    c->comb_cap = 0;
    HIPCHK(hipMalloc(&c->comb, (size_t)3 * PART_PLANES * 12 * kc * 4));
    c->comb_cap = kc;
  }
  auto regF = [&](int r) { return Slab{c->comb + (size_t)r * PART_PLANES * 12 * c->comb_cap, c->comb_cap}; };
  auto regS = [&](int r) {
    return Slab{c->comb + (size_t)r * PART_PLANES * 12 * c->comb_cap + (size_t)12 * 12 * c->comb_cap, c->comb_cap};
  };
  k_unpack_partials<<<(uint32_t)((k * PART_PLANES + 63) / 64), 64, 0, c->stream>>>((uint32_t)k,
                                                                                   (const uint32_t*)d_partials, regF(0),
                                                                                   regS(0));
  uint32_t m = (uint32_t)k;
  int reg = 0;
  while (m > 4) {
    const uint32_t mo = (m + 3) / 4;
    const int ro = reg == 1 ? 2 : 1;
    k_vm_fold<VM_FOLD_UNITS><<<(mo + VM_FOLD_UNITS - 1) / VM_FOLD_UNITS, 64, LDS_FOLD, c->stream>>>(
        m, c->vm_fold, c->vm_consts, regF(reg), regS(reg), regF(ro), nullptr);
    reg = ro;
    m = mo;
  }
  enqueue_final(c, c->stream, regF(reg), regS(reg), m, c->result + RES_SYNC);
  HIPCHK(hipGetLastError());
  int32_t r = -1;
  HIPCHK(hipMemcpyAsync(&r, c->result + RES_SYNC, 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  *verdict = 0;
  CHK(pool_failed(c));  // partials of this context's timed-out batch may be among the inputs
  *verdict = r == 1 ? 1 : 0;
  return 0;
}

int ovh_batch_fallback_device(ovh_ctx* c, size_t n, int32_t* d_codes) {
  if (!c || !c->sub.empty() || !d_codes) return OVH_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  if (n == 0) return 0;
  if (n != c->last_n || c->slot_n[c->last_slot] != n) return OVH_ERR_ARG;
  HIPCHK(hipStreamWaitEvent(c->stream, c->ev_back[c->last_slot], 0));  // the slot's final-stream work
  enqueue_bisect(c, c->stream, c->last_slot, (uint32_t)n, d_codes, nullptr);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(c->stream));
  return pool_failed(c);
}

int ovh_combine_partials_device_async(ovh_ctx* c, size_t k, const uint8_t* d_partials, size_t n, int32_t* d_codes,
                                      void* stream) {
  if (!c || !c->sub.empty() || !d_partials || k == 0 || k > 16 || (n && !d_codes)) return OVH_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  if (n != c->last_n || (n && c->slot_n[c->last_slot] != n)) return OVH_ERR_ARG;
  const int slot = c->last_slot;
  hipStream_t st = (hipStream_t)stream, fst = c->fs[slot];
  if (st) {  // the partials are complete in `st` order (after the caller's all-gather)
    plog_stamp(c, slot, PLOG_EV_GATH, st);
    HIPCHK(hipEventRecord(c->ev_x[2], st));
    HIPCHK(hipStreamWaitEvent(fst, c->ev_x[2], 0));
  }
  uint32_t* scratch = c->fin + (size_t)slot * FIN_STRIDE;
  Slab F, S;
  uint32_t m;
  CHK(stage_partials(c, fst, k, d_partials, scratch, &F, &S, &m));
  plog_stamp(c, slot, PLOG_EV_COMB, fst);
  if (st) {  // the caller may reuse d_partials once they were read
    HIPCHK(hipEventRecord(c->ev_x[3], fst));
    HIPCHK(hipStreamWaitEvent(st, c->ev_x[3], 0));
  }
  int32_t* verdict = c->result + RES_COMBINE + slot;
  enqueue_final(c, fst, F, S, m, verdict);
  plog_stamp(c, slot, PLOG_EV_FE, fst);
  if (n) enqueue_bisect(c, fst, slot, (uint32_t)n, d_codes, verdict);
  plog_stamp(c, slot, PLOG_EV_BACK, fst);
  HIPCHK(hipEventRecord(c->ev_back[slot], fst));
  HIPCHK(hipGetLastError());
  return 0;
}

int ovh_sign_batch_device(ovh_ctx* c, size_t n, const uint8_t* d_sks, const uint8_t* d_hashes, uint8_t* d_sigs) {
  if (!c || !c->sub.empty() || (n && (!d_sks || !d_hashes || !d_sigs))) return OVH_ERR_ARG;
  if (n == 0) return 0;
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  CHK(ensure_scr(c, n));
  CHK(enqueue_sign(c, n, d_sks, d_hashes, d_sigs));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int ovh_sk_to_pk_batch_device(ovh_ctx* c, size_t n, const uint8_t* d_sks, uint8_t* d_pks) {
  if (!c || !c->sub.empty() || (n && (!d_sks || !d_pks))) return OVH_ERR_ARG;
  if (n == 0) return 0;
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  CHK(ensure_scr(c, n));
  Slab bl;
  CHK(upload_blinds(c, n, 0, 1, &bl));
  constexpr uint32_t SL = 64 / VM_PKGEN_W;
  k_vm_pkgen<<<(uint32_t)((n + SL - 1) / SL), 64, LDS_PKGEN, c->stream>>>((uint32_t)n, c->vm_pkgen, c->vm_consts, d_sks,
                                                                        d_pks, bl);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

}  // extern "C"
