// Pippenger MSM of the batch's sum r_i sigma_i in G2 (north_star: "Pippenger MSM for
// random-linear-combination batch verification, with buckets staged in LDS"; SURVEY.md
// Appendix C "sum r_i sigma_i G2 Pippenger share"). Included by ovhip.hip after the VM kernels.
//
// Scalars: the vote's 64-bit RLC value (a, b) stands for r = a + b lambda (lambda = -x^2), so
// r sigma = [a] sigma + [b] tau with tau = -psi^2(sigma) (the vote program stores both, affine).
// That is 2n points with 32-bit scalars, cut into four unsigned 8-bit windows: point p, window w,
// digit d = byte w of its scalar lands in bucket w * 255 + d - 1 (d = 0: nothing).
//
//   k_msm_count    lane per vote: bucket histogram in LDS, then one global add per bucket
//   k_msm_scan     one wave: bucket offsets, and per tree level the prefix of the bucket's
//                  pair counts (the level kernels' work lists)
//   k_msm_scatter  lane per vote: point ids into their bucket's range (counting sort)
//   k_msm_pair     the VM pair kernels (8- or 16-lane slices, Fp-VM slots in LDS hold the
//                  bucket accumulators): bucket tree level 0 (madd, affine points), levels >= 1
//                  (padd, in place), bit-plane sums T_t = sum of the buckets whose digit has bit
//                  t % 8 set, window combination sum_t 2^t T_t (hdbl<m>: A + [2^m] B)
// Buckets are summed as trees over the sorted entries (entry k of bucket b absorbs k + 2^l at
// level l), so a bucket of c points needs ceil(log2 c) levels and no sequential chain; the
// host launches the worst case's levels and the device exits the empty ones.
#pragma once

#define MSM_NBW 255                 // buckets per window (digits 1..255)
#define MSM_NB (4 * MSM_NBW)        // buckets
#define MSM_NT 32                   // bit-plane targets: window w, bit k -> t = 8 w + k
#define MSM_TM 64                   // pairs of a target's level-0 sum (128 member buckets)
#define MSM_LV 27                   // bucket tree levels (2^26 >= 2 x 2^24 points in one bucket)
#define MSM_U (MSM_NT * MSM_TM)     // U plane entries

struct MsmArgs {
  const uint32_t* cnt;  // NB: points per bucket
  const uint32_t* off;  // NB + 1: first sorted entry of each bucket
  const uint32_t* pf;   // MSM_LV x (NB + 1): prefix of the per-bucket pair counts per level
  const uint32_t* ent;  // sorted entries: point id 2 i + h (h = 1: tau of vote i)
  Slab st;              // vote state (sigma / tau planes)
  Slab A;               // bucket trees: entry k of bucket b (k even) at pf[0][b] + k / 2
  Slab U;               // bit-plane sums and window combination; U[0] = sum r_i sigma_i
};

__device__ __forceinline__ uint32_t msm_half(uint64_t r, uint32_t h) { return h ? (uint32_t)(r >> 32) : (uint32_t)r; }

// One-wave workgroups: beside two co-resident vote grids (two waves per SIMD everywhere) a
// workgroup of four or sixteen waves waits until that many slots free up on one CU -- r04w trace:
// the 256-thread count kernel averaged 0.59 ms and peaked at 8.7 ms there, holding up the final.
#define MSM_TPB 64

__global__ __launch_bounds__(MSM_TPB) void k_msm_zero(uint32_t* __restrict__ cnt) {
  const uint32_t k = blockIdx.x * MSM_TPB + threadIdx.x;
  if (k < MSM_NB) cnt[k] = 0;
}

__global__ __launch_bounds__(MSM_TPB) void k_msm_count(uint32_t n, uint64_t seed, uint64_t base,
                                                       const int32_t* __restrict__ codes, uint32_t* __restrict__ cnt) {
  __shared__ uint32_t h[MSM_NB];
  for (uint32_t k = threadIdx.x; k < MSM_NB; k += MSM_TPB) h[k] = 0;
  __syncthreads();
  const uint32_t i = blockIdx.x * MSM_TPB + threadIdx.x;
  if (i < n && codes[i] == 0) {  // failed votes contribute the identity
    const uint64_t r = vote_scalar(seed, base, i);
    for (uint32_t hh = 0; hh < 2; ++hh) {
      const uint32_t s = msm_half(r, hh);
      for (uint32_t w = 0; w < 4; ++w) {
        const uint32_t d = (s >> (8 * w)) & 255u;
        if (d) atomicAdd(&h[w * MSM_NBW + d - 1], 1u);
      }
    }
  }
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < MSM_NB; k += MSM_TPB)
    if (h[k]) atomicAdd(&cnt[k], h[k]);
}

// Exclusive prefix over the MSM_NB values v(b) of one wave: lane t owns the 16 consecutive
// entries 16 t .. 16 t + 15 (MSM_NB <= 1024), scans them serially, and the lanes' sums are
// scanned across the wave (shuffles). out(b) = the prefix; returns the total (every lane).
template <class F, class G>
__device__ __forceinline__ uint32_t wave_scan_nb(F v, G out) {
  static_assert(MSM_NB <= 16 * 64, "16 entries per lane");
  const uint32_t t = threadIdx.x;
  uint32_t loc[16], sum = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint32_t b = 16 * t + j;
    loc[j] = b < MSM_NB ? v(b) : 0u;
    sum += loc[j];
  }
  uint32_t incl = sum;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t x = __shfl_up(incl, d, 64);
    if (t >= (uint32_t)d) incl += x;
  }
  uint32_t run = incl - sum;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint32_t b = 16 * t + j;
    if (b < MSM_NB) out(b, run);
    run += loc[j];
  }
  return __shfl(incl, 63, 64);
}

__global__ __launch_bounds__(64) void k_msm_scan(uint32_t nlev, const uint32_t* __restrict__ cnt,
                                                 uint32_t* __restrict__ off, uint32_t* __restrict__ cur,
                                                 uint32_t* __restrict__ pf) {
  const uint32_t tot = wave_scan_nb([&](uint32_t b) { return cnt[b]; },
                                    [&](uint32_t b, uint32_t e) {
                                      off[b] = e;
                                      cur[b] = e;
                                    });
  if (threadIdx.x == 0) off[MSM_NB] = tot;
  for (uint32_t lv = 0; lv < nlev; ++lv) {
    // level 0: every even entry (its pair, or alone at a bucket's odd end); level l: entries
    // k = j 2^(l+1) whose partner k + 2^l exists
    const uint32_t h = 1u << lv;
    uint32_t* p = pf + (size_t)lv * (MSM_NB + 1);
    const uint32_t t = wave_scan_nb(
        [&](uint32_t b) {
          const uint32_t c = cnt[b];
          return lv == 0 ? (c + 1) / 2 : (c > h ? (c - h + 2 * h - 1) >> (lv + 1) : 0u);
        },
        [&](uint32_t b, uint32_t e) { p[b] = e; });
    if (threadIdx.x == 0) p[MSM_NB] = t;
  }
}

__global__ __launch_bounds__(MSM_TPB) void k_msm_scatter(uint32_t n, uint64_t seed, uint64_t base,
                                                         const int32_t* __restrict__ codes, uint32_t* __restrict__ cur,
                                                         uint32_t* __restrict__ ent) {
  const uint32_t i = blockIdx.x * MSM_TPB + threadIdx.x;
  if (i >= n || codes[i] != 0) return;
  const uint64_t r = vote_scalar(seed, base, i);
  for (uint32_t hh = 0; hh < 2; ++hh) {
    const uint32_t s = msm_half(r, hh);
    for (uint32_t w = 0; w < 4; ++w) {
      const uint32_t d = (s >> (8 * w)) & 255u;
      if (d) ent[atomicAdd(&cur[w * MSM_NBW + d - 1], 1u)] = 2 * i + hh;
    }
  }
}

// single-vote batch (UNIT_BASE): S = sigma (affine -> (x : y : 1)), or O if the vote failed
__global__ __launch_bounds__(64) void k_sig_as_S(Slab st, const int32_t* __restrict__ codes, Slab U) {
  const uint32_t c = threadIdx.x;
  if (c >= 6) return;
  Fp v;
  const bool ok = codes[0] == 0;
  if (ok && c < 4) st.ld(v, S_SIG + c, 0);
  else if (c == (ok ? 4u : 2u)) fp_one(v);
  else fp_zero(v);
  U.st(v, c, 0);
}

enum : uint32_t { MSM_L0 = 0, MSM_LVL = 1, MSM_T0 = 2, MSM_TL = 3, MSM_HRN = 4 };
// operand source: identity, a vote's sigma / tau (affine, staged with Z = 1), A or U entry
enum : uint32_t { SRC_ID = 0, SRC_PT = 1, SRC_A = 2, SRC_U = 3 };

// bucket b with (pf[b] <= q < pf[b + 1]) in one level's prefix row (nondecreasing, pf[0] = 0)
__device__ __forceinline__ uint32_t msm_find(const uint32_t* __restrict__ row, uint32_t q) {
  uint32_t lo = 0, hi = MSM_NB;  // row[lo] <= q < row[hi]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (row[mid] <= q) lo = mid;
    else hi = mid;
  }
  return lo;
}

// the j-th digit value (1..255) with bit k set (128 of them)
__device__ __forceinline__ uint32_t msm_member(uint32_t j, uint32_t k) {
  return ((j >> k) << (k + 1)) | (1u << k) | (j & ((1u << k) - 1));
}

// coordinate c (0..5, projective X0 X1 Y0 Y1 Z0 Z1) of an operand
__device__ __forceinline__ void msm_coord(Fp& v, const MsmArgs& a, uint32_t kind, uint32_t idx, uint32_t c) {
  if (kind == SRC_PT) {
    if (c < 4) a.st.ld(v, ((idx & 1) ? S_TAU : S_SIG) + c, idx >> 1);
    else if (c == 4) fp_one(v);
    else fp_zero(v);
  } else if (kind == SRC_A) {
    a.A.ld(v, c, idx);
  } else if (kind == SRC_U) {
    a.U.ld(v, c, idx);
  } else if (c == 2) {
    fp_one(v);  // (0 : 1 : 0)
  } else {
    fp_zero(v);
  }
}

// One pair add per W-lane slice: dst = A + B (madd / padd) or A + [2^m] B (hdbl<m>).
// lv: the tree level (MSM_LVL, MSM_TL) or the combination level h = 1..5 (MSM_HRN).
template <int W, int MODE>
__global__ __launch_bounds__(64) void k_msm_pair(uint32_t lv, VmDev prog, uint32_t nin, uint32_t stride_w,
                                                 const uint32_t* __restrict__ cst_g, MsmArgs a) {
  constexpr uint32_t SL = 64 / W;
  const uint32_t* row = a.pf + (size_t)(MODE == MSM_L0 ? 0 : lv) * (MSM_NB + 1);
  const uint32_t total = MODE == MSM_L0 || MODE == MSM_LVL ? row[MSM_NB]
                         : MODE == MSM_T0                  ? MSM_U
                         : MODE == MSM_TL                  ? MSM_NT * (MSM_TM >> lv)
                                                           : (MSM_NT >> lv);
  if (blockIdx.x * SL >= total) return;  // whole workgroup idle (empty upper tree levels)
  // above the pool's waves (2), as k_vm_final: the MSM levels are the final stream's longest
  // stretch beside the pool (r05y pool log: 1.7-2.9 ms against 0.67 alone). r05q: at 2 (with the
  // final at 3) 1,432k verifs/s vs 1,131k-1,316k at 0; r05z: at 3, 1,389k-1,407k vs 1,378k-1,386k
  __builtin_amdgcn_s_setprio(3);
  extern __shared__ uint4 lds4[];
  uint32_t* lds = reinterpret_cast<uint32_t*>(lds4);
  uint32_t* cst = lds;
  const uint32_t slice = threadIdx.x / W, lane = threadIdx.x % W;
  uint32_t* slots = lds + SLOT_BASE_W + slice * stride_w;
  const uint32_t q = blockIdx.x * SL + slice;
  const bool active = q < total;
  load_consts(cst, cst_g, VM_NCONST);
  uint32_t ka = SRC_ID, ia = 0, kb = SRC_ID, ib = 0, kd = SRC_A, id = 0;
  if (active) {
    if (MODE == MSM_L0 || MODE == MSM_LVL) {
      const uint32_t b = msm_find(row, q), j = q - row[b];
      const uint32_t a0 = a.pf[b];  // A index of the bucket's entry 0
      if (MODE == MSM_L0) {
        const uint32_t k = 2 * j, e = a.off[b] + k;
        ka = SRC_PT, ia = a.ent[e];
        if (k + 1 < a.cnt[b]) kb = SRC_PT, ib = a.ent[e + 1];
        id = a0 + j;
      } else {
        const uint32_t k = j << (lv + 1);
        ka = SRC_A, ia = a0 + (k >> 1);
        kb = SRC_A, ib = a0 + ((k + (1u << lv)) >> 1);
        id = ia;
      }
    } else if (MODE == MSM_T0) {
      const uint32_t t = q / MSM_TM, i = q % MSM_TM, w = t >> 3, k = t & 7;
      const uint32_t b0 = w * MSM_NBW + msm_member(2 * i, k) - 1, b1 = w * MSM_NBW + msm_member(2 * i + 1, k) - 1;
      if (a.cnt[b0]) ka = SRC_A, ia = a.pf[b0];
      if (a.cnt[b1]) kb = SRC_A, ib = a.pf[b1];
      kd = SRC_U, id = q;
    } else if (MODE == MSM_TL) {
      const uint32_t per = MSM_TM >> lv, t = q / per, i = q % per, e = t * MSM_TM + (i << lv);
      ka = SRC_U, ia = e;
      kb = SRC_U, ib = e + (1u << (lv - 1));
      kd = SRC_U, id = e;
    } else {  // window combination level h = lv: U[2 m i] + [2^m] U[2 m i + m] (targets), m = 2^(h-1)
      const uint32_t m = 1u << (lv - 1), e = 2 * m * q * MSM_TM;
      ka = SRC_U, ia = e;
      kb = SRC_U, ib = e + m * MSM_TM;
      kd = SRC_U, id = e;
    }
    // stage the operands: madd takes A affine (4 inputs) then B; the others A, B projective
    const uint32_t na = nin - 6;
    for (uint32_t k = lane; k < nin; k += W) {
      Fp v;
      if (k < na) msm_coord(v, a, ka, ia, k);
      else msm_coord(v, a, kb, ib, k - na);
      slot_put(slots, prog.in[k], v.v);
    }
  }
  __syncthreads();
  vm::run(prog.code, prog.nphases, W, lane, active, slots, cst, 0, vm::Out{nullptr, 0, 0});
  if (active) {
    const Slab& d = kd == SRC_U ? a.U : a.A;
    for (uint32_t k = lane; k < 6; k += W) {
      Fp v;
      const uint32_t src = prog.out[k];
      for (int l = 0; l < 12; ++l) v.v[l] = slots[src * 12 + l];
      vm::canon(v, v);
      d.st(v, k, id);
    }
  }
}
