// libovhip: HIP (gfx950) implementation of the C ABI in include/ovhip.h.
//
// Batch verification data path (ovh_verify_batch_device), one lane per unit of work:
//   k_parse_pk   vote i : pk decompress + G1 subgroup check        (consensus.rs:406)
//   k_parse_sig  vote i : sig decompress + G2 subgroup check       (consensus.rs:409)
//   k_codes      vote i : reference error precedence -> codes[i]
//   k_h2f        vote i : expand_message_xmd + hash_to_field       (verify -> hash_to_G2)
//   k_sswu       (vote, j) for j in {0,1}: SSWU + 3-isogeny
//   k_h2c_fin    vote i : Q0 + Q1, clear cofactor, affine H_i
//   k_scalar     vote i : r_i pk_i (affine), r_i sig_i (Jacobian), r_i from (seed, i)
//   k_miller     vote i : f_i = Miller(r_i pk_i, H_i)
//   k_reduce_*   chunked product of f_i / sum of r_i sig_i
//   k_final      prod f_i * Miller(-G1, sum r_i sig_i) -> final exponentiation == 1 ?
//   k_fallback   vote i : full per-vote pairing check when the combined check fails
// Per-vote state lives in HBM as structure-of-arrays by limb: limb k of element i of an Fp
// slab at slab[k * cap + i], so a wave's loads/stores are coalesced 256-byte lines.
#include <hip/hip_runtime.h>

#include <mutex>
#include <new>
#include <string.h>
#include <vector>

#include "../../include/ovhip.h"
#include "bls/verify.hpp"
#include "sm3.hpp"

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

// Number of Fp slabs per vote region.
enum : uint32_t {
  S_PK = 0,     // 2 Fp: pk affine
  S_RP = 2,     // 2 Fp: r * pk affine
  S_SIG = 4,    // 4 Fp: sig affine
  S_U = 8,      // 4 Fp: u0, u1
  S_Q0 = 12,    // 6 Fp: SSWU/iso output 0 (Jacobian)
  S_Q1 = 18,    // 6 Fp
  S_H = 24,     // 4 Fp: H(m) affine
  S_RS = 28,    // 6 Fp: r * sig (Jacobian)
  S_F = 34,     // 12 Fp: Miller output
  S_TOTAL = 46,
};

enum : int {
  ST_PARSE_PK = 0, ST_PARSE_SIG, ST_CODES, ST_H2F, ST_SSWU, ST_H2C_FIN,
  ST_SCALAR, ST_MILLER, ST_REDUCE, ST_FINAL, ST_FALLBACK,
};
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
__global__ __launch_bounds__(WG) void k_parse_pk(uint32_t n, const uint8_t* __restrict__ pks, int32_t* __restrict__ st,
                                                 Slab s) {
  const uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  G1A a;
  bool inf;
  int e = g1_from_bytes(a, inf, pks + (size_t)i * 48, 48);
  int code = 0;
  if (e != BLST_SUCCESS) {
    code = OVH_ERR_PUBKEY;
  } else if (inf) {
    code = BLST_PK_IS_INFINITY;
  } else {
    G1J j;
    jac_from_aff(j, a);
    if (!g1_in_subgroup(j)) code = BLST_POINT_NOT_IN_GROUP;
  }
  if (code == 0 || code == BLST_POINT_NOT_IN_GROUP) s.st_g1a(a, i);
  st[i] = code;
}

#define SIG_INF_MARK 1000
__global__ __launch_bounds__(WG) void k_parse_sig(uint32_t n, const uint8_t* __restrict__ sigs, int32_t* __restrict__ st,
                                                  Slab s) {
  const uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  G2A a;
  bool inf;
  int code = g2_from_bytes(a, inf, sigs + (size_t)i * 96, 96);
  if (code == BLST_SUCCESS) {
    if (inf) {
      code = SIG_INF_MARK;
    } else {
      G2J j;
      jac_from_aff(j, a);
      if (!g2_in_subgroup(j)) code = BLST_POINT_NOT_IN_GROUP;
      s.st_g2a(a, i);
    }
  }
  st[i] = code;
}

// verify_signature precedence: pk parse (102) > sig parse (1..3) > sig group (3) >
// pk infinity (6) > pk group (3) > [infinite sig -> pairing fails: 5] > pairing.
__global__ __launch_bounds__(WG) void k_codes(uint32_t n, const int32_t* __restrict__ pk_st,
                                              const int32_t* __restrict__ sig_st, int32_t* __restrict__ codes) {
  const uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  const int p = pk_st[i], s = sig_st[i];
  int c;
  if (p == OVH_ERR_PUBKEY) c = OVH_ERR_PUBKEY;
  else if (s != 0 && s != SIG_INF_MARK) c = s;
  else if (p != 0) c = p;
  else if (s == SIG_INF_MARK) c = BLST_VERIFY_FAIL;
  else c = 0;
  codes[i] = c;
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

__global__ __launch_bounds__(WG) void k_sswu(uint32_t n, Slab s) {
  const uint32_t t = blockIdx.x * WG + threadIdx.x;
  if (t >= 2 * n) return;
  const uint32_t i = t < n ? t : t - n;
  const uint32_t j = t < n ? 0 : 1;
  Fp2 u, x, y;
  s.ld2(u, S_U + 2 * j, i);
  map_to_curve_sswu(x, y, u);
  G2J q;
  iso_map_g2(q, x, y);
  Slab o{s.p + (size_t)(j ? S_Q1 : S_Q0) * 12 * s.cap, s.cap};
  o.st_g2j(q, i);
}

__global__ __launch_bounds__(WG) void k_h2c_fin(uint32_t n, Slab s, int32_t* __restrict__ codes) {
  const uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  Slab q0{s.p + (size_t)S_Q0 * 12 * s.cap, s.cap}, q1{s.p + (size_t)S_Q1 * 12 * s.cap, s.cap};
  G2J a, b;
  q0.ld_g2j(a, i);
  q1.ld_g2j(b, i);
  jac_add(a, a, b);
  g2_clear_cofactor(a, a);
  G2A h;
  if (!jac_to_aff(h, a)) {
    if (codes[i] == 0) codes[i] = BLST_VERIFY_FAIL;  // H(m) = O (probability ~2^-255)
    return;
  }
  Slab o{s.p + (size_t)S_H * 12 * s.cap, s.cap};
  o.st_g2a(h, i);
}

__global__ __launch_bounds__(WG) void k_scalar(uint32_t n, uint64_t seed, Slab s, const int32_t* __restrict__ codes) {
  const uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  Slab rs{s.p + (size_t)S_RS * 12 * s.cap, s.cap};
  G2J S;
  if (codes[i] != 0) {
    jac_set_inf(S);
    rs.st_g2j(S, i);
    return;
  }
  const uint64_t r = rlc_scalar(seed, i);
  G1A pk;
  s.ld_g1a(pk, i);
  G1J P;
  jac_mul_u64(P, pk, r);
  G1A rp;
  jac_to_aff(rp, P);  // r != 0 mod the group order, pk != O
  Slab o{s.p + (size_t)S_RP * 12 * s.cap, s.cap};
  o.st_g1a(rp, i);
  Slab sg{s.p + (size_t)S_SIG * 12 * s.cap, s.cap};
  G2A sig;
  sg.ld_g2a(sig, i);
  jac_mul_u64(S, sig, r);
  rs.st_g2j(S, i);
}

__global__ __launch_bounds__(WG) void k_miller(uint32_t n, Slab s, const int32_t* __restrict__ codes) {
  const uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  Fp12 f;
  if (codes[i] == 0) {
    Slab rp{s.p + (size_t)S_RP * 12 * s.cap, s.cap};
    Slab hh{s.p + (size_t)S_H * 12 * s.cap, s.cap};
    G1A p;
    G2A h;
    rp.ld_g1a(p, i);
    hh.ld_g2a(h, i);
    miller_loop(f, p, h);
  } else {
    fp12_one(f);
  }
  Slab fo{s.p + (size_t)S_F * 12 * s.cap, s.cap};
  fo.st_f12(f, i);
}

// out[t] = prod_{k in chunk t} in[k]
__global__ __launch_bounds__(WG) void k_reduce_f(uint32_t n, uint32_t chunk, Slab in, Slab out) {
  const uint32_t t = blockIdx.x * WG + threadIdx.x;
  const uint32_t lo = t * chunk;
  if (lo >= n) return;
  const uint32_t hi = lo + chunk < n ? lo + chunk : n;
  Fp12 acc, x;
  in.ld_f12(acc, lo);
  for (uint32_t k = lo + 1; k < hi; ++k) {
    in.ld_f12(x, k);
    fp12_mul(acc, acc, x);
  }
  out.st_f12(acc, t);
}

__global__ __launch_bounds__(WG) void k_reduce_s(uint32_t n, uint32_t chunk, Slab in, Slab out) {
  const uint32_t t = blockIdx.x * WG + threadIdx.x;
  const uint32_t lo = t * chunk;
  if (lo >= n) return;
  const uint32_t hi = lo + chunk < n ? lo + chunk : n;
  G2J acc, x;
  in.ld_g2j(acc, lo);
  for (uint32_t k = lo + 1; k < hi; ++k) {
    in.ld_g2j(x, k);
    jac_add(acc, acc, x);
  }
  out.st_g2j(acc, t);
}

// Pack (F, S) of one shard into the 864-byte partial (216 words, AoS).
__global__ __launch_bounds__(WG) void k_pack_partial(Slab f, Slab s, uint32_t* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  for (int j = 0; j < 12; ++j)
    for (int k = 0; k < 12; ++k) out[j * 12 + k] = f.p[(size_t)(j * 12 + k) * f.cap];
  for (int j = 0; j < 6; ++j)
    for (int k = 0; k < 12; ++k) out[144 + j * 12 + k] = s.p[(size_t)(j * 12 + k) * s.cap];
}

// Combined check over k partials: prod F * Miller(-G1, sum S) -> FE == 1.
__global__ __launch_bounds__(WG) void k_final(uint32_t k, const uint32_t* __restrict__ parts, int32_t* __restrict__ result) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  Fp12 F, x;
  G2J S, y;
  fp12_one(F);
  jac_set_inf(S);
  for (uint32_t q = 0; q < k; ++q) {
    const uint32_t* p = parts + (size_t)q * 216;
    Fp* c = &x.c0.c0.c0;
    for (int j = 0; j < 12; ++j)
      for (int l = 0; l < 12; ++l) c[j].v[l] = p[j * 12 + l];
    Fp* d = &y.X.c0;
    for (int j = 0; j < 6; ++j)
      for (int l = 0; l < 12; ++l) d[j].v[l] = p[144 + j * 12 + l];
    fp12_mul(F, F, x);
    jac_add(S, S, y);
  }
  G2A sa;
  if (jac_to_aff(sa, S)) {
    G1A ng1;
    fp_load(ng1.x, G1X_M);
    fp_load(ng1.y, G1NY_M);
    Fp12 m;
    miller_loop(m, ng1, sa);
    fp12_mul(F, F, m);
  }
  final_exponentiation(F, F);
  *result = fp12_is_one(F) ? 1 : 0;
}

__global__ __launch_bounds__(WG) void k_fallback(uint32_t n, Slab s, int32_t* __restrict__ codes) {
  const uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n || codes[i] != 0) return;
  G1A pk;
  G2A sig, h;
  s.ld_g1a(pk, i);
  Slab sg{s.p + (size_t)S_SIG * 12 * s.cap, s.cap};
  Slab hh{s.p + (size_t)S_H * 12 * s.cap, s.cap};
  sg.ld_g2a(sig, i);
  hh.ld_g2a(h, i);
  codes[i] = pairing_check(pk, h, sig) ? 0 : BLST_VERIFY_FAIL;
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
  // OVH_FLAG_PROFILE: start/stop events per stage of the last batch call
  hipEvent_t ev0[OVH_NSTAGES] = {}, ev1[OVH_NSTAGES] = {};
  uint32_t ev_mask = 0;
};

static const char* const STAGE_NAMES[OVH_NSTAGES] = {
    "parse_pk", "parse_sig", "codes", "hash_to_field", "sswu_iso", "h2c_finish",
    "rlc_scalar", "miller", "reduce", "final", "fallback"};

// Stage bracket: events on the context's stream around the stage's kernels.
struct StageScope {
  ovh_ctx* c;
  int k;
  StageScope(ovh_ctx* c_, int k_) : c(c_), k(k_) {
    if (c->flags & OVH_FLAG_PROFILE) (void)hipEventRecord(c->ev0[k], c->stream);
  }
  ~StageScope() {
    if (c->flags & OVH_FLAG_PROFILE) {
      (void)hipEventRecord(c->ev1[k], c->stream);
      c->ev_mask |= 1u << k;
    }
  }
};

#define HIPCHK(x)                                  \
  do {                                             \
    if ((x) != hipSuccess) return OVH_ERR_DEVICE;  \
  } while (0)

static const uint8_t DEFAULT_DST[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_";

static uint32_t nblk(size_t n) { return (uint32_t)((n + WG - 1) / WG); }

static int ensure_cap(ovh_ctx* c, size_t n) {
  if (n > (1u << 24)) return OVH_ERR_ARG;
  if (n <= c->cap && c->state) return 0;
  uint32_t cap = 256;
  while (cap < n) cap <<= 1;
  if (c->state) (void)hipFree(c->state);
  if (c->red) (void)hipFree(c->red);
  if (c->st_pk) (void)hipFree(c->st_pk);
  if (c->st_sig) (void)hipFree(c->st_sig);
  if (c->codes) (void)hipFree(c->codes);
  c->state = nullptr;
  c->red = nullptr;
  HIPCHK(hipMalloc(&c->state, (size_t)S_TOTAL * 12 * cap * 4));
  c->red_cap = cap / 8 > 64 ? cap / 8 : 64;
  HIPCHK(hipMalloc(&c->red, (size_t)2 * 18 * 12 * c->red_cap * 4));
  HIPCHK(hipMalloc(&c->st_pk, (size_t)cap * 4));
  HIPCHK(hipMalloc(&c->st_sig, (size_t)cap * 4));
  HIPCHK(hipMalloc(&c->codes, (size_t)cap * 4));
  c->cap = cap;
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
  for (void* p : {(void*)c->state, (void*)c->red, (void*)c->st_pk, (void*)c->st_sig, (void*)c->codes,
                  (void*)c->in_buf, (void*)c->partial, (void*)c->result})
    if (p) (void)hipFree(p);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  for (int k = 0; k < OVH_NSTAGES; ++k) {
    if (c->ev0[k]) (void)hipEventDestroy(c->ev0[k]);
    if (c->ev1[k]) (void)hipEventDestroy(c->ev1[k]);
  }
  delete c;
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
  if (ensure_cap(c, n > 0 ? n : 1)) return OVH_ERR_DEVICE;
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
  if (ensure_cap(c, n > 0 ? n : 1)) return OVH_ERR_DEVICE;
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
static int batch_front(ovh_ctx* c, uint32_t n, const uint8_t* d_sigs, const uint8_t* d_hashes, const uint8_t* d_pks,
                       uint64_t seed, int32_t* d_codes) {
  Slab s{c->state, c->cap};
  Slab sig{c->state + (size_t)S_SIG * 12 * c->cap, c->cap};
  hipStream_t st = c->stream;
  c->ev_mask = 0;
  { StageScope p(c, ST_PARSE_PK); k_parse_pk<<<nblk(n), WG, 0, st>>>(n, d_pks, c->st_pk, s); }
  { StageScope p(c, ST_PARSE_SIG); k_parse_sig<<<nblk(n), WG, 0, st>>>(n, d_sigs, c->st_sig, sig); }
  { StageScope p(c, ST_CODES); k_codes<<<nblk(n), WG, 0, st>>>(n, c->st_pk, c->st_sig, d_codes); }
  { StageScope p(c, ST_H2F); k_h2f<<<nblk(n), WG, 0, st>>>(n, d_hashes, c->xmd, s); }
  { StageScope p(c, ST_SSWU); k_sswu<<<nblk(2 * (size_t)n), WG, 0, st>>>(n, s); }
  { StageScope p(c, ST_H2C_FIN); k_h2c_fin<<<nblk(n), WG, 0, st>>>(n, s, d_codes); }
  { StageScope p(c, ST_SCALAR); k_scalar<<<nblk(n), WG, 0, st>>>(n, seed, s, d_codes); }
  { StageScope p(c, ST_MILLER); k_miller<<<nblk(n), WG, 0, st>>>(n, s, d_codes); }
  HIPCHK(hipGetLastError());
  // reductions
  const uint32_t chunk = 16;
  Slab fin{c->state + (size_t)S_F * 12 * c->cap, c->cap};
  Slab sin{c->state + (size_t)S_RS * 12 * c->cap, c->cap};
  {
    StageScope p(c, ST_REDUCE);
    uint32_t m = n;
    int flip = 0;
    while (m > 1) {
      const uint32_t mo = (m + chunk - 1) / chunk;
      uint32_t* base = c->red + (size_t)flip * 18 * 12 * c->red_cap;
      Slab fo{base, c->red_cap}, so{base + (size_t)12 * 12 * c->red_cap, c->red_cap};
      k_reduce_f<<<nblk(mo), WG, 0, st>>>(m, chunk, fin, fo);
      k_reduce_s<<<nblk(mo), WG, 0, st>>>(m, chunk, sin, so);
      fin = fo;
      sin = so;
      m = mo;
      flip ^= 1;
    }
    k_pack_partial<<<1, WG, 0, st>>>(fin, sin, c->partial);
  }
  HIPCHK(hipGetLastError());
  c->last_n = n;
  return 0;
}

int ovh_batch_partial_device(ovh_ctx* c, size_t n, const uint8_t* d_sigs, const uint8_t* d_hashes, const uint8_t* d_pks,
                             uint64_t seed, int32_t* d_codes, uint8_t* d_partial) {
  if (!c || !d_codes || !d_partial || (n && (!d_sigs || !d_hashes || !d_pks))) return OVH_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  if (n == 0) {
    // neutral partial: F = 1, S = O
    std::vector<uint32_t> p(216, 0);
    for (int k = 0; k < 12; ++k) p[k] = ONE_M[k];
    for (int k = 0; k < 12; ++k) p[144 + k] = ONE_M[k];       // X = 1
    for (int k = 0; k < 12; ++k) p[144 + 24 + k] = ONE_M[k];  // Y = 1 (Z = 0)
    HIPCHK(hipMemcpyAsync(d_partial, p.data(), 864, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
  }
  if (ensure_cap(c, n)) return OVH_ERR_DEVICE;
  int e = batch_front(c, (uint32_t)n, d_sigs, d_hashes, d_pks, seed, d_codes);
  if (e) return e;
  HIPCHK(hipMemcpyAsync(d_partial, c->partial, 864, hipMemcpyDeviceToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int ovh_combine_partials_device(ovh_ctx* c, size_t k, const uint8_t* d_partials) {
  if (!c || !d_partials || k == 0 || k > 4096) return -OVH_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return -OVH_ERR_DEVICE;
  {
    StageScope p(c, ST_FINAL);
    k_final<<<1, WG, 0, c->stream>>>((uint32_t)k, (const uint32_t*)d_partials, c->result);
  }
  if (hipGetLastError() != hipSuccess) return -OVH_ERR_DEVICE;
  int32_t r = -1;
  if (hipMemcpyAsync(&r, c->result, 4, hipMemcpyDeviceToHost, c->stream) != hipSuccess) return -OVH_ERR_DEVICE;
  if (hipStreamSynchronize(c->stream) != hipSuccess) return -OVH_ERR_DEVICE;
  return r;
}

int ovh_batch_fallback_device(ovh_ctx* c, size_t n, int32_t* d_codes) {
  if (!c || !d_codes) return OVH_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  if (n == 0) return 0;
  if (n != c->last_n) return OVH_ERR_ARG;
  Slab s{c->state, c->cap};
  {
    StageScope p(c, ST_FALLBACK);
    k_fallback<<<nblk(n), WG, 0, c->stream>>>((uint32_t)n, s, d_codes);
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int ovh_verify_batch_device(ovh_ctx* c, size_t n, const uint8_t* d_sigs, const uint8_t* d_hashes, const uint8_t* d_pks,
                            uint64_t seed, int32_t* d_codes) {
  if (!c || (n && (!d_sigs || !d_hashes || !d_pks || !d_codes))) return OVH_ERR_ARG;
  if (n == 0) return 0;
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  if (ensure_cap(c, n)) return OVH_ERR_DEVICE;
  int e = batch_front(c, (uint32_t)n, d_sigs, d_hashes, d_pks, seed, d_codes);
  if (e) return e;
  {
    StageScope p(c, ST_FINAL);
    k_final<<<1, WG, 0, c->stream>>>(1, c->partial, c->result);
  }
  HIPCHK(hipGetLastError());
  int32_t r = -1;
  HIPCHK(hipMemcpyAsync(&r, c->result, 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (r != 1) {
    Slab s{c->state, c->cap};
    StageScope p(c, ST_FALLBACK);
    k_fallback<<<nblk(n), WG, 0, c->stream>>>((uint32_t)n, s, d_codes);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->stream));
  }
  return 0;
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
