// Work model: counts the Fp Montgomery multiplications (M, squarings included) that each
// batch stage of libovhip performs for ONE vote, by running the device arithmetic headers on
// the host (g++) with OVH_COUNT_MULS. Each block below mirrors the body of the kernel named
// in its label (consensus_overlord_amd/csrc/ovhip.hip); the counts are the per-unit
// algorithmic work bench.py prices the roofline with (DESIGN.md "Work model").
//
//   g++ -O2 -std=c++17 -DOVH_COUNT_MULS -o /tmp/count_muls tools/count_muls.cpp && /tmp/count_muls
//
// Prints one JSON object: {"stage": M_per_unit, ...}. Tool only: not part of the product.
#include <stdio.h>
#include <string.h>

#include "../consensus_overlord_amd/csrc/bls/verify.hpp"

namespace ovh {
unsigned long long g_fp_mul_count = 0;
}
using namespace ovh;

static const uint8_t DST[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_";

static unsigned long long take() {
  unsigned long long v = g_fp_mul_count;
  g_fp_mul_count = 0;
  return v;
}

int main() {
  XmdTemplates t;
  xmd_build_templates(t, DST, 43);
  // one synthetic vote: sk = 0x1234...; msg = 32 bytes
  uint32_t sk[8] = {0x9abcdef1u, 0x12345678u, 0x0badf00du, 0xdeadbeefu, 0x01020304u, 0x05060708u, 0x11223344u, 0x2ec0ffeeu};
  uint8_t hash[32];
  for (int i = 0; i < 32; ++i) hash[i] = (uint8_t)(7 * i + 3);
  uint32_t msg[8];
  be_words_from_bytes(msg, hash, 8);
  uint8_t pk48[48], sig96[96];
  {
    G1J g, p;
    fp_load(g.X, G1X_M);
    fp_load(g.Y, G1Y_M);
    fp_one(g.Z);
    jac_mul_words(p, g, sk, 8);
    g1_compress(pk48, p);
    G2J h, s;
    hash_to_g2(h, msg, t);
    jac_mul_words(s, h, sk, 8);
    g2_compress(sig96, s);
  }
  take();
  printf("{");
  // k_parse_pk
  G1A pk;
  bool inf;
  g1_from_bytes(pk, inf, pk48, 48);
  {
    G1J j;
    jac_from_aff(j, pk);
    g1_in_subgroup(j);
  }
  printf("\"parse_pk\": %llu", take());
  // k_parse_sig
  G2A sig;
  g2_from_bytes(sig, inf, sig96, 96);
  {
    G2J j;
    jac_from_aff(j, sig);
    g2_in_subgroup(j);
  }
  printf(", \"parse_sig\": %llu", take());
  // k_h2f
  uint32_t uni[64];
  expand_message_xmd_256(uni, msg, t);
  Fp2 u0, u1;
  hash_to_field_fp2x2(u0, u1, uni);
  printf(", \"hash_to_field\": %llu", take());
  // k_sswu: two units (u0, u1) per vote -> per vote
  G2J q0, q1;
  {
    Fp2 x, y;
    map_to_curve_sswu(x, y, u0);
    iso_map_g2(q0, x, y);
    map_to_curve_sswu(x, y, u1);
    iso_map_g2(q1, x, y);
  }
  printf(", \"sswu_iso\": %llu", take());
  // k_h2c_fin
  G2A h;
  {
    G2J a;
    jac_add(a, q0, q1);
    g2_clear_cofactor(a, a);
    jac_to_aff(h, a);
  }
  printf(", \"h2c_finish\": %llu", take());
  // k_scalar (r: a full-weight 64-bit scalar)
  const uint64_t r = 0xd7a1c3b5e9f20486ull;
  G1A rp;
  G2J rs;
  {
    G1J P;
    jac_mul_u64(P, pk, r);
    jac_to_aff(rp, P);
    jac_mul_u64(rs, sig, r);
  }
  printf(", \"rlc_scalar\": %llu", take());
  // k_miller
  Fp12 f;
  miller_loop(f, rp, h);
  printf(", \"miller\": %llu", take());
  // k_reduce_f / k_reduce_s: one fp12_mul and one G2 Jacobian add per vote
  {
    Fp12 g = f;
    fp12_mul(g, g, f);
    G2J s2 = rs;
    jac_add(s2, s2, rs);
  }
  printf(", \"reduce\": %llu", take());
  // k_final (once per batch): Miller(-G1, S) + final exponentiation
  {
    G2J S = rs;
    G2A sa;
    jac_to_aff(sa, S);
    G1A ng1;
    fp_load(ng1.x, G1X_M);
    fp_load(ng1.y, G1NY_M);
    Fp12 m;
    miller_loop(m, ng1, sa);
    fp12_mul(m, m, f);
    final_exponentiation(m, m);
  }
  printf(", \"final_per_batch\": %llu", take());
  // k_fallback (per vote, only when the combined check fails)
  pairing_check(pk, h, sig);
  printf(", \"fallback\": %llu", take());
  // single-call verify_one (the reference's per-call shape)
  verify_one(sig96, 96, hash, 32, pk48, 48, t);
  printf(", \"verify_one\": %llu", take());
  printf("}\n");
  return 0;
}
