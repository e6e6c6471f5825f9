// Single-lane verification with the reference's semantics and error precedence
// (ConsensusCrypto::verify_signature, src/consensus.rs:397-416):
//   hash length (100) -> public key parse (102) -> signature parse (blst code)
//   -> blst core_verify: sig group check, pk infinity, pk group check, pairing equation.
#pragma once
#include "h2c.hpp"
#include "pairing.hpp"

namespace ovh {

// Same values as include/ovhip.h.
#ifndef OVH_OK
#define OVH_OK 0
#define OVH_ERR_HASH_LEN 100
#define OVH_ERR_LEN_MISMATCH 101
#define OVH_ERR_PUBKEY 102
#define OVH_ERR_ARG 103
#define OVH_ERR_DEVICE 200
#endif

OVH_HD void be_words_from_bytes(uint32_t* w, const uint8_t* b, int nwords) {
  for (int i = 0; i < nwords; ++i)
    w[i] = ((uint32_t)b[4 * i] << 24) | ((uint32_t)b[4 * i + 1] << 16) | ((uint32_t)b[4 * i + 2] << 8) | b[4 * i + 3];
}

// e(pk, H(m)) == e(G1, sig)  <=>  FE(Miller(pk, H) * Miller(-G1, sig)) == 1
OVH_HDNI bool pairing_check(const G1A& pk, const G2A& h, const G2A& sig) {
  Fp12 f1, f2;
  miller_loop(f1, pk, h);
  G1A ng1;
  fp_load(ng1.x, G1X_M);
  fp_load(ng1.y, G1NY_M);
  miller_loop(f2, ng1, sig);
  fp12_mul(f1, f1, f2);
  final_exponentiation(f1, f1);
  return fp12_is_one(f1);
}

// blst core_verify (min-pk) on parsed points. sig_inf / pk_inf flag the infinity encodings.
OVH_HDNI int core_verify(const G1A& pk, bool pk_inf, const G2A& sig, bool sig_inf, const uint32_t msg[8],
                         const XmdTemplates& t) {
  if (!sig_inf) {
    G2J sj;
    jac_from_aff(sj, sig);
    if (!g2_in_subgroup(sj)) return BLST_POINT_NOT_IN_GROUP;
  }
  if (pk_inf) return BLST_PK_IS_INFINITY;
  G1J pj;
  jac_from_aff(pj, pk);
  if (!g1_in_subgroup(pj)) return BLST_POINT_NOT_IN_GROUP;
  G2J hj;
  hash_to_g2(hj, msg, t);
  G2A h;
  if (!jac_to_aff(h, hj)) return BLST_VERIFY_FAIL;  // H(m) = O: e(pk, O) = 1 != e(G1, sig) unless sig = O
  if (sig_inf) return BLST_VERIFY_FAIL;               // e(pk, H) != 1 for pk, H != O
  return pairing_check(pk, h, sig) ? BLST_SUCCESS : BLST_VERIFY_FAIL;
}

OVH_HDNI int verify_one(const uint8_t* sig, uint32_t sig_len, const uint8_t* hash, uint32_t hash_len, const uint8_t* pk,
                        uint32_t pk_len, const XmdTemplates& t) {
  if (hash_len != 32) return OVH_ERR_HASH_LEN;
  G1A p;
  bool pinf;
  if (g1_from_bytes(p, pinf, pk, pk_len) != BLST_SUCCESS) return OVH_ERR_PUBKEY;
  G2A s;
  bool sinf;
  int e = g2_from_bytes(s, sinf, sig, sig_len);
  if (e != BLST_SUCCESS) return e;
  uint32_t msg[8];
  be_words_from_bytes(msg, hash, 8);
  return core_verify(p, pinf, s, sinf, msg, t);
}

}  // namespace ovh
