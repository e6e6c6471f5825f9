// overlord 0.4 `Vote` RLP encoding (the bytes Consensus::check_block and the vote signer hash,
// /root/reference/src/consensus.rs:169-175; rlp 0.5, Cargo.toml:25): rlp([height u64,
// round u64, vote_type u8, block_hash bytes]) -- the same rules as consensus_overlord_amd/vote.py
// (SURVEY.md Appendix B). Host/device portable: k_vote_digest (ovh_vote_digests*) runs it with
// SM3 on the device, tests/host/harness.cpp on the host.
#pragma once
#include <stdint.h>

#include "sm3.hpp"

namespace ovh {

constexpr uint32_t VOTE_HASH_MAX = 64;       // block_hash bytes per vote (stride of the inputs)
// list header 2, height 9, round 9, vote_type 2 (a type >= 0x80 encodes as 0x81 xx), hash 2 + 64
constexpr uint32_t VOTE_RLP_MAX = 2 + 9 + 9 + 2 + 2 + VOTE_HASH_MAX;

// an unsigned integer: 0x80 for zero, a single byte < 0x80 as itself, else 0x80 + len || BE
SM3_HD uint32_t rlp_uint(uint8_t* o, uint64_t v) {
  if (v == 0) {
    o[0] = 0x80;
    return 1;
  }
  if (v < 0x80) {
    o[0] = (uint8_t)v;
    return 1;
  }
  uint32_t nb = 0;
  for (uint64_t t = v; t; t >>= 8) ++nb;
  o[0] = (uint8_t)(0x80 + nb);
  for (uint32_t k = 0; k < nb; ++k) o[1 + k] = (uint8_t)(v >> (8 * (nb - 1 - k)));
  return 1 + nb;
}

// a byte string of len <= VOTE_HASH_MAX (< 256)
SM3_HD uint32_t rlp_bytes(uint8_t* o, const uint8_t* b, uint32_t len) {
  if (len == 1 && b[0] < 0x80) {
    o[0] = b[0];
    return 1;
  }
  uint32_t h = 1;
  if (len < 56) {
    o[0] = (uint8_t)(0x80 + len);
  } else {
    o[0] = 0xB8;  // 0xB7 + one length byte
    o[1] = (uint8_t)len;
    h = 2;
  }
  for (uint32_t k = 0; k < len; ++k) o[h + k] = b[k];
  return h + len;
}

// rlp(Vote) into out (>= VOTE_RLP_MAX bytes); returns its length
SM3_HD uint32_t rlp_vote(uint8_t* out, uint64_t height, uint64_t round, uint8_t vote_type, const uint8_t* block_hash,
                         uint32_t hash_len) {
  uint8_t pay[VOTE_RLP_MAX];
  uint32_t n = rlp_uint(pay, height);
  n += rlp_uint(pay + n, round);
  n += rlp_uint(pay + n, vote_type);
  n += rlp_bytes(pay + n, block_hash, hash_len);
  uint32_t h = 1;
  if (n < 56) {
    out[0] = (uint8_t)(0xC0 + n);
  } else {
    out[0] = 0xF8;  // 0xF7 + one length byte
    out[1] = (uint8_t)n;
    h = 2;
  }
  for (uint32_t k = 0; k < n; ++k) out[h + k] = pay[k];
  return h + n;
}

// Crypto::hash(rlp(Vote)) = SM3 (util.rs:83-87)
SM3_HD void vote_digest(uint8_t out[32], uint64_t height, uint64_t round, uint8_t vote_type, const uint8_t* block_hash,
                        uint32_t hash_len) {
  uint8_t buf[VOTE_RLP_MAX];
  const uint32_t n = rlp_vote(buf, height, round, vote_type, block_hash, hash_len);
  sm3_digest(buf, n, out);
}

}  // namespace ovh
