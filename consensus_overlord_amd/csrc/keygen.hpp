// Private-key parse of ConsensusCrypto::new (src/consensus.rs:349-350):
// `BlsPrivateKey::try_from(hex::decode(file))` in ophelia-blst 0.3 [dep, un-vendored].
//
// The reference's own key, example/private_key = ed391472...1690, is >= r, and the reference
// unwraps the parse (consensus.rs:350, README.md:66), so the parse is NOT blst's strict
// `SecretKey::from_bytes` (32-byte big-endian, 0 < sk < r). blst's Rust API has exactly one
// other constructor from bytes, `SecretKey::key_gen(ikm, key_info)`: IETF KeyGen
// (draft-irtf-cfrg-bls-signature-04 section 2.3, = EIP-2333 HKDF_mod_r) with ikm >= 32 bytes.
// That is the default here; OVH_FLAG_SK_RAW selects the strict scalar form instead.
//
//   salt = "BLS-SIG-KEYGEN-SALT-"; SK = 0
//   while SK == 0:
//     salt = SHA-256(salt)
//     PRK  = HKDF-Extract(salt, IKM || I2OSP(0, 1))
//     OKM  = HKDF-Expand(PRK, key_info || I2OSP(48, 2), 48)
//     SK   = OS2IP(OKM) mod r
//
// Host code: a key is parsed once per ConsensusCrypto::new; every curve operation on the
// scalar runs in the HIP kernels.
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "bls/h2c.hpp"

namespace ovh {
namespace keygen {

struct Sha256 {
  uint32_t st[8];
  uint8_t buf[64];
  uint64_t len = 0;
  size_t fill = 0;
  Sha256() { sha256_iv(st); }
  void block(const uint8_t* p) {
    uint32_t w[16];
    for (int i = 0; i < 16; ++i)
      w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
    sha256_compress(st, w);
  }
  void update(const uint8_t* p, size_t n) {
    len += n;
    while (n) {
      const size_t k = n < 64 - fill ? n : 64 - fill;
      memcpy(buf + fill, p, k);
      fill += k;
      p += k;
      n -= k;
      if (fill == 64) {
        block(buf);
        fill = 0;
      }
    }
  }
  void final(uint8_t out[32]) {
    const uint64_t bits = len * 8;
    const uint8_t one = 0x80, zero = 0;
    update(&one, 1);
    while (fill != 56) update(&zero, 1);
    uint8_t l[8];
    for (int i = 0; i < 8; ++i) l[i] = (uint8_t)(bits >> (56 - 8 * i));
    update(l, 8);
    for (int i = 0; i < 8; ++i)
      for (int b = 0; b < 4; ++b) out[4 * i + b] = (uint8_t)(st[i] >> (24 - 8 * b));
  }
};

// zero secret intermediates (volatile stores: not removed as dead by the optimiser)
inline void wipe(void* p, size_t n) {
  volatile uint8_t* q = (volatile uint8_t*)p;
  while (n--) *q++ = 0;
}

inline void sha256(uint8_t out[32], const uint8_t* m, size_t n) {
  Sha256 h;
  h.update(m, n);
  h.final(out);
}

// HMAC-SHA256(key, m1 || m2 || m3) (RFC 2104)
inline void hmac(uint8_t out[32], const uint8_t* key, size_t klen, const uint8_t* m1, size_t n1,
                 const uint8_t* m2 = nullptr, size_t n2 = 0, const uint8_t* m3 = nullptr, size_t n3 = 0) {
  uint8_t k[64] = {0}, pad[64], inner[32];
  if (klen > 64) sha256(k, key, klen);
  else memcpy(k, key, klen);
  Sha256 hi, ho;
  for (int i = 0; i < 64; ++i) pad[i] = k[i] ^ 0x36;
  hi.update(pad, 64);
  hi.update(m1, n1);
  if (n2) hi.update(m2, n2);
  if (n3) hi.update(m3, n3);
  hi.final(inner);
  for (int i = 0; i < 64; ++i) pad[i] = k[i] ^ 0x5c;
  ho.update(pad, 64);
  ho.update(inner, 32);
  ho.final(out);
  wipe(k, sizeof k);
  wipe(pad, sizeof pad);
  wipe(inner, sizeof inner);
}

// RFC 5869 HKDF-Expand with SHA-256, L <= 255 * 32.
inline void hkdf_expand(uint8_t* okm, size_t L, const uint8_t prk[32], const uint8_t* info, size_t ilen) {
  uint8_t t[32], prev[32];
  size_t done = 0;
  for (uint8_t i = 1; done < L; ++i) {
    // T(i) = HMAC(PRK, T(i-1) || info || i), T(0) = ""
    const uint8_t msg_i[1] = {i};
    memcpy(prev, t, 32);
    hmac(t, prk, 32, prev, i > 1 ? 32 : 0, info, ilen, msg_i, 1);
    const size_t k = L - done < 32 ? L - done : 32;
    memcpy(okm + done, t, k);
    done += k;
  }
  wipe(t, sizeof t);
  wipe(prev, sizeof prev);
}

static const uint8_t R_BE[32] = {0x73, 0xed, 0xa7, 0x53, 0x29, 0x9d, 0x7d, 0x48, 0x33, 0x39, 0xd8,
                                 0x08, 0x09, 0xa1, 0xd8, 0x05, 0x53, 0xbd, 0xa4, 0x02, 0xff, 0xfe,
                                 0x5b, 0xfe, 0xff, 0xff, 0xff, 0xff, 0x00, 0x00, 0x00, 0x01};

// out (32 bytes, big-endian) = OS2IP(in[0..n)) mod r, by shift-and-subtract.
inline void be_mod_r(uint8_t out[32], const uint8_t* in, size_t n) {
  uint8_t acc[33] = {0};  // acc < 2r < 2^256, one spare byte for the shift
  for (size_t i = 0; i < n * 8; ++i) {
    const int bit = (in[i / 8] >> (7 - i % 8)) & 1;
    int c = bit;
    for (int j = 32; j >= 0; --j) {
      const int v = (acc[j] << 1) | c;
      acc[j] = (uint8_t)v;
      c = v >> 8;
    }
    // acc >= r ? acc - r
    bool ge = acc[0] != 0;
    if (!ge) {
      ge = true;
      for (int j = 0; j < 32; ++j)
        if (acc[j + 1] != R_BE[j]) {
          ge = acc[j + 1] > R_BE[j];
          break;
        }
    }
    if (ge) {
      int br = 0;
      for (int j = 31; j >= 0; --j) {
        const int v = (int)acc[j + 1] - R_BE[j] - br;
        acc[j + 1] = (uint8_t)v;
        br = v < 0;
      }
      acc[0] = (uint8_t)(acc[0] - br);
    }
  }
  memcpy(out, acc + 1, 32);
  wipe(acc, sizeof acc);
}

inline bool is_zero32(const uint8_t* a) {
  uint8_t z = 0;
  for (int i = 0; i < 32; ++i) z |= a[i];
  return z == 0;
}

// blst SecretKey::key_gen(ikm, key_info = ""): false if ikm is shorter than 32 bytes.
inline bool key_gen(uint8_t sk_be[32], const uint8_t* ikm, size_t ilen) {
  if (!ikm || ilen < 32) return false;
  uint8_t salt[32];
  static const uint8_t SALT0[] = "BLS-SIG-KEYGEN-SALT-";
  sha256(salt, SALT0, 20);
  static const uint8_t ZERO1[1] = {0}, L2[2] = {0, 48};
  for (;;) {
    uint8_t prk[32], okm[48];
    hmac(prk, salt, 32, ikm, ilen, ZERO1, 1);  // HKDF-Extract(salt, IKM || I2OSP(0, 1))
    hkdf_expand(okm, 48, prk, L2, 2);         // info = key_info ("") || I2OSP(L, 2)
    be_mod_r(sk_be, okm, 48);
    wipe(prk, sizeof prk);
    wipe(okm, sizeof okm);
    if (!is_zero32(sk_be)) return true;
    sha256(salt, salt, 32);
  }
}

// blst SecretKey::from_bytes: 32-byte big-endian, 0 < sk < r.
inline bool sk_raw(uint8_t sk_be[32], const uint8_t* b, size_t n) {
  if (!b || n != 32 || is_zero32(b) || memcmp(b, R_BE, 32) >= 0) return false;
  memcpy(sk_be, b, 32);
  return true;
}

}  // namespace keygen
}  // namespace ovh
