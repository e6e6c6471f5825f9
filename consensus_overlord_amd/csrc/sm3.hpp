// SM3 (GB/T 32905-2016), the digest behind Crypto::hash (src/util.rs:83-87, libsm 0.6).
// Host/device portable; the C ABI's ovh_sm3 runs it on the host (one 64-byte compression
// per vote, < 1 us), the batch kernels can call it on device.
#pragma once
#include <stddef.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define SM3_HD __host__ __device__ inline
#else
#define SM3_HD inline
#endif

namespace ovh {

SM3_HD uint32_t sm3_rotl(uint32_t x, int n) {
  n &= 31;
  return n ? (x << n) | (x >> (32 - n)) : x;
}

SM3_HD void sm3_compress(uint32_t v[8], const uint8_t blk[64]) {
  uint32_t w[68], w1[64];
  for (int j = 0; j < 16; ++j)
    w[j] = ((uint32_t)blk[4 * j] << 24) | ((uint32_t)blk[4 * j + 1] << 16) | ((uint32_t)blk[4 * j + 2] << 8) | blk[4 * j + 3];
  for (int j = 16; j < 68; ++j) {
    uint32_t x = w[j - 16] ^ w[j - 9] ^ sm3_rotl(w[j - 3], 15);
    x = x ^ sm3_rotl(x, 15) ^ sm3_rotl(x, 23);
    w[j] = x ^ sm3_rotl(w[j - 13], 7) ^ w[j - 6];
  }
  for (int j = 0; j < 64; ++j) w1[j] = w[j] ^ w[j + 4];
  uint32_t a = v[0], b = v[1], c = v[2], d = v[3], e = v[4], f = v[5], g = v[6], h = v[7];
  for (int j = 0; j < 64; ++j) {
    const uint32_t tj = j < 16 ? 0x79cc4519u : 0x7a879d8au;
    const uint32_t ss1 = sm3_rotl(sm3_rotl(a, 12) + e + sm3_rotl(tj, j), 7);
    const uint32_t ss2 = ss1 ^ sm3_rotl(a, 12);
    const uint32_t ff = j < 16 ? (a ^ b ^ c) : ((a & b) | (a & c) | (b & c));
    const uint32_t gg = j < 16 ? (e ^ f ^ g) : ((e & f) | (~e & g));
    const uint32_t tt1 = ff + d + ss2 + w1[j];
    const uint32_t tt2 = gg + h + ss1 + w[j];
    d = c;
    c = sm3_rotl(b, 9);
    b = a;
    a = tt1;
    h = g;
    g = sm3_rotl(f, 19);
    f = e;
    e = tt2 ^ sm3_rotl(tt2, 9) ^ sm3_rotl(tt2, 17);
  }
  v[0] ^= a;
  v[1] ^= b;
  v[2] ^= c;
  v[3] ^= d;
  v[4] ^= e;
  v[5] ^= f;
  v[6] ^= g;
  v[7] ^= h;
}

SM3_HD void sm3_digest(const uint8_t* msg, size_t len, uint8_t out[32]) {
  uint32_t v[8] = {0x7380166fu, 0x4914b2b9u, 0x172442d7u, 0xda8a0600u,
                   0xa96f30bcu, 0x163138aau, 0xe38dee4du, 0xb0fb0e4eu};
  size_t off = 0;
  while (len - off >= 64) {
    sm3_compress(v, msg + off);
    off += 64;
  }
  uint8_t blk[128];
  size_t rem = len - off;
  for (size_t i = 0; i < rem; ++i) blk[i] = msg[off + i];
  blk[rem] = 0x80;
  size_t total = (rem + 9 <= 64) ? 64 : 128;
  for (size_t i = rem + 1; i < total; ++i) blk[i] = 0;
  const uint64_t bits = (uint64_t)len * 8;
  for (int i = 0; i < 8; ++i) blk[total - 1 - i] = (uint8_t)(bits >> (8 * i));
  sm3_compress(v, blk);
  if (total == 128) sm3_compress(v, blk + 64);
  for (int i = 0; i < 8; ++i) {
    out[4 * i] = (uint8_t)(v[i] >> 24);
    out[4 * i + 1] = (uint8_t)(v[i] >> 16);
    out[4 * i + 2] = (uint8_t)(v[i] >> 8);
    out[4 * i + 3] = (uint8_t)v[i];
  }
}

}  // namespace ovh
