/* CPU ORACLE (test infrastructure + the timed CPU baseline; never linked into the product).
 *
 * A plain-C restatement of the BLS12-381 min-pk signature path behind the reference's
 * overlord `Crypto` implementation `ConsensusCrypto` (/root/reference/src/consensus.rs:334-463),
 * whose arithmetic lives in the un-vendored ophelia-blst 0.3 -> blst 0.3.x
 * (/root/reference/Cargo.toml:19-20). It restates oracle/py/bls12_381.py (pinned to RFC 9380
 * and the generator/KAT values by tests/test_oracle_kat.py) with 6 x 64-bit Montgomery limbs,
 * independently of the HIP code (which uses 12 x 32-bit limbs and its own formulas):
 *
 *   orc_verify              ConsensusCrypto::verify_signature       consensus.rs:397-416
 *   orc_aggregate_sigs      ConsensusCrypto::aggregate_signatures   consensus.rs:418-444
 *   orc_aggregate_pks       BlsPublicKey::aggregate                 consensus.rs:371
 *   orc_verify_aggregated   verify_aggregated_signature + inner_... consensus.rs:446-462, 365-382
 *   orc_sign / orc_sk_to_pk ConsensusCrypto::sign / new             consensus.rs:390-395, 347-359
 *   orc_sk_keygen           BlsPrivateKey::try_from = IETF KeyGen  consensus.rs:349-350 (see below)
 *   orc_verify_many         the serial per-vote shape overlord drives, threaded
 *   orc_verify_batch_rlc    the random-linear-combination batch check the GPU runs, threaded
 *
 * Return codes are those of include/ovhip.h (0 ok, 1..7 BLST_ERROR, 100 hash length,
 * 101 length mismatch, 102 "lose public key"). Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg load this library.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;

/* ------------------------------------------------------------------------------ Fp */
typedef struct {
  uint64_t l[6];
} fp;

static const uint64_t P[6] = {0xb9feffffffffaaabull, 0x1eabfffeb153ffffull, 0x6730d2a0f6b0f624ull,
                              0x64774b84f38512bfull, 0x4b1ba7b6434bacd7ull, 0x1a0111ea397fe69aull};
static uint64_t PINV;                          /* -p^-1 mod 2^64 */
static fp ONE, R2, R3;                         /* R, R^2, R^3 mod p (R = 2^384) */
static uint64_t E_PM2[6], E_SQRT[6], E_LEG[6]; /* p-2, (p+1)/4, (p-1)/2 */

static int limbs_geq_p(const uint64_t* a) {
  for (int i = 5; i >= 0; --i) {
    if (a[i] > P[i]) return 1;
    if (a[i] < P[i]) return 0;
  }
  return 1;
}

static void sub_p(uint64_t* a) {
  uint64_t br = 0;
  for (int i = 0; i < 6; ++i) {
    u128 d = (u128)a[i] - P[i] - br;
    a[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
}

static void fp_add(fp* r, const fp* a, const fp* b) {
  uint64_t c = 0, t[6];
  for (int i = 0; i < 6; ++i) {
    u128 s = (u128)a->l[i] + b->l[i] + c;
    t[i] = (uint64_t)s;
    c = (uint64_t)(s >> 64);
  }
  if (c || limbs_geq_p(t)) sub_p(t);
  memcpy(r->l, t, 48);
}

static void fp_sub(fp* r, const fp* a, const fp* b) {
  uint64_t br = 0, t[6];
  for (int i = 0; i < 6; ++i) {
    u128 d = (u128)a->l[i] - b->l[i] - br;
    t[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
  if (br) {
    uint64_t c = 0;
    for (int i = 0; i < 6; ++i) {
      u128 s = (u128)t[i] + P[i] + c;
      t[i] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
  }
  memcpy(r->l, t, 48);
}

/* CIOS Montgomery product a b R^-1 mod p (portable; the reference for the mulx form below) */
static void fp_mul_cios(fp* r, const fp* a, const fp* b) {
  uint64_t t[8] = {0};
  for (int i = 0; i < 6; ++i) {
    uint64_t c = 0;
    for (int j = 0; j < 6; ++j) {
      u128 s = (u128)a->l[j] * b->l[i] + t[j] + c;
      t[j] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
    u128 s = (u128)t[6] + c;
    t[6] = (uint64_t)s;
    t[7] = (uint64_t)(s >> 64);
    const uint64_t m = t[0] * PINV;
    s = (u128)m * P[0] + t[0];
    c = (uint64_t)(s >> 64);
    for (int j = 1; j < 6; ++j) {
      s = (u128)m * P[j] + t[j] + c;
      t[j - 1] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
    s = (u128)t[6] + c;
    t[5] = (uint64_t)s;
    t[6] = t[7] + (uint64_t)(s >> 64);
  }
  if (t[6] || limbs_geq_p(t)) sub_p(t);
  memcpy(r->l, t, 48);
}

#if defined(__x86_64__)
#include "mont_mulx.h"
#endif
/* 1: the product runs as BMI2 mulx + ADX adcx / adox asm (tools/gen_mulx.py; chosen at init by
 * CPUID unless ORC_NO_MULX is set), 0: the portable CIOS. The two agree bit for bit
 * (orc_mulx_selftest, tests/test_oracle_c.py); only the timed CPU baseline cares which runs. */
static int g_mulx = 0;

static void fp_mul(fp* r, const fp* a, const fp* b) {
#if defined(__x86_64__)
  /* (the asm form assumes canonical operands, t < 2^447 in seven limbs; hash_to_field multiplies
   * raw 384-bit halves, which take the CIOS) */
  if (g_mulx && a->l[5] < P[5] && b->l[5] < P[5]) {
    fp_mul_mulx(r->l, a->l, b->l, P, PINV);
    return;
  }
#endif
  fp_mul_cios(r, a, b);
}

static void fp_sqr(fp* r, const fp* a) { fp_mul(r, a, a); }
static void fp_zero(fp* r) { memset(r, 0, sizeof(*r)); }
static void fp_one(fp* r) { *r = ONE; }
static int fp_is_zero(const fp* a) { return (a->l[0] | a->l[1] | a->l[2] | a->l[3] | a->l[4] | a->l[5]) == 0; }
static int fp_eq(const fp* a, const fp* b) { return memcmp(a, b, sizeof(fp)) == 0; }
static void fp_neg(fp* r, const fp* a) {
  fp z;
  fp_zero(&z);
  fp_sub(r, &z, a);
}

static void fp_pow(fp* r, const fp* a, const uint64_t* e) {
  fp acc = ONE;
  int started = 0;
  for (int w = 5; w >= 0; --w)
    for (int b = 63; b >= 0; --b) {
      if (started) fp_sqr(&acc, &acc);
      if ((e[w] >> b) & 1) {
        if (started) fp_mul(&acc, &acc, a);
        else {
          acc = *a;
          started = 1;
        }
      }
    }
  *r = acc;
}

static void fp_inv(fp* r, const fp* a) { fp_pow(r, a, E_PM2); }

static int fp_sqrt(fp* r, const fp* a) {
  fp s, s2;
  fp_pow(&s, a, E_SQRT);
  fp_sqr(&s2, &s);
  *r = s;
  return fp_eq(&s2, a);
}

static int fp_is_square(const fp* a) {
  if (fp_is_zero(a)) return 1;
  fp t;
  fp_pow(&t, a, E_LEG);
  return fp_eq(&t, &ONE);
}

static void fp_from_plain(fp* r, const uint64_t* v) {
  fp t;
  memcpy(t.l, v, 48);
  fp_mul(r, &t, &R2);
}

static void fp_to_plain(uint64_t* v, const fp* a) {
  fp one_plain, t;
  fp_zero(&one_plain);
  one_plain.l[0] = 1;
  fp_mul(&t, a, &one_plain);
  memcpy(v, t.l, 48);
}

static void be48_to_limbs(uint64_t* v, const uint8_t* b) {
  for (int i = 0; i < 6; ++i) {
    uint64_t x = 0;
    for (int k = 0; k < 8; ++k) x = (x << 8) | b[40 - 8 * i + k];
    v[i] = x;
  }
}

static void limbs_to_be48(uint8_t* b, const uint64_t* v) {
  for (int i = 0; i < 6; ++i)
    for (int k = 0; k < 8; ++k) b[40 - 8 * i + k] = (uint8_t)(v[i] >> (56 - 8 * k));
}

/* canonical value > (p-1)/2 ?  (ZCash sort flag) */
static int fp_lex_largest(const fp* a) {
  uint64_t v[6], h[6];
  fp_to_plain(v, a);
  /* h = (p-1)/2 */
  memcpy(h, E_LEG, 48);
  for (int i = 5; i >= 0; --i) {
    if (v[i] > h[i]) return 1;
    if (v[i] < h[i]) return 0;
  }
  return 0;
}

static int fp_sgn0(const fp* a) {
  uint64_t v[6];
  fp_to_plain(v, a);
  return (int)(v[0] & 1);
}

static void fp_small(fp* r, uint64_t v) {
  uint64_t t[6] = {v, 0, 0, 0, 0, 0};
  fp_from_plain(r, t);
}

static void fp_from_hex(fp* r, const char* hex) {
  uint64_t v[6] = {0};
  size_t n = strlen(hex);
  for (size_t i = 0; i < n; ++i) {
    char ch = hex[i];
    uint64_t d = (ch >= '0' && ch <= '9') ? (uint64_t)(ch - '0') : (uint64_t)((ch | 0x20) - 'a' + 10);
    /* v = v * 16 + d */
    uint64_t c = d;
    for (int k = 0; k < 6; ++k) {
      u128 s = ((u128)v[k] << 4) + c;
      v[k] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
  }
  fp_from_plain(r, v);
}

static void fp_add_b(fp* r, const fp* a); /* + 4 */

/* ------------------------------------------------------------------------------ Fp2 */
typedef struct {
  fp c0, c1;
} fp2;

static void f2_add(fp2* r, const fp2* a, const fp2* b) {
  fp_add(&r->c0, &a->c0, &b->c0);
  fp_add(&r->c1, &a->c1, &b->c1);
}
static void f2_sub(fp2* r, const fp2* a, const fp2* b) {
  fp_sub(&r->c0, &a->c0, &b->c0);
  fp_sub(&r->c1, &a->c1, &b->c1);
}
static void f2_neg(fp2* r, const fp2* a) {
  fp_neg(&r->c0, &a->c0);
  fp_neg(&r->c1, &a->c1);
}
static void f2_conj(fp2* r, const fp2* a) {
  r->c0 = a->c0;
  fp_neg(&r->c1, &a->c1);
}
static void f2_mul(fp2* r, const fp2* a, const fp2* b) {
  fp t0, t1, s, u, v;
  fp_mul(&t0, &a->c0, &b->c0);
  fp_mul(&t1, &a->c1, &b->c1);
  fp_add(&s, &a->c0, &a->c1);
  fp_add(&u, &b->c0, &b->c1);
  fp_mul(&v, &s, &u);
  fp_sub(&r->c0, &t0, &t1);
  fp_sub(&v, &v, &t0);
  fp_sub(&r->c1, &v, &t1);
}
static void f2_sqr(fp2* r, const fp2* a) {
  fp s, d, m;
  fp_add(&s, &a->c0, &a->c1);
  fp_sub(&d, &a->c0, &a->c1);
  fp_mul(&m, &a->c0, &a->c1);
  fp_mul(&r->c0, &s, &d);
  fp_add(&r->c1, &m, &m);
}
static void f2_mul_fp(fp2* r, const fp2* a, const fp* b) {
  fp_mul(&r->c0, &a->c0, b);
  fp_mul(&r->c1, &a->c1, b);
}
static void f2_mul_xi(fp2* r, const fp2* a) { /* (1 + u) a */
  fp t0, t1;
  fp_sub(&t0, &a->c0, &a->c1);
  fp_add(&t1, &a->c0, &a->c1);
  r->c0 = t0;
  r->c1 = t1;
}
static void f2_zero(fp2* r) { memset(r, 0, sizeof(*r)); }
static void f2_one(fp2* r) {
  r->c0 = ONE;
  fp_zero(&r->c1);
}
static int f2_is_zero(const fp2* a) { return fp_is_zero(&a->c0) && fp_is_zero(&a->c1); }
static int f2_eq(const fp2* a, const fp2* b) { return fp_eq(&a->c0, &b->c0) && fp_eq(&a->c1, &b->c1); }
static void f2_inv(fp2* r, const fp2* a) {
  fp n, t, ni;
  fp_sqr(&n, &a->c0);
  fp_sqr(&t, &a->c1);
  fp_add(&n, &n, &t);
  fp_inv(&ni, &n);
  fp_mul(&r->c0, &a->c0, &ni);
  fp_mul(&t, &a->c1, &ni);
  fp_neg(&r->c1, &t);
}
static void f2_pow_words(fp2* r, const fp2* a, const uint64_t* e, int nw) {
  fp2 acc;
  f2_one(&acc);
  for (int w = nw - 1; w >= 0; --w)
    for (int b = 63; b >= 0; --b) {
      f2_sqr(&acc, &acc);
      if ((e[w] >> b) & 1) f2_mul(&acc, &acc, a);
    }
  *r = acc;
}
static int f2_is_square(const fp2* a) {
  fp n, t;
  fp_sqr(&n, &a->c0);
  fp_sqr(&t, &a->c1);
  fp_add(&n, &n, &t);
  return fp_is_square(&n);
}
static fp INV2;
/* some square root of a, or 0 (callers fix the sign) -- bls12_381.py f2_sqrt */
static int f2_sqrt(fp2* r, const fp2* a) {
  if (f2_is_zero(a)) {
    f2_zero(r);
    return 1;
  }
  if (fp_is_zero(&a->c1)) {
    fp s, na;
    if (fp_sqrt(&s, &a->c0)) {
      r->c0 = s;
      fp_zero(&r->c1);
      return 1;
    }
    fp_neg(&na, &a->c0);
    if (fp_sqrt(&s, &na)) {
      fp_zero(&r->c0);
      r->c1 = s;
      return 1;
    }
    return 0;
  }
  fp n, t, nr;
  fp_sqr(&n, &a->c0);
  fp_sqr(&t, &a->c1);
  fp_add(&n, &n, &t);
  if (!fp_sqrt(&nr, &n)) return 0;
  for (int k = 0; k < 2; ++k) {
    fp cand, x0, x1, d, di;
    if (k == 0) fp_add(&cand, &a->c0, &nr);
    else fp_sub(&cand, &a->c0, &nr);
    fp_mul(&cand, &cand, &INV2);
    if (!fp_sqrt(&x0, &cand) || fp_is_zero(&x0)) continue;
    fp_add(&d, &x0, &x0);
    fp_inv(&di, &d);
    fp_mul(&x1, &a->c1, &di);
    fp2 rr = {x0, x1}, chk;
    f2_sqr(&chk, &rr);
    if (f2_eq(&chk, a)) {
      *r = rr;
      return 1;
    }
  }
  return 0;
}
static int f2_sgn0(const fp2* a) {
  int s0 = fp_sgn0(&a->c0), z0 = fp_is_zero(&a->c0), s1 = fp_sgn0(&a->c1);
  return s0 | (z0 & s1);
}
static int f2_lex_largest(const fp2* a) {
  if (!fp_is_zero(&a->c1)) return fp_lex_largest(&a->c1);
  return fp_lex_largest(&a->c0);
}
static fp B1;      /* 4 */
static fp2 B2;     /* 4 + 4u */
static fp2 B2_3;   /* 3 b' */
static void fp_add_b(fp* r, const fp* a) { fp_add(r, a, &B1); }
static void f2_add_b(fp2* r, const fp2* a) { f2_add(r, a, &B2); }

/* ------------------------------------------------------------------------------ Fp6, Fp12 */
typedef struct {
  fp2 c0, c1, c2;
} fp6;
typedef struct {
  fp6 c0, c1;
} fp12;

static void f6_add(fp6* r, const fp6* a, const fp6* b) {
  f2_add(&r->c0, &a->c0, &b->c0);
  f2_add(&r->c1, &a->c1, &b->c1);
  f2_add(&r->c2, &a->c2, &b->c2);
}
static void f6_sub(fp6* r, const fp6* a, const fp6* b) {
  f2_sub(&r->c0, &a->c0, &b->c0);
  f2_sub(&r->c1, &a->c1, &b->c1);
  f2_sub(&r->c2, &a->c2, &b->c2);
}
static void f6_neg(fp6* r, const fp6* a) {
  f2_neg(&r->c0, &a->c0);
  f2_neg(&r->c1, &a->c1);
  f2_neg(&r->c2, &a->c2);
}
static void f6_mul(fp6* r, const fp6* a, const fp6* b) {
  fp2 t0, t1, t2, s, u, v, c0, c1, c2;
  f2_mul(&t0, &a->c0, &b->c0);
  f2_mul(&t1, &a->c1, &b->c1);
  f2_mul(&t2, &a->c2, &b->c2);
  f2_add(&s, &a->c1, &a->c2);
  f2_add(&u, &b->c1, &b->c2);
  f2_mul(&v, &s, &u);
  f2_sub(&v, &v, &t1);
  f2_sub(&v, &v, &t2);
  f2_mul_xi(&v, &v);
  f2_add(&c0, &t0, &v);
  f2_add(&s, &a->c0, &a->c1);
  f2_add(&u, &b->c0, &b->c1);
  f2_mul(&v, &s, &u);
  f2_sub(&v, &v, &t0);
  f2_sub(&v, &v, &t1);
  f2_mul_xi(&s, &t2);
  f2_add(&c1, &v, &s);
  f2_add(&s, &a->c0, &a->c2);
  f2_add(&u, &b->c0, &b->c2);
  f2_mul(&v, &s, &u);
  f2_sub(&v, &v, &t0);
  f2_sub(&v, &v, &t2);
  f2_add(&c2, &v, &t1);
  r->c0 = c0;
  r->c1 = c1;
  r->c2 = c2;
}
static void f6_mul_v(fp6* r, const fp6* a) {
  fp2 t;
  f2_mul_xi(&t, &a->c2);
  r->c2 = a->c1;
  r->c1 = a->c0;
  r->c0 = t;
}
static void f6_inv(fp6* r, const fp6* a) {
  fp2 c0, c1, c2, t, s;
  f2_sqr(&c0, &a->c0);
  f2_mul(&t, &a->c1, &a->c2);
  f2_mul_xi(&t, &t);
  f2_sub(&c0, &c0, &t);
  f2_sqr(&c1, &a->c2);
  f2_mul_xi(&c1, &c1);
  f2_mul(&t, &a->c0, &a->c1);
  f2_sub(&c1, &c1, &t);
  f2_sqr(&c2, &a->c1);
  f2_mul(&t, &a->c0, &a->c2);
  f2_sub(&c2, &c2, &t);
  f2_mul(&t, &a->c2, &c1);
  f2_mul(&s, &a->c1, &c2);
  f2_add(&t, &t, &s);
  f2_mul_xi(&t, &t);
  f2_mul(&s, &a->c0, &c0);
  f2_add(&t, &t, &s);
  f2_inv(&t, &t);
  f2_mul(&r->c0, &c0, &t);
  f2_mul(&r->c1, &c1, &t);
  f2_mul(&r->c2, &c2, &t);
}
static void f12_one(fp12* r) {
  memset(r, 0, sizeof(*r));
  r->c0.c0.c0 = ONE;
}
static void f12_mul(fp12* r, const fp12* a, const fp12* b) {
  fp6 t0, t1, s, u, c0, c1;
  f6_mul(&t0, &a->c0, &b->c0);
  f6_mul(&t1, &a->c1, &b->c1);
  f6_mul_v(&c0, &t1);
  f6_add(&c0, &c0, &t0);
  f6_add(&s, &a->c0, &a->c1);
  f6_add(&u, &b->c0, &b->c1);
  f6_mul(&c1, &s, &u);
  f6_sub(&c1, &c1, &t0);
  f6_sub(&c1, &c1, &t1);
  r->c0 = c0;
  r->c1 = c1;
}
static void f12_sqr(fp12* r, const fp12* a) { f12_mul(r, a, a); }
static void f12_conj(fp12* r, const fp12* a) {
  r->c0 = a->c0;
  f6_neg(&r->c1, &a->c1);
}
static void f12_inv(fp12* r, const fp12* a) {
  fp6 t, s, ti;
  f6_mul(&t, &a->c0, &a->c0);
  f6_mul(&s, &a->c1, &a->c1);
  f6_mul_v(&s, &s);
  f6_sub(&t, &t, &s);
  f6_inv(&ti, &t);
  f6_mul(&r->c0, &a->c0, &ti);
  f6_mul(&s, &a->c1, &ti);
  f6_neg(&r->c1, &s);
}
static int f12_is_one(const fp12* a) {
  fp12 one;
  f12_one(&one);
  return memcmp(a, &one, sizeof(fp12)) == 0;
}
static fp2 GAMMA[6]; /* xi^(k (p-1)/6) */
static void f12_frob(fp12* r, const fp12* a) {
  /* coefficient of w^k: c0.c0 (0), c1.c0 (1), c0.c1 (2), c1.c1 (3), c0.c2 (4), c1.c2 (5) */
  const fp2* in[6] = {&a->c0.c0, &a->c1.c0, &a->c0.c1, &a->c1.c1, &a->c0.c2, &a->c1.c2};
  fp2 out[6];
  for (int k = 0; k < 6; ++k) {
    fp2 c;
    f2_conj(&c, in[k]);
    f2_mul(&out[k], &c, &GAMMA[k]);
  }
  r->c0.c0 = out[0];
  r->c1.c0 = out[1];
  r->c0.c1 = out[2];
  r->c1.c1 = out[3];
  r->c0.c2 = out[4];
  r->c1.c2 = out[5];
}

/* ------------------------------------------------------------------------------ curves */
#define FT fp
#define F(x) fp_##x
#define PT_(x) g1_##x
#include "ec_impl.h"
#undef FT
#undef F
#undef PT_

#define fp2_one f2_one
#define fp2_zero f2_zero
#define fp2_is_zero f2_is_zero
#define fp2_inv f2_inv
#define fp2_sqr f2_sqr
#define fp2_mul f2_mul
#define fp2_add f2_add
#define fp2_sub f2_sub
#define fp2_neg f2_neg
#define fp2_eq f2_eq
#define fp2_add_b f2_add_b
#define FT fp2
#define F(x) fp2_##x
#define PT_(x) g2_##x
#include "ec_impl.h"
#undef FT
#undef F
#undef PT_

static const uint64_t X_ABS = 0xd201000000010000ull; /* BLS parameter x = -X_ABS */
static g1_jac G1_GEN_J, G1_NEG_J;
static g1_aff G1_NEG_A;
static g2_aff G2_GEN_A;
static fp BETA;       /* cube root of unity for the G1 endomorphism */
static fp2 PSI_CX, PSI_CY;

static void g2_psi(g2_jac* r, const g2_jac* p) {
  /* psi(X, Y, Z) = (conj(X) cx, conj(Y) cy, conj(Z)) in Jacobian coordinates */
  fp2 x, y, z;
  f2_conj(&x, &p->X);
  f2_conj(&y, &p->Y);
  f2_conj(&z, &p->Z);
  f2_mul(&r->X, &x, &PSI_CX);
  f2_mul(&r->Y, &y, &PSI_CY);
  r->Z = z;
}

/* Scott 2021: Q in G2 <=> psi(Q) == [x] Q   (bls12_381.py g2_in_subgroup_fast) */
static int g2_in_group(const g2_jac* q) {
  if (g2_is_inf(q)) return 1;
  g2_jac a, b;
  g2_psi(&a, q);
  g2_mul_words(&b, q, &X_ABS, 1);
  g2_neg(&b, &b);
  return g2_eq(&a, &b);
}

/* P in G1 <=> (beta x, y) == [-x^2] P   (bls12_381.py g1_in_subgroup_fast) */
static int g1_in_group(const g1_jac* p) {
  if (g1_is_inf(p)) return 1;
  const u128 x2 = (u128)X_ABS * X_ABS;
  const uint64_t k[2] = {(uint64_t)x2, (uint64_t)(x2 >> 64)};
  g1_jac a, b;
  g1_mul_words(&b, p, k, 2);
  g1_neg(&b, &b);
  a = *p;
  fp_mul(&a.X, &p->X, &BETA);
  return g1_eq(&a, &b);
}

/* ------------------------------------------------------------------------------ serialization */
enum { OK = 0, BAD_ENCODING = 1, NOT_ON_CURVE = 2, NOT_IN_GROUP = 3, AGGR_TYPE_MISMATCH = 4, VERIFY_FAIL = 5,
       PK_IS_INFINITY = 6, ERR_HASH_LEN = 100, ERR_LEN_MISMATCH = 101, ERR_PUBKEY = 102, ERR_ARG = 103 };

static int all_zero(const uint8_t* b, size_t n) {
  for (size_t i = 0; i < n; ++i)
    if (b[i]) return 0;
  return 1;
}

static int fp_read(fp* r, const uint8_t* b48, int mask_top) {
  uint8_t t[48];
  memcpy(t, b48, 48);
  if (mask_top) t[0] &= 0x1f;
  uint64_t v[6];
  be48_to_limbs(v, t);
  if (limbs_geq_p(v)) return 0;
  fp_from_plain(r, v);
  return 1;
}

static void fp_write(uint8_t* b48, const fp* a) {
  uint64_t v[6];
  fp_to_plain(v, a);
  limbs_to_be48(b48, v);
}

/* blst PublicKey::from_bytes semantics (bls12_381.py g1_from_bytes) */
static int g1_decode(g1_aff* out, const uint8_t* b, size_t len) {
  if (!((len == 48 && (b[0] & 0x80)) || (len == 96 && !(b[0] & 0x80)))) return BAD_ENCODING;
  if (b[0] & 0x40) {
    if ((b[0] & 0x3f) == 0 && all_zero(b + 1, len - 1)) {
      out->inf = 1;
      fp_zero(&out->x);
      fp_zero(&out->y);
      return OK;
    }
    return BAD_ENCODING;
  }
  out->inf = 0;
  if (len == 48) {
    if (!fp_read(&out->x, b, 1)) return BAD_ENCODING;
    fp rhs, t;
    fp_sqr(&t, &out->x);
    fp_mul(&rhs, &t, &out->x);
    fp_add_b(&rhs, &rhs);
    if (!fp_sqrt(&out->y, &rhs)) return NOT_ON_CURVE;
    if (fp_lex_largest(&out->y) != !!(b[0] & 0x20)) fp_neg(&out->y, &out->y);
  } else {
    if (b[0] & 0x20) return BAD_ENCODING;
    if (!fp_read(&out->x, b, 1) || !fp_read(&out->y, b + 48, 0)) return BAD_ENCODING;
    if (!g1_on_curve(out)) return NOT_ON_CURVE;
  }
  if (fp_is_zero(&out->x)) return NOT_IN_GROUP;
  return OK;
}

static int g2_decode(g2_aff* out, const uint8_t* b, size_t len) {
  if (!((len == 96 && (b[0] & 0x80)) || (len == 192 && !(b[0] & 0x80)))) return BAD_ENCODING;
  if (b[0] & 0x40) {
    if ((b[0] & 0x3f) == 0 && all_zero(b + 1, len - 1)) {
      out->inf = 1;
      f2_zero(&out->x);
      f2_zero(&out->y);
      return OK;
    }
    return BAD_ENCODING;
  }
  out->inf = 0;
  if (!fp_read(&out->x.c1, b, 1) || !fp_read(&out->x.c0, b + 48, 0)) return BAD_ENCODING;
  if (len == 96) {
    fp2 rhs, t;
    f2_sqr(&t, &out->x);
    f2_mul(&rhs, &t, &out->x);
    f2_add_b(&rhs, &rhs);
    if (!f2_sqrt(&out->y, &rhs)) return NOT_ON_CURVE;
    if (f2_lex_largest(&out->y) != !!(b[0] & 0x20)) f2_neg(&out->y, &out->y);
  } else {
    if (b[0] & 0x20) return BAD_ENCODING;
    if (!fp_read(&out->y.c1, b + 96, 0) || !fp_read(&out->y.c0, b + 144, 0)) return BAD_ENCODING;
    if (!g2_on_curve(out)) return NOT_ON_CURVE;
  }
  if (f2_is_zero(&out->x)) return NOT_IN_GROUP;
  return OK;
}

static void g1_compress(uint8_t* out, const g1_jac* p) {
  if (g1_is_inf(p)) {
    memset(out, 0, 48);
    out[0] = 0xc0;
    return;
  }
  g1_aff a;
  g1_to_aff(&a, p);
  fp_write(out, &a.x);
  out[0] |= 0x80 | (fp_lex_largest(&a.y) ? 0x20 : 0);
}

static void g2_compress(uint8_t* out, const g2_jac* p) {
  if (g2_is_inf(p)) {
    memset(out, 0, 96);
    out[0] = 0xc0;
    return;
  }
  g2_aff a;
  g2_to_aff(&a, p);
  fp_write(out, &a.x.c1);
  fp_write(out + 48, &a.x.c0);
  out[0] |= 0x80 | (f2_lex_largest(&a.y) ? 0x20 : 0);
}

static void g2_serialize(uint8_t* out, const g2_jac* p) {
  if (g2_is_inf(p)) {
    memset(out, 0, 192);
    out[0] = 0x40;
    return;
  }
  g2_aff a;
  g2_to_aff(&a, p);
  fp_write(out, &a.x.c1);
  fp_write(out + 48, &a.x.c0);
  fp_write(out + 96, &a.y.c1);
  fp_write(out + 144, &a.y.c0);
}

/* ------------------------------------------------------------------------------ SHA-256 */
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5, 0xd807aa98,
    0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786,
    0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8,
    0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13,
    0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819,
    0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a,
    0x5b9cca4f, 0x682e6ff3, 0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
    0xc67178f2};
#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))
static void sha256_block(uint32_t* h, const uint8_t* p) {
  uint32_t w[64];
  for (int i = 0; i < 16; ++i) w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
  for (int i = 16; i < 64; ++i) {
    uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int i = 0; i < 64; ++i) {
    uint32_t S1 = ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25), ch = (e & f) ^ (~e & g);
    uint32_t t1 = hh + S1 + ch + K256[i] + w[i];
    uint32_t S0 = ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22), mj = (a & b) ^ (a & c) ^ (b & c);
    uint32_t t2 = S0 + mj;
    hh = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  h[0] += a;
  h[1] += b;
  h[2] += c;
  h[3] += d;
  h[4] += e;
  h[5] += f;
  h[6] += g;
  h[7] += hh;
}
static void sha256(uint8_t out[32], const uint8_t* m, size_t len) {
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  size_t i = 0;
  for (; i + 64 <= len; i += 64) sha256_block(h, m + i);
  uint8_t tail[128];
  size_t r = len - i;
  memset(tail, 0, sizeof(tail));
  memcpy(tail, m + i, r);
  tail[r] = 0x80;
  size_t tl = (r + 9 <= 64) ? 64 : 128;
  uint64_t bits = (uint64_t)len * 8;
  for (int k = 0; k < 8; ++k) tail[tl - 1 - k] = (uint8_t)(bits >> (8 * k));
  sha256_block(h, tail);
  if (tl == 128) sha256_block(h, tail + 64);
  for (int k = 0; k < 8; ++k) {
    out[4 * k] = (uint8_t)(h[k] >> 24);
    out[4 * k + 1] = (uint8_t)(h[k] >> 16);
    out[4 * k + 2] = (uint8_t)(h[k] >> 8);
    out[4 * k + 3] = (uint8_t)h[k];
  }
}

/* RFC 9380 5.3.1 expand_message_xmd(SHA-256); len_in_bytes <= 255*32, dst_len <= 255 */
static int expand_message_xmd(uint8_t* out, size_t len_in_bytes, const uint8_t* msg, size_t msg_len,
                              const uint8_t* dst, size_t dst_len) {
  const size_t ell = (len_in_bytes + 31) / 32;
  if (ell > 255 || dst_len > 255) return -1;
  size_t n0 = 64 + msg_len + 2 + 1 + dst_len + 1;
  uint8_t* buf = (uint8_t*)malloc(n0 > 32 + 1 + 256 ? n0 : 32 + 1 + 256);
  if (!buf) return -1;
  memset(buf, 0, 64);
  memcpy(buf + 64, msg, msg_len);
  buf[64 + msg_len] = (uint8_t)(len_in_bytes >> 8);
  buf[64 + msg_len + 1] = (uint8_t)len_in_bytes;
  buf[64 + msg_len + 2] = 0;
  memcpy(buf + 64 + msg_len + 3, dst, dst_len);
  buf[64 + msg_len + 3 + dst_len] = (uint8_t)dst_len;
  uint8_t b0[32], bi[32];
  sha256(b0, buf, n0);
  for (size_t i = 1; i <= ell; ++i) {
    for (int k = 0; k < 32; ++k) buf[k] = (i == 1) ? b0[k] : (uint8_t)(b0[k] ^ bi[k]);
    buf[32] = (uint8_t)i;
    memcpy(buf + 33, dst, dst_len);
    buf[33 + dst_len] = (uint8_t)dst_len;
    sha256(bi, buf, 34 + dst_len);
    size_t take = len_in_bytes - (i - 1) * 32 < 32 ? len_in_bytes - (i - 1) * 32 : 32;
    memcpy(out + (i - 1) * 32, bi, take);
  }
  free(buf);
  return 0;
}

/* 64 big-endian bytes mod p, Montgomery: lo R + hi 2^384 R  (hi < 2^128) */
static void fp_from_be64(fp* r, const uint8_t* b) {
  uint64_t lo[6], hi[6] = {0};
  be48_to_limbs(lo, b + 16);
  for (int k = 0; k < 8; ++k) {
    hi[1] = (hi[1] << 8) | b[k];
    hi[0] = (hi[0] << 8) | b[8 + k];
  }
  fp a, c, t1, t2;
  memcpy(a.l, lo, 48);
  memcpy(c.l, hi, 48);
  fp_mul(&t1, &a, &R2);
  fp_mul(&t2, &c, &R3);
  fp_add(r, &t1, &t2);
}

/* ------------------------------------------------------------------------------ hash to G2 */
static fp2 SSWU_A, SSWU_B, SSWU_Z, SSWU_MB_OVER_A, SSWU_B_OVER_ZA;
static fp2 ISO_XNUM[4], ISO_XDEN[3], ISO_YNUM[4], ISO_YDEN[4];

static void g2p_rhs(fp2* r, const fp2* x) {
  fp2 t, u;
  f2_sqr(&t, x);
  f2_mul(&t, &t, x);
  f2_mul(&u, &SSWU_A, x);
  f2_add(&t, &t, &u);
  f2_add(r, &t, &SSWU_B);
}

/* RFC 9380 6.6.2 simplified SWU on E2' (bls12_381.py map_to_curve_sswu) */
static void map_to_curve_sswu(fp2* xo, fp2* yo, const fp2* u) {
  fp2 u2, zu2, tv1, x1, gx1, t, y;
  f2_sqr(&u2, u);
  f2_mul(&zu2, &SSWU_Z, &u2);
  f2_sqr(&tv1, &zu2);
  f2_add(&tv1, &tv1, &zu2);
  if (f2_is_zero(&tv1)) {
    x1 = SSWU_B_OVER_ZA;
  } else {
    f2_inv(&t, &tv1);
    fp2 one;
    f2_one(&one);
    f2_add(&t, &t, &one);
    f2_mul(&x1, &SSWU_MB_OVER_A, &t);
  }
  g2p_rhs(&gx1, &x1);
  if (f2_is_square(&gx1)) {
    *xo = x1;
    f2_sqrt(&y, &gx1);
  } else {
    fp2 x2, gx2;
    f2_mul(&x2, &zu2, &x1);
    g2p_rhs(&gx2, &x2);
    *xo = x2;
    f2_sqrt(&y, &gx2);
  }
  if (f2_sgn0(u) != f2_sgn0(&y)) f2_neg(&y, &y);
  *yo = y;
}

static void poly_eval(fp2* r, const fp2* c, int n, const fp2* x) {
  fp2 acc;
  f2_zero(&acc);
  for (int i = n - 1; i >= 0; --i) {
    f2_mul(&acc, &acc, x);
    f2_add(&acc, &acc, &c[i]);
  }
  *r = acc;
}

/* 3-isogeny E2' -> E2 (RFC 9380 E.3), to Jacobian (infinity when a denominator vanishes) */
static void iso_map(g2_jac* r, const fp2* x, const fp2* y) {
  fp2 xn, xd, yn, yd, t;
  poly_eval(&xd, ISO_XDEN, 3, x);
  poly_eval(&yd, ISO_YDEN, 4, x);
  if (f2_is_zero(&xd) || f2_is_zero(&yd)) {
    g2_set_inf(r);
    return;
  }
  poly_eval(&xn, ISO_XNUM, 4, x);
  poly_eval(&yn, ISO_YNUM, 4, x);
  f2_inv(&t, &xd);
  f2_mul(&r->X, &xn, &t);
  f2_inv(&t, &yd);
  f2_mul(&t, &yn, &t);
  f2_mul(&r->Y, y, &t);
  f2_one(&r->Z);
}

/* h_eff P = [x^2 - x - 1] P + [x - 1] psi(P) + psi^2(2P)  (Budroni-Pintore; RFC 9380 G.3) */
static void clear_cofactor(g2_jac* r, const g2_jac* p) {
  const u128 k1 = (u128)X_ABS * X_ABS + X_ABS - 1; /* x^2 - x - 1 with x = -X_ABS */
  const uint64_t w1[2] = {(uint64_t)k1, (uint64_t)(k1 >> 64)};
  const uint64_t w2 = X_ABS + 1; /* x - 1 = -(X_ABS + 1) */
  g2_jac t1, t2, t3, ps;
  g2_mul_words(&t1, p, w1, 2);
  g2_psi(&ps, p);
  g2_mul_words(&t2, &ps, &w2, 1);
  g2_neg(&t2, &t2);
  g2_dbl(&t3, p);
  g2_psi(&t3, &t3);
  g2_psi(&t3, &t3);
  g2_add(r, &t1, &t2);
  g2_add(r, r, &t3);
}

static int hash_to_g2(g2_jac* r, const uint8_t* msg, size_t len, const uint8_t* dst, size_t dst_len) {
  uint8_t ub[256];
  if (expand_message_xmd(ub, 256, msg, len, dst, dst_len)) return -1;
  fp2 u0, u1, x, y;
  fp_from_be64(&u0.c0, ub);
  fp_from_be64(&u0.c1, ub + 64);
  fp_from_be64(&u1.c0, ub + 128);
  fp_from_be64(&u1.c1, ub + 192);
  g2_jac q0, q1;
  map_to_curve_sswu(&x, &y, &u0);
  iso_map(&q0, &x, &y);
  map_to_curve_sswu(&x, &y, &u1);
  iso_map(&q1, &x, &y);
  g2_add(&q0, &q0, &q1);
  clear_cofactor(r, &q0);
  return 0;
}

/* ------------------------------------------------------------------------------ pairing */
/* f * (l0 + l1 v + l4 v w): the sparse line of the M-type twist */
static void f12_mul_line(fp12* f, const fp2* l0, const fp2* l1, const fp2* l4) {
  fp12 l;
  memset(&l, 0, sizeof(l));
  l.c0.c0 = *l0;
  l.c0.c1 = *l1;
  l.c1.c1 = *l4;
  f12_mul(f, f, &l);
}

/* Optimal-ate Miller loop with T projective (bls12_381.py miller_loop_proj) */
static void miller_loop(fp12* out, const g1_aff* p1, const g2_aff* q2) {
  if (p1->inf || q2->inf) {
    f12_one(out);
    return;
  }
  fp m3xp, m1xp, yp2, t;
  fp_add(&t, &p1->x, &p1->x);
  fp_add(&t, &t, &p1->x);
  fp_neg(&m3xp, &t);
  fp_neg(&m1xp, &p1->x);
  fp_add(&yp2, &p1->y, &p1->y);
  fp2 X = q2->x, Y = q2->y, Z;
  f2_one(&Z);
  fp12 f;
  f12_one(&f);
  int first = 1;
  for (int b = 62; b >= 0; --b) {
    fp2 XX, YY, ZZ, E, l0, l1, l4, A, Fv, X3, Y3, Z3, G, s, u;
    f2_sqr(&XX, &X);
    f2_sqr(&YY, &Y);
    f2_sqr(&ZZ, &Z);
    f2_mul(&E, &B2_3, &ZZ);
    f2_sub(&l0, &YY, &E);
    f2_mul_fp(&l1, &XX, &m3xp);
    f2_mul(&s, &Y, &Z);
    f2_mul_fp(&l4, &s, &yp2);
    f2_mul(&A, &X, &Y);
    f2_add(&Fv, &E, &E);
    f2_add(&Fv, &Fv, &E);
    f2_sub(&u, &YY, &Fv);
    f2_mul(&X3, &A, &u);
    f2_add(&X3, &X3, &X3);
    f2_add(&G, &YY, &Fv);
    f2_sqr(&Y3, &G);
    f2_sqr(&u, &E);
    fp2 u12;
    f2_add(&u12, &u, &u);     /* 2 */
    f2_add(&u12, &u12, &u);   /* 3 */
    f2_add(&u12, &u12, &u12); /* 6 */
    f2_add(&u12, &u12, &u12); /* 12 */
    f2_sub(&Y3, &Y3, &u12);
    f2_mul(&Z3, &YY, &s);
    f2_add(&Z3, &Z3, &Z3);
    f2_add(&Z3, &Z3, &Z3);
    f2_add(&Z3, &Z3, &Z3);
    X = X3;
    Y = Y3;
    Z = Z3;
    if (!first) f12_sqr(&f, &f);
    first = 0;
    f12_mul_line(&f, &l0, &l1, &l4);
    if ((X_ABS >> b) & 1) {
      fp2 theta, lam, C, D, Ee, Fz, H;
      f2_mul(&s, &q2->y, &Z);
      f2_sub(&theta, &Y, &s);
      f2_mul(&s, &q2->x, &Z);
      f2_sub(&lam, &X, &s);
      f2_mul(&s, &theta, &q2->x);
      f2_mul(&u, &lam, &q2->y);
      f2_sub(&l0, &s, &u);
      f2_mul_fp(&l1, &theta, &m1xp);
      f2_mul_fp(&l4, &lam, &p1->y);
      f2_sqr(&C, &theta);
      f2_sqr(&D, &lam);
      f2_mul(&Ee, &D, &lam);
      f2_mul(&Fz, &Z, &C);
      f2_mul(&G, &X, &D);
      f2_add(&H, &Ee, &Fz);
      f2_sub(&H, &H, &G);
      f2_sub(&H, &H, &G);
      f2_mul(&X3, &lam, &H);
      f2_sub(&s, &G, &H);
      f2_mul(&Y3, &theta, &s);
      f2_mul(&s, &Y, &Ee);
      f2_sub(&Y3, &Y3, &s);
      f2_mul(&Z3, &Z, &Ee);
      X = X3;
      Y = Y3;
      Z = Z3;
      f12_mul_line(&f, &l0, &l1, &l4);
    }
  }
  f12_conj(out, &f);
}

static void f12_exp_x(fp12* r, const fp12* f) { /* f^x, f cyclotomic (x < 0 -> conjugate) */
  fp12 acc = *f;
  for (int b = 62; b >= 0; --b) {
    f12_sqr(&acc, &acc);
    if ((X_ABS >> b) & 1) f12_mul(&acc, &acc, f);
  }
  f12_conj(r, &acc);
}

/* f^(3 (p^12 - 1)/r) via 3 Phi12(p)/r = (x-1)^2 (x+p) (x^2+p^2-1) + 3
 * (bls12_381.py final_exponentiation_x_chain); is_one is unaffected by the cube. */
static void final_exp(fp12* r, const fp12* fin) {
  fp12 f, t, u, v;
  f12_conj(&t, fin);
  f12_inv(&u, fin);
  f12_mul(&f, &t, &u);
  f12_frob(&t, &f);
  f12_frob(&t, &t);
  f12_mul(&f, &t, &f);
  /* t = f^(x-1)^2 */
  f12_exp_x(&t, &f);
  f12_conj(&u, &f);
  f12_mul(&t, &t, &u);
  f12_exp_x(&u, &t);
  f12_conj(&v, &t);
  f12_mul(&t, &u, &v);
  /* t = t^(x+p) */
  f12_exp_x(&u, &t);
  f12_frob(&v, &t);
  f12_mul(&t, &u, &v);
  /* t = t^(x^2+p^2-1) */
  f12_exp_x(&u, &t);
  f12_exp_x(&u, &u);
  f12_frob(&v, &t);
  f12_frob(&v, &v);
  f12_mul(&u, &u, &v);
  f12_conj(&v, &t);
  f12_mul(&t, &u, &v);
  /* * f^3 */
  f12_sqr(&u, &f);
  f12_mul(&u, &u, &f);
  f12_mul(r, &t, &u);
}

/* ------------------------------------------------------------------------------ init */
static const char* ISO_HEX[15][2] = {
    /* XNUM k0..k3 */
    {"5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6",
     "5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6"},
    {"0", "11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71a"},
    {"11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71e",
     "8ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38d"},
    {"171d6541fa38ccfaed6dea691f5fb614cb14b4e7f4e810aa22d6108f142b85757098e38d0f671c7188e2aaaaaaaa5ed1", "0"},
    /* XDEN k0..k2 */
    {"0", "1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaa63"},
    {"c", "1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaa9f"},
    {"1", "0"},
    /* YNUM k0..k3 */
    {"1530477c7ab4113b59a4c18b076d11930f7da5d4a07f649bf54439d87d27e500fc8c25ebf8c92f6812cfc71c71c6d706",
     "1530477c7ab4113b59a4c18b076d11930f7da5d4a07f649bf54439d87d27e500fc8c25ebf8c92f6812cfc71c71c6d706"},
    {"0", "5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97be"},
    {"11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71c",
     "8ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38f"},
    {"124c9ad43b6cf79bfbf7043de3811ad0761b0f37a1e26286b0e977c69aa274524e79097a56dc4bd9e1b371c71c718b10", "0"},
    /* YDEN k0..k3 */
    {"1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffa8fb",
     "1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffa8fb"},
    {"0", "1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffa9d3"},
    {"12", "1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaa99"},
    {"1", "0"},
};

static void f2_hex(fp2* r, const char* a, const char* b) {
  fp_from_hex(&r->c0, a);
  fp_from_hex(&r->c1, b);
}

static void init_once(void) {
  /* -p^-1 mod 2^64 by Newton iteration */
  uint64_t inv = 1;
  for (int i = 0; i < 7; ++i) inv *= 2 - P[0] * inv;
  PINV = (uint64_t)0 - inv;
#if defined(__x86_64__)
  {
    const char* off = getenv("ORC_NO_MULX");
    g_mulx = __builtin_cpu_supports("bmi2") && __builtin_cpu_supports("adx") && !(off && *off && *off != '0');
  }
#endif
  /* R mod p, R^2, R^3 by doubling (plain arithmetic on limbs) */
  uint64_t v[6] = {1, 0, 0, 0, 0, 0};
  for (int k = 0; k < 384 * 2; ++k) {
    uint64_t c = 0;
    for (int i = 0; i < 6; ++i) {
      uint64_t nv = (v[i] << 1) | c;
      c = v[i] >> 63;
      v[i] = nv;
    }
    if (c || limbs_geq_p(v)) sub_p(v);
    if (k == 383) memcpy(ONE.l, v, 48);
  }
  memcpy(R2.l, v, 48);
  fp_mul(&R3, &R2, &R2); /* R^2 R^2 / R = R^3 */
  /* exponents */
  memcpy(E_PM2, P, 48);
  E_PM2[0] -= 2;
  memcpy(E_LEG, P, 48);
  E_LEG[0] -= 1;
  for (int i = 0; i < 6; ++i) E_LEG[i] = (E_LEG[i] >> 1) | (i < 5 ? E_LEG[i + 1] << 63 : 0);
  memcpy(E_SQRT, P, 48);
  E_SQRT[0] += 1; /* no carry: P[0] is odd and != 2^64-1 */
  for (int i = 0; i < 6; ++i) E_SQRT[i] = (E_SQRT[i] >> 2) | (i < 5 ? E_SQRT[i + 1] << 62 : 0);
  fp_small(&INV2, 2);
  fp_inv(&INV2, &INV2);
  fp_small(&B1, 4);
  B2.c0 = B1;
  B2.c1 = B1;
  f2_add(&B2_3, &B2, &B2);
  f2_add(&B2_3, &B2_3, &B2);
  /* Frobenius constants gamma_k = xi^(k (p-1)/6) */
  {
    uint64_t e[6];
    memcpy(e, P, 48);
    e[0] -= 1;
    /* e /= 6 */
    u128 rem = 0;
    for (int i = 5; i >= 0; --i) {
      u128 cur = (rem << 64) | e[i];
      e[i] = (uint64_t)(cur / 6);
      rem = cur % 6;
    }
    fp2 xi;
    xi.c0 = ONE;
    xi.c1 = ONE;
    fp2 g1;
    f2_pow_words(&g1, &xi, e, 6);
    f2_one(&GAMMA[0]);
    for (int k = 1; k < 6; ++k) f2_mul(&GAMMA[k], &GAMMA[k - 1], &g1);
    f2_inv(&PSI_CX, &GAMMA[2]); /* xi^((p-1)/3) */
    f2_inv(&PSI_CY, &GAMMA[3]); /* xi^((p-1)/2) */
  }
  /* generators */
  {
    g1_aff g;
    fp_from_hex(&g.x, "17f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb");
    fp_from_hex(&g.y, "08b3f481e3aaa0f1a09e30ed741d8ae4fcf5e095d5d00af600db18cb2c04b3edd03cc744a2888ae40caa232946c5e7e1");
    g.inf = 0;
    g1_from_aff(&G1_GEN_J, &g);
    g1_neg(&G1_NEG_J, &G1_GEN_J);
    G1_NEG_A = g;
    fp_neg(&G1_NEG_A.y, &g.y);
    f2_hex(&G2_GEN_A.x, "024aa2b2f08f0a91260805272dc51051c6e47ad4fa403b02b4510b647ae3d1770bac0326a805bbefd48056c8c121bdb8",
           "13e02b6052719f607dacd3a088274f65596bd0d09920b61ab5da61bbdc7f5049334cf11213945d57e5ac7d055d042b7e");
    f2_hex(&G2_GEN_A.y, "0ce5d527727d6e118cc9cdc6da2e351aadfd9baa8cbdd3a76d429a695160d12c923ac9cc3baca289e193548608b82801",
           "0606c4a02ea734cc32acd2b02bc28b99cb3e287e85a763af267492ab572e99ab3f370d275cec1da1aaa9075ff05f79be");
    G2_GEN_A.inf = 0;
  }
  /* beta: the cube root of unity with phi(G1) == [-x^2] G1 */
  {
    uint64_t e[6];
    memcpy(e, P, 48);
    e[0] -= 1;
    u128 rem = 0;
    for (int i = 5; i >= 0; --i) {
      u128 cur = (rem << 64) | e[i];
      e[i] = (uint64_t)(cur / 3);
      rem = cur % 3;
    }
    fp two, b0, b1;
    fp_small(&two, 2);
    fp_pow(&b0, &two, e);
    fp_sqr(&b1, &b0);
    BETA = b0;
    if (!g1_in_group(&G1_GEN_J)) BETA = b1;
  }
  /* SSWU constants for E2': A' = 240 u, B' = 1012 (1 + u), Z = -(2 + u) */
  {
    fp_zero(&SSWU_A.c0);
    fp_small(&SSWU_A.c1, 240);
    fp_small(&SSWU_B.c0, 1012);
    SSWU_B.c1 = SSWU_B.c0;
    fp two, one;
    fp_small(&two, 2);
    fp_small(&one, 1);
    fp_neg(&SSWU_Z.c0, &two);
    fp_neg(&SSWU_Z.c1, &one);
    fp2 t;
    f2_inv(&t, &SSWU_A);
    f2_mul(&t, &SSWU_B, &t);
    f2_neg(&SSWU_MB_OVER_A, &t);
    f2_mul(&t, &SSWU_Z, &SSWU_A);
    f2_inv(&t, &t);
    f2_mul(&SSWU_B_OVER_ZA, &SSWU_B, &t);
  }
  for (int i = 0; i < 4; ++i) f2_hex(&ISO_XNUM[i], ISO_HEX[i][0], ISO_HEX[i][1]);
  for (int i = 0; i < 3; ++i) f2_hex(&ISO_XDEN[i], ISO_HEX[4 + i][0], ISO_HEX[4 + i][1]);
  for (int i = 0; i < 4; ++i) f2_hex(&ISO_YNUM[i], ISO_HEX[7 + i][0], ISO_HEX[7 + i][1]);
  for (int i = 0; i < 4; ++i) f2_hex(&ISO_YDEN[i], ISO_HEX[11 + i][0], ISO_HEX[11 + i][1]);
}

static pthread_once_t ONCE = PTHREAD_ONCE_INIT;
static void init(void) { pthread_once(&ONCE, init_once); }

/* ------------------------------------------------------------------------------ API */
static const uint8_t DEFAULT_DST[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_";
static const uint8_t* g_dst = DEFAULT_DST;
static size_t g_dst_len = 43;

/* Which Montgomery product the oracle runs (1: mulx / ADX asm, 0: portable CIOS). */
int orc_mulx_active(void) {
  init();
  return g_mulx;
}

/* The mulx product against the portable CIOS on n pseudo-random canonical operand pairs (and
 * the edge values 0, 1, p - 1): the number of mismatches (0 when the mulx form is unavailable). */
int orc_mulx_selftest(uint64_t seed, int n) {
  init();
  int bad = 0;
#if defined(__x86_64__)
  if (!(__builtin_cpu_supports("bmi2") && __builtin_cpu_supports("adx"))) return 0;
  uint64_t x = seed | 1;
  for (int k = 0; k < n + 9; ++k) {
    fp a, b, r1, r2;
    for (int h = 0; h < 2; ++h) {
      fp* t = h ? &b : &a;
      const int e = k < 9 ? (h ? k % 3 : k / 3) : -1;
      if (e >= 0) { /* 0, 1, p - 1 */
        memset(t->l, 0, 48);
        if (e == 1) t->l[0] = 1;
        if (e == 2) { memcpy(t->l, P, 48); t->l[0] -= 1; }
        continue;
      }
      for (int i = 0; i < 6; ++i) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        t->l[i] = x;
      }
      t->l[5] &= (1ull << 61) - 1;
      while (limbs_geq_p(t->l)) sub_p(t->l);
    }
    fp_mul_cios(&r1, &a, &b);
    fp_mul_mulx(r2.l, a.l, b.l, P, PINV);
    bad += memcmp(r1.l, r2.l, 48) != 0;
  }
#endif
  return bad;
}

void orc_set_dst(const uint8_t* dst, size_t len) {
  static uint8_t buf[256];
  if (!dst || len > 255) {
    g_dst = DEFAULT_DST;
    g_dst_len = 43;
    return;
  }
  memcpy(buf, dst, len);
  g_dst = buf;
  g_dst_len = len;
}

int orc_hash_to_g2(const uint8_t* msg, size_t len, uint8_t out192[192]) {
  init();
  g2_jac h;
  if (hash_to_g2(&h, msg, len, g_dst, g_dst_len)) return ERR_ARG;
  g2_serialize(out192, &h);
  return OK;
}

static int sk_parse(uint64_t k[4], const uint8_t* sk, size_t len) {
  static const uint8_t R_BE[32] = {0x73, 0xed, 0xa7, 0x53, 0x29, 0x9d, 0x7d, 0x48, 0x33, 0x39, 0xd8,
                                   0x08, 0x09, 0xa1, 0xd8, 0x05, 0x53, 0xbd, 0xa4, 0x02, 0xff, 0xfe,
                                   0x5b, 0xfe, 0xff, 0xff, 0xff, 0xff, 0x00, 0x00, 0x00, 0x01};
  if (!sk || len != 32 || all_zero(sk, 32) || memcmp(sk, R_BE, 32) >= 0) return BAD_ENCODING;
  for (int i = 0; i < 4; ++i) {
    uint64_t x = 0;
    for (int b = 0; b < 8; ++b) x = (x << 8) | sk[24 - 8 * i + b];
    k[i] = x;
  }
  return OK;
}

/* ophelia-blst BlsPrivateKey::try_from (consensus.rs:349-350) [dep]: blst SecretKey::key_gen(ikm,
 * "") = IETF KeyGen (draft-irtf-cfrg-bls-signature-04 2.3; = EIP-2333 HKDF_mod_r): salt =
 * SHA-256("BLS-SIG-KEYGEN-SALT-"); PRK = HKDF-Extract(salt, IKM || 0x00); OKM = HKDF-Expand(PRK,
 * 0x0030, 48); SK = OS2IP(OKM) mod r, re-hashing the salt while SK = 0. ikm >= 32 bytes. */
static void hmac_sha256(uint8_t out[32], const uint8_t* key, size_t klen, const uint8_t* msg, size_t mlen) {
  uint8_t k[64], buf[64 + 256], inner[32];
  memset(k, 0, sizeof k);
  if (klen > 64) sha256(k, key, klen);
  else memcpy(k, key, klen);
  if (mlen > 256) return; /* callers stay below */
  for (int i = 0; i < 64; ++i) buf[i] = k[i] ^ 0x36;
  memcpy(buf + 64, msg, mlen);
  sha256(inner, buf, 64 + mlen);
  for (int i = 0; i < 64; ++i) buf[i] = k[i] ^ 0x5c;
  memcpy(buf + 64, inner, 32);
  sha256(out, buf, 96);
}

static const uint8_t R_ORDER_BE[32] = {0x73, 0xed, 0xa7, 0x53, 0x29, 0x9d, 0x7d, 0x48, 0x33, 0x39, 0xd8,
                                       0x08, 0x09, 0xa1, 0xd8, 0x05, 0x53, 0xbd, 0xa4, 0x02, 0xff, 0xfe,
                                       0x5b, 0xfe, 0xff, 0xff, 0xff, 0xff, 0x00, 0x00, 0x00, 0x01};

/* out = OS2IP(in[0..48)) mod r: 384-bit value as 6 limbs, reduced by 128-bit arithmetic on the
 * 4-limb order with shift-and-subtract over the bits */
static void os2ip_mod_r(uint8_t out[32], const uint8_t in[48]) {
  uint64_t r[4], a[5] = {0, 0, 0, 0, 0};
  for (int i = 0; i < 4; ++i) {
    uint64_t x = 0;
    for (int b = 0; b < 8; ++b) x = (x << 8) | R_ORDER_BE[24 - 8 * i + b];
    r[i] = x;
  }
  for (int bit = 0; bit < 384; ++bit) {
    const uint64_t in_bit = (in[bit / 8] >> (7 - bit % 8)) & 1;
    for (int i = 4; i > 0; --i) a[i] = (a[i] << 1) | (a[i - 1] >> 63);
    a[0] = (a[0] << 1) | in_bit;
    int ge = a[4] != 0;
    if (!ge) {
      ge = 1;
      for (int i = 3; i >= 0; --i)
        if (a[i] != r[i]) {
          ge = a[i] > r[i];
          break;
        }
    }
    if (ge) {
      uint64_t br = 0;
      for (int i = 0; i < 4; ++i) {
        u128 d = (u128)a[i] - r[i] - br;
        a[i] = (uint64_t)d;
        br = (uint64_t)(d >> 64) & 1;
      }
      a[4] -= br;
    }
  }
  for (int i = 0; i < 4; ++i)
    for (int b = 0; b < 8; ++b) out[24 - 8 * i + b] = (uint8_t)(a[i] >> (56 - 8 * b));
}

int orc_sk_keygen(const uint8_t* ikm, size_t len, uint8_t out32[32]) {
  if (!ikm || len < 32 || len > 200 || !out32) return BAD_ENCODING;
  uint8_t salt[32], prk[32], okm[64], msg[256];
  sha256(salt, (const uint8_t*)"BLS-SIG-KEYGEN-SALT-", 20);
  for (;;) {
    memcpy(msg, ikm, len);
    msg[len] = 0; /* IKM || I2OSP(0, 1) */
    hmac_sha256(prk, salt, 32, msg, len + 1);
    /* T(1) = HMAC(PRK, info || 1), T(2) = HMAC(PRK, T(1) || info || 2); info = I2OSP(48, 2) */
    uint8_t m1[3] = {0x00, 0x30, 0x01}, m2[35];
    hmac_sha256(okm, prk, 32, m1, 3);
    memcpy(m2, okm, 32);
    m2[32] = 0x00;
    m2[33] = 0x30;
    m2[34] = 0x02;
    hmac_sha256(okm + 32, prk, 32, m2, 35);
    os2ip_mod_r(out32, okm);
    if (!all_zero(out32, 32)) return OK;
    sha256(salt, salt, 32);
  }
}

int orc_sk_to_pk(const uint8_t* sk, size_t sk_len, uint8_t out48[48]) {
  init();
  uint64_t k[4];
  int e = sk_parse(k, sk, sk_len);
  if (e) return e;
  g1_jac p;
  g1_mul_words(&p, &G1_GEN_J, k, 4);
  g1_compress(out48, &p);
  return OK;
}

int orc_sign(const uint8_t* sk, size_t sk_len, const uint8_t* hash, size_t hash_len, uint8_t out96[96]) {
  init();
  if (!hash || hash_len != 32) return ERR_HASH_LEN;
  uint64_t k[4];
  int e = sk_parse(k, sk, sk_len);
  if (e) return e;
  g2_jac h, s;
  hash_to_g2(&h, hash, 32, g_dst, g_dst_len);
  g2_mul_words(&s, &h, k, 4);
  g2_compress(out96, &s);
  return OK;
}

/* e(pk, H) == e(G1, sig) */
static int pairing_check(const g1_aff* pk, const g2_aff* h, const g2_aff* sig) {
  fp12 f1, f2;
  miller_loop(&f1, pk, h);
  miller_loop(&f2, &G1_NEG_A, sig);
  f12_mul(&f1, &f1, &f2);
  final_exp(&f1, &f1);
  return f12_is_one(&f1);
}

/* blst core_verify (min-pk, sig group-checked, pk validated) on parsed points
 * (bls12_381.py core_verify) */
static int core_verify(const g1_aff* pk, const g2_aff* sig, const uint8_t* msg, size_t msg_len) {
  if (!sig->inf) {
    g2_jac s;
    g2_from_aff(&s, sig);
    if (!g2_in_group(&s)) return NOT_IN_GROUP;
  }
  if (pk->inf) return PK_IS_INFINITY;
  g1_jac pj;
  g1_from_aff(&pj, pk);
  if (!g1_in_group(&pj)) return NOT_IN_GROUP;
  g2_jac hj;
  hash_to_g2(&hj, msg, msg_len, g_dst, g_dst_len);
  g2_aff h;
  g2_to_aff(&h, &hj);
  if (h.inf || sig->inf) {
    /* e(pk, H) * e(-G1, sig) with a factor at infinity: only 1 if both are */
    return (h.inf && sig->inf) ? OK : VERIFY_FAIL;
  }
  return pairing_check(pk, &h, sig) ? OK : VERIFY_FAIL;
}

/* ConsensusCrypto::verify_signature (consensus.rs:397-416): hash length, pk parse, sig parse,
 * then blst verify */
int orc_verify(const uint8_t* sig, size_t sig_len, const uint8_t* hash, size_t hash_len, const uint8_t* pk,
               size_t pk_len) {
  init();
  if (!hash || hash_len != 32) return ERR_HASH_LEN;
  g1_aff p;
  if (!pk || g1_decode(&p, pk, pk_len) != OK) return ERR_PUBKEY;
  g2_aff s;
  int e = sig ? g2_decode(&s, sig, sig_len) : BAD_ENCODING;
  if (e) return e;
  return core_verify(&p, &s, hash, 32);
}

/* ConsensusCrypto::aggregate_signatures (consensus.rs:418-444) */
int orc_aggregate_sigs(const uint8_t* sigs, const size_t* sig_lens, size_t n_sigs, const uint8_t* pks,
                       const size_t* pk_lens, size_t n_pks, uint8_t out96[96]) {
  init();
  if (n_sigs != n_pks) return ERR_LEN_MISMATCH;
  const size_t n = n_sigs;
  g2_aff* pts = (g2_aff*)malloc(sizeof(g2_aff) * (n ? n : 1));
  if (!pts) return ERR_ARG;
  size_t so = 0, po = 0;
  for (size_t i = 0; i < n; ++i) {
    int e = g2_decode(&pts[i], sigs + so, sig_lens[i]);
    if (e) {
      free(pts);
      return e;
    }
    g1_aff p;
    if (g1_decode(&p, pks + po, pk_lens[i]) != OK) {
      free(pts);
      return ERR_PUBKEY;
    }
    so += sig_lens[i];
    po += pk_lens[i];
  }
  if (n == 0) {
    free(pts);
    return AGGR_TYPE_MISMATCH;
  }
  g2_jac acc, t;
  g2_set_inf(&acc);
  for (size_t i = 0; i < n; ++i) {
    g2_from_aff(&t, &pts[i]);
    if (!pts[i].inf && !g2_in_group(&t)) {
      free(pts);
      return NOT_IN_GROUP;
    }
    g2_add(&acc, &acc, &t);
  }
  g2_compress(out96, &acc);
  free(pts);
  return OK;
}

static int sum_pks(g1_jac* acc, const uint8_t* pks, const size_t* pk_lens, size_t n) {
  g1_set_inf(acc);
  size_t po = 0;
  for (size_t i = 0; i < n; ++i) {
    g1_aff p;
    g1_jac t;
    if (g1_decode(&p, pks + po, pk_lens[i]) != OK) return ERR_PUBKEY;
    po += pk_lens[i];
    g1_from_aff(&t, &p);
    g1_add(acc, acc, &t);
  }
  return n ? OK : AGGR_TYPE_MISMATCH;
}

/* BlsPublicKey::aggregate (consensus.rs:371) */
int orc_aggregate_pks(const uint8_t* pks, const size_t* pk_lens, size_t n, uint8_t out48[48]) {
  init();
  g1_jac acc;
  int e = sum_pks(&acc, pks, pk_lens, n);
  if (e) return e;
  g1_compress(out48, &acc);
  return OK;
}

/* verify_aggregated_signature (consensus.rs:446-462) -> inner_verify_aggregated_signature
 * (consensus.rs:365-382): pk parse, aggregate (empty -> 4), sig parse, hash length, verify */
int orc_verify_aggregated(const uint8_t* agg, size_t agg_len, const uint8_t* hash, size_t hash_len,
                          const uint8_t* pks, const size_t* pk_lens, size_t n) {
  init();
  g1_jac acc;
  int e = sum_pks(&acc, pks, pk_lens, n);
  if (e) return e;
  g2_aff s;
  e = agg ? g2_decode(&s, agg, agg_len) : BAD_ENCODING;
  if (e) return e;
  if (!hash || hash_len != 32) return ERR_HASH_LEN;
  g1_aff pa;
  g1_to_aff(&pa, &acc);
  return core_verify(&pa, &s, hash, 32);
}

/* ---- threaded drivers (the CPU baselines) ---- */
typedef struct {
  size_t lo, hi;
  const uint8_t *sigs, *hashes, *pks;
  int32_t* codes;
  uint64_t seed, base; /* vote i's coefficient: SplitMix64(seed, base + i) */
  fp12 f;
  g2_jac S;
} job_t;

static void* verify_many_worker(void* arg) {
  job_t* j = (job_t*)arg;
  for (size_t i = j->lo; i < j->hi; ++i)
    j->codes[i] = orc_verify(j->sigs + 96 * i, 96, j->hashes + 32 * i, 32, j->pks + 48 * i, 48);
  return NULL;
}

static int run_jobs(job_t* jobs, int threads, void* (*fn)(void*)) {
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
  if (!th) return ERR_ARG;
  int started = 0;
  for (int t = 1; t < threads; ++t)
    if (pthread_create(&th[t], NULL, fn, &jobs[t]) == 0) ++started;
    else fn(&jobs[t]);
  fn(&jobs[0]);
  for (int t = 1; t <= started; ++t) pthread_join(th[t], NULL);
  free(th);
  return OK;
}

static job_t* make_jobs(size_t n, int threads, const uint8_t* sigs, const uint8_t* hashes, const uint8_t* pks,
                        int32_t* codes, uint64_t seed) {
  job_t* jobs = (job_t*)calloc((size_t)threads, sizeof(job_t));
  if (!jobs) return NULL;
  for (int t = 0; t < threads; ++t) {
    jobs[t].lo = n * (size_t)t / (size_t)threads;
    jobs[t].hi = n * (size_t)(t + 1) / (size_t)threads;
    jobs[t].sigs = sigs;
    jobs[t].hashes = hashes;
    jobs[t].pks = pks;
    jobs[t].codes = codes;
    jobs[t].seed = seed;
  }
  return jobs;
}

/* n per-vote verifies (96-byte sigs, 32-byte hashes, 48-byte pks) on `threads` threads */
int orc_verify_many(size_t n, const uint8_t* sigs, const uint8_t* hashes, const uint8_t* pks, int32_t* codes,
                    int threads) {
  init();
  if (threads < 1) threads = 1;
  job_t* jobs = make_jobs(n, threads, sigs, hashes, pks, codes, 0);
  if (!jobs) return ERR_ARG;
  run_jobs(jobs, threads, verify_many_worker);
  free(jobs);
  return OK;
}

static uint64_t splitmix(uint64_t seed, uint64_t i) {
  uint64_t z = seed + 0x9e3779b97f4a7c15ull * (i + 1);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  z = z ^ (z >> 31);
  return z ? z : 1;
}

/* RLC batch: per vote parse + checks (codes), H_i, r_i pk_i, r_i sig_i; partial product of
 * Miller(r_i pk_i, H_i) and sum of r_i sig_i over the thread's range */
static void* rlc_worker(void* arg) {
  job_t* j = (job_t*)arg;
  f12_one(&j->f);
  g2_set_inf(&j->S);
  for (size_t i = j->lo; i < j->hi; ++i) {
    g1_aff p;
    g2_aff s;
    int32_t c;
    if (g1_decode(&p, j->pks + 48 * i, 48) != OK) {
      j->codes[i] = ERR_PUBKEY;
      continue;
    }
    c = g2_decode(&s, j->sigs + 96 * i, 96);
    if (c) {
      j->codes[i] = c;
      continue;
    }
    if (!s.inf) {
      g2_jac sj;
      g2_from_aff(&sj, &s);
      if (!g2_in_group(&sj)) {
        j->codes[i] = NOT_IN_GROUP;
        continue;
      }
    }
    if (p.inf) {
      j->codes[i] = PK_IS_INFINITY;
      continue;
    }
    g1_jac pj;
    g1_from_aff(&pj, &p);
    if (!g1_in_group(&pj)) {
      j->codes[i] = NOT_IN_GROUP;
      continue;
    }
    if (s.inf) {
      j->codes[i] = VERIFY_FAIL;
      continue;
    }
    g2_jac hj;
    hash_to_g2(&hj, j->hashes + 32 * i, 32, g_dst, g_dst_len);
    g2_aff h;
    g2_to_aff(&h, &hj);
    if (h.inf) {
      j->codes[i] = VERIFY_FAIL;
      continue;
    }
    j->codes[i] = OK;
    /* r = a + b lambda (mod r), lambda = -x^2, (a, b) = the 32-bit halves of SplitMix64 (the
     * device's tools/fpvm/alg.py LAMBDA): [r] pk = [a] pk + [b] phi(pk), [r] sig = [a] sig +
     * [b] (-psi^2(sig)); pk in G1 and sig in G2 were checked above. */
    const uint64_t r = splitmix(j->seed, j->base + i);
    const uint32_t ra = (uint32_t)r, rb = (uint32_t)(r >> 32);
    g1_jac rp, phi = pj;
    fp_mul(&phi.X, &pj.X, &BETA);
    g1_mul2_32(&rp, &pj, &phi, ra, rb);
    g1_aff rpa;
    g1_to_aff(&rpa, &rp);
    g2_jac sj, rs, ps;
    g2_from_aff(&sj, &s);
    g2_psi(&ps, &sj);
    g2_psi(&ps, &ps);
    g2_neg(&ps, &ps);
    g2_mul2_32(&rs, &sj, &ps, ra, rb);
    g2_add(&j->S, &j->S, &rs);
    fp12 m;
    miller_loop(&m, &rpa, &h);
    f12_mul(&j->f, &j->f, &m);
  }
  return NULL;
}

static void* rlc_fallback_worker(void* arg) {
  job_t* j = (job_t*)arg;
  for (size_t i = j->lo; i < j->hi; ++i)
    if (j->codes[i] == OK)
      j->codes[i] = orc_verify(j->sigs + 96 * i, 96, j->hashes + 32 * i, 32, j->pks + 48 * i, 48);
  return NULL;
}

/* Random-linear-combination batch verify; codes[i] equals orc_verify's code for every vote.
 * Returns OK; *combined_ok (if non-NULL) says whether the combined check passed. */
int orc_verify_batch_rlc(size_t n, const uint8_t* sigs, const uint8_t* hashes, const uint8_t* pks, uint64_t seed,
                         int32_t* codes, int threads, int* combined_ok) {
  init();
  if (threads < 1) threads = 1;
  job_t* jobs = make_jobs(n, threads, sigs, hashes, pks, codes, seed);
  if (!jobs) return ERR_ARG;
  run_jobs(jobs, threads, rlc_worker);
  fp12 f;
  g2_jac S;
  f12_one(&f);
  g2_set_inf(&S);
  for (int t = 0; t < threads; ++t) {
    f12_mul(&f, &f, &jobs[t].f);
    g2_add(&S, &S, &jobs[t].S);
  }
  g2_aff Sa;
  g2_to_aff(&Sa, &S);
  fp12 m;
  miller_loop(&m, &G1_NEG_A, &Sa);
  f12_mul(&f, &f, &m);
  final_exp(&f, &f);
  const int ok = f12_is_one(&f);
  if (!ok) run_jobs(jobs, threads, rlc_fallback_worker);
  if (combined_ok) *combined_ok = ok;
  free(jobs);
  return OK;
}

/* ---- multi-GPU split of orc_verify_batch_rlc in libovhip's partial format ----
 * (include/ovhip.h, OVH_PARTIAL_BYTES = 864): F (576 B) = Fp12 product of the shard's Miller
 * outputs as 12 Fp in Montgomery form (R = 2^384, little-endian limbs), c0.c0.c0 first -- the
 * fp12 struct's own layout; S (288 B) = sum of r_i sig_i in homogeneous projective
 * coordinates (X : Y : Z), O = (0 : 1 : 0). Partials from this oracle and from the GPU combine
 * with each other: they differ only by line scalings the final exponentiation removes. */
static void part_write(uint8_t* out, const fp12* f, const g2_jac* S) {
  fp2 X, Y, Z, z2;
  memcpy(out, f, 576);
  if (f2_is_zero(&S->Z)) {
    memset(&X, 0, sizeof X);
    f2_one(&Y);
    memset(&Z, 0, sizeof Z);
  } else { /* Jacobian (x = X / Z^2, y = Y / Z^3) -> homogeneous (X Z : Y : Z^3) */
    f2_mul(&X, &S->X, &S->Z);
    Y = S->Y;
    f2_sqr(&z2, &S->Z);
    f2_mul(&Z, &z2, &S->Z);
  }
  memcpy(out + 576, &X, 96);
  memcpy(out + 672, &Y, 96);
  memcpy(out + 768, &Z, 96);
}

static void part_read(fp12* f, g2_jac* S, const uint8_t* in) {
  fp2 X, Y, Z, z2;
  memcpy(f, in, 576);
  memcpy(&X, in + 576, 96);
  memcpy(&Y, in + 672, 96);
  memcpy(&Z, in + 768, 96);
  if (f2_is_zero(&Z)) {
    g2_set_inf(S);
    return;
  } /* homogeneous -> Jacobian (X Z : Y Z^2 : Z) */
  f2_mul(&S->X, &X, &Z);
  f2_sqr(&z2, &Z);
  f2_mul(&S->Y, &Y, &z2);
  S->Z = Z;
}

/* Per-shard partial of the RLC batch (codes[i] = parse / subgroup codes, OK for the votes
 * that entered the partial); out864 as above. */
int orc_batch_partial(size_t n, const uint8_t* sigs, const uint8_t* hashes, const uint8_t* pks, uint64_t seed,
                      uint64_t base, int32_t* codes, int threads, uint8_t* out864) {
  init();
  if (threads < 1) threads = 1;
  fp12 f;
  g2_jac S;
  f12_one(&f);
  g2_set_inf(&S);
  if (n) {
    job_t* jobs = make_jobs(n, threads, sigs, hashes, pks, codes, seed);
    if (!jobs) return ERR_ARG;
    for (int t = 0; t < threads; ++t) jobs[t].base = base;
    run_jobs(jobs, threads, rlc_worker);
    for (int t = 0; t < threads; ++t) {
      f12_mul(&f, &f, &jobs[t].f);
      g2_add(&S, &S, &jobs[t].S);
    }
    free(jobs);
  }
  part_write(out864, &f, &S);
  return OK;
}

/* Combined check of k partials: *ok = [prod F * Miller(-G1, sum S)]^FE == 1. */
int orc_combine_partials(size_t k, const uint8_t* parts, int* ok) {
  init();
  if (!parts || !ok || k == 0) return ERR_ARG;
  fp12 f, fi, m;
  g2_jac S, Si;
  f12_one(&f);
  g2_set_inf(&S);
  for (size_t i = 0; i < k; ++i) {
    part_read(&fi, &Si, parts + 864 * i);
    f12_mul(&f, &f, &fi);
    g2_add(&S, &S, &Si);
  }
  g2_aff Sa;
  g2_to_aff(&Sa, &S);
  miller_loop(&m, &G1_NEG_A, &Sa);
  f12_mul(&f, &f, &m);
  final_exp(&f, &f);
  *ok = f12_is_one(&f);
  return OK;
}

/* The per-vote fallback of a shard whose combined check failed: every code still OK becomes
 * orc_verify's code. */
int orc_batch_fallback(size_t n, const uint8_t* sigs, const uint8_t* hashes, const uint8_t* pks, int32_t* codes,
                       int threads) {
  init();
  if (threads < 1) threads = 1;
  if (!n) return OK;
  job_t* jobs = make_jobs(n, threads, sigs, hashes, pks, codes, 0);
  if (!jobs) return ERR_ARG;
  run_jobs(jobs, threads, rlc_fallback_worker);
  free(jobs);
  return OK;
}

/* e(G1, G2)^3 coefficients (c0.c0.c0, c0.c0.c1, c0.c1.c0, ...), 12 x 48 BE bytes */
void orc_gt_g1g2(uint8_t out576[576]) {
  init();
  g1_aff g;
  g1_jac gj = G1_GEN_J;
  g1_to_aff(&g, &gj);
  fp12 f;
  miller_loop(&f, &g, &G2_GEN_A);
  final_exp(&f, &f);
  const fp2* c[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
  for (int k = 0; k < 6; ++k) {
    fp_write(out576 + 96 * k, &c[k]->c0);
    fp_write(out576 + 96 * k + 48, &c[k]->c1);
  }
}
