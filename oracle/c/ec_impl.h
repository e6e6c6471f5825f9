/* CPU ORACLE (test infrastructure only). Short-Weierstrass (a = 0) Jacobian arithmetic,
 * instantiated twice by bls_oracle.c: over Fp for E1 (G1, public keys) and over Fp2 for E2
 * (G2, signatures). Restates oracle/py/bls12_381.py _jac_dbl/_jac_add/pt_mul (the
 * arithmetic blst performs for BlsPublicKey/BlsSignature, reached from
 * src/consensus.rs:371,441 via ophelia-blst).
 *
 * Parameters: FT (field type), F(x) (field op prefix), PT (point prefix). */

typedef struct {
  FT x, y;
  int inf;
} PT_(aff);
typedef struct {
  FT X, Y, Z;
} PT_(jac);

static void PT_(set_inf)(PT_(jac) * r) {
  F(one)(&r->X);
  F(one)(&r->Y);
  F(zero)(&r->Z);
}
static int PT_(is_inf)(const PT_(jac) * a) { return F(is_zero)(&a->Z); }

static void PT_(from_aff)(PT_(jac) * r, const PT_(aff) * a) {
  if (a->inf) {
    PT_(set_inf)(r);
    return;
  }
  r->X = a->x;
  r->Y = a->y;
  F(one)(&r->Z);
}

static void PT_(to_aff)(PT_(aff) * r, const PT_(jac) * p) {
  if (PT_(is_inf)(p)) {
    F(zero)(&r->x);
    F(zero)(&r->y);
    r->inf = 1;
    return;
  }
  FT zi, zi2, zi3;
  F(inv)(&zi, &p->Z);
  F(sqr)(&zi2, &zi);
  F(mul)(&zi3, &zi2, &zi);
  F(mul)(&r->x, &p->X, &zi2);
  F(mul)(&r->y, &p->Y, &zi3);
  r->inf = 0;
}

/* dbl-2009-l */
static void PT_(dbl)(PT_(jac) * r, const PT_(jac) * p) {
  if (PT_(is_inf)(p) || F(is_zero)(&p->Y)) {
    PT_(set_inf)(r);
    return;
  }
  FT A, B, C, D, E, Fv, t, X3, Y3, Z3;
  F(sqr)(&A, &p->X);
  F(sqr)(&B, &p->Y);
  F(sqr)(&C, &B);
  F(add)(&t, &p->X, &B);
  F(sqr)(&t, &t);
  F(sub)(&t, &t, &A);
  F(sub)(&t, &t, &C);
  F(add)(&D, &t, &t);
  F(add)(&E, &A, &A);
  F(add)(&E, &E, &A);
  F(sqr)(&Fv, &E);
  F(add)(&t, &D, &D);
  F(sub)(&X3, &Fv, &t);
  F(sub)(&t, &D, &X3);
  F(mul)(&Y3, &E, &t);
  F(add)(&t, &C, &C);
  F(add)(&t, &t, &t);
  F(add)(&t, &t, &t);
  F(sub)(&Y3, &Y3, &t);
  F(mul)(&Z3, &p->Y, &p->Z);
  F(add)(&Z3, &Z3, &Z3);
  r->X = X3;
  r->Y = Y3;
  r->Z = Z3;
}

/* add-2007-bl style, with the doubling / inverse special cases */
static void PT_(add)(PT_(jac) * r, const PT_(jac) * p, const PT_(jac) * q) {
  if (PT_(is_inf)(p)) {
    *r = *q;
    return;
  }
  if (PT_(is_inf)(q)) {
    *r = *p;
    return;
  }
  FT Z1Z1, Z2Z2, U1, U2, S1, S2, t, H, Rr, H2, H3, U1H2, X3, Y3, Z3;
  F(sqr)(&Z1Z1, &p->Z);
  F(sqr)(&Z2Z2, &q->Z);
  F(mul)(&U1, &p->X, &Z2Z2);
  F(mul)(&U2, &q->X, &Z1Z1);
  F(mul)(&t, &q->Z, &Z2Z2);
  F(mul)(&S1, &p->Y, &t);
  F(mul)(&t, &p->Z, &Z1Z1);
  F(mul)(&S2, &q->Y, &t);
  if (F(eq)(&U1, &U2)) {
    if (F(eq)(&S1, &S2)) {
      PT_(dbl)(r, p);
    } else {
      PT_(set_inf)(r);
    }
    return;
  }
  F(sub)(&H, &U2, &U1);
  F(sub)(&Rr, &S2, &S1);
  F(sqr)(&H2, &H);
  F(mul)(&H3, &H2, &H);
  F(mul)(&U1H2, &U1, &H2);
  F(sqr)(&X3, &Rr);
  F(sub)(&X3, &X3, &H3);
  F(sub)(&X3, &X3, &U1H2);
  F(sub)(&X3, &X3, &U1H2);
  F(sub)(&t, &U1H2, &X3);
  F(mul)(&Y3, &Rr, &t);
  F(mul)(&t, &S1, &H3);
  F(sub)(&Y3, &Y3, &t);
  F(mul)(&t, &p->Z, &q->Z);
  F(mul)(&Z3, &H, &t);
  r->X = X3;
  r->Y = Y3;
  r->Z = Z3;
}

static void PT_(neg)(PT_(jac) * r, const PT_(jac) * p) {
  *r = *p;
  F(neg)(&r->Y, &p->Y);
}

static int PT_(eq)(const PT_(jac) * p, const PT_(jac) * q) {
  int pi = PT_(is_inf)(p), qi = PT_(is_inf)(q);
  if (pi || qi) return pi && qi;
  FT Z1Z1, Z2Z2, a, b, t;
  F(sqr)(&Z1Z1, &p->Z);
  F(sqr)(&Z2Z2, &q->Z);
  F(mul)(&a, &p->X, &Z2Z2);
  F(mul)(&b, &q->X, &Z1Z1);
  if (!F(eq)(&a, &b)) return 0;
  F(mul)(&t, &Z2Z2, &q->Z);
  F(mul)(&a, &p->Y, &t);
  F(mul)(&t, &Z1Z1, &p->Z);
  F(mul)(&b, &q->Y, &t);
  return F(eq)(&a, &b);
}

/* k * p for a little-endian multi-word unsigned scalar (MSB-first double-and-add) */
static void PT_(mul_words)(PT_(jac) * r, const PT_(jac) * p, const uint64_t* k, int nwords) {
  PT_(jac) acc, base = *p;
  PT_(set_inf)(&acc);
  for (int w = nwords - 1; w >= 0; --w)
    for (int b = 63; b >= 0; --b) {
      PT_(dbl)(&acc, &acc);
      if ((k[w] >> b) & 1) PT_(add)(&acc, &acc, &base);
    }
  *r = acc;
}

/* [a] p + [b] q for 32-bit a, b (public): one shared double-and-add chain (Shamir) */
static void PT_(mul2_32)(PT_(jac) * r, const PT_(jac) * p, const PT_(jac) * q, uint32_t a, uint32_t b) {
  PT_(jac) pq, acc;
  PT_(add)(&pq, p, q);
  PT_(set_inf)(&acc);
  for (int k = 31; k >= 0; --k) {
    PT_(dbl)(&acc, &acc);
    const int ba = (a >> k) & 1, bb = (b >> k) & 1;
    if (ba && bb) PT_(add)(&acc, &acc, &pq);
    else if (ba) PT_(add)(&acc, &acc, p);
    else if (bb) PT_(add)(&acc, &acc, q);
  }
  *r = acc;
}

static int PT_(on_curve)(const PT_(aff) * a) {
  if (a->inf) return 1;
  FT l, rr, t;
  F(sqr)(&l, &a->y);
  F(sqr)(&t, &a->x);
  F(mul)(&rr, &t, &a->x);
  F(add_b)(&rr, &rr);
  return F(eq)(&l, &rr);
}
