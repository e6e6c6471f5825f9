"""CPU ORACLE (test infrastructure only) — BLS12-381 min-pk signatures, pure Python.

This module is a from-scratch restatement of the arithmetic that the reference reaches
through ophelia-blst 0.3 -> blst 0.3.x (un-vendored; `/root/reference/Cargo.toml:19-20`).
It is imported ONLY by `tests/`, `tests/golden/make_golden.py` and nothing under
`consensus_overlord_amd/`. It is never the thing measured or shipped.

Call sites in the reference that this file restates:
  * `ConsensusCrypto::verify_signature`        src/consensus.rs:397-416
  * `ConsensusCrypto::aggregate_signatures`    src/consensus.rs:418-444
  * `ConsensusCrypto::verify_aggregated_signature` + `inner_verify_aggregated_signature`
                                               src/consensus.rs:446-462, 365-382
  * `ConsensusCrypto::sign` / `new`            src/consensus.rs:390-395, 347-359

Standards restated (the algorithms blst implements):
  * RFC 9380 hash_to_curve, suite BLS12381G2_XMD:SHA-256_SSWU_RO_ (expand_message_xmd,
    hash_to_field, simplified SWU on the 3-isogenous curve E2', iso_map, clear_cofactor).
  * draft-irtf-cfrg-bls-signature (min-pk: pk in G1, sig in G2), DST
    "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_" (believed ophelia-blst default; parameter).
  * ZCash compressed/uncompressed point serialization (flag bits 0x80/0x40/0x20).
  * Optimal-ate pairing (Miller loop over |x| = 0xd201000000010000) + final exponentiation.

Parity pinning: see tests/test_oracle_kat.py — generators, RFC 9380 expand_message_xmd
vectors, RFC 9380 hash_to_curve G2 vectors, the iso-map/E2 consistency, h_eff vs the
psi-endomorphism formula, and pairing bilinearity.
"""
from __future__ import annotations

import hashlib
import hmac

# ----------------------------------------------------------------------------------------
# Parameters
# ----------------------------------------------------------------------------------------
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
X_ABS = 0xD201000000010000  # BLS parameter x = -X_ABS
X = -X_ABS

DST_NUL = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_"

# ----------------------------------------------------------------------------------------
# Fp
# ----------------------------------------------------------------------------------------


def fp_inv(a: int) -> int:
    if a % P == 0:
        raise ZeroDivisionError("fp_inv(0)")
    return pow(a, P - 2, P)


def fp_sqrt(a: int):
    """Return a square root of a in Fp or None (p = 3 mod 4)."""
    a %= P
    s = pow(a, (P + 1) // 4, P)
    return s if s * s % P == a else None


def fp_is_square(a: int) -> bool:
    a %= P
    return a == 0 or pow(a, (P - 1) // 2, P) == 1


def fp_sgn0(a: int) -> int:
    """RFC 9380 sgn0 for Fp: parity."""
    return (a % P) & 1


def fp_lex_largest(a: int) -> bool:
    """ZCash sort flag for Fp: y > (p-1)/2."""
    return (a % P) > (P - 1) // 2


# ----------------------------------------------------------------------------------------
# Fp2 = Fp[u]/(u^2 + 1); elements are tuples (c0, c1)
# ----------------------------------------------------------------------------------------
F2_ZERO = (0, 0)
F2_ONE = (1, 0)


def f2(a, b=0):
    return (a % P, b % P)


def f2_add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2_sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def f2_neg(a):
    return ((-a[0]) % P, (-a[1]) % P)


def f2_mul(a, b):
    a0, a1 = a
    b0, b1 = b
    return ((a0 * b0 - a1 * b1) % P, (a0 * b1 + a1 * b0) % P)


def f2_sqr(a):
    a0, a1 = a
    return ((a0 + a1) * (a0 - a1) % P, 2 * a0 * a1 % P)


def f2_muls(a, s: int):
    return (a[0] * s % P, a[1] * s % P)


def f2_conj(a):
    return (a[0], (-a[1]) % P)


def f2_inv(a):
    a0, a1 = a
    t = fp_inv(a0 * a0 + a1 * a1)
    return (a0 * t % P, (-a1) * t % P)


def f2_is_zero(a) -> bool:
    return a[0] % P == 0 and a[1] % P == 0


def f2_eq(a, b) -> bool:
    return (a[0] - b[0]) % P == 0 and (a[1] - b[1]) % P == 0


def f2_pow(a, e: int):
    r = F2_ONE
    base = a
    while e > 0:
        if e & 1:
            r = f2_mul(r, base)
        base = f2_sqr(base)
        e >>= 1
    return r


def f2_mul_xi(a):
    """Multiply by xi = 1 + u."""
    a0, a1 = a
    return ((a0 - a1) % P, (a0 + a1) % P)


def f2_is_square(a) -> bool:
    # norm map: a is a square in Fp2 iff N(a) = a0^2 + a1^2 is a square in Fp
    return fp_is_square(a[0] * a[0] + a[1] * a[1])


def f2_sqrt(a):
    """Return some square root of a in Fp2, or None. (Any root: callers fix the sign.)"""
    if f2_is_zero(a):
        return F2_ZERO
    a0, a1 = a
    if a1 % P == 0:
        s = fp_sqrt(a0)
        if s is not None:
            return (s, 0)
        s = fp_sqrt(-a0)
        return (0, s) if s is not None else None
    n = fp_sqrt(a0 * a0 + a1 * a1)
    if n is None:
        return None
    inv2 = fp_inv(2)
    for cand in ((a0 + n) * inv2, (a0 - n) * inv2):
        x0 = fp_sqrt(cand)
        if x0 is not None and x0 % P != 0:
            x1 = a1 * fp_inv(2 * x0) % P
            r = (x0, x1)
            if f2_eq(f2_sqr(r), a):
                return r
    return None


def f2_sgn0(a) -> int:
    """RFC 9380 sgn0 for Fp2 (m = 2)."""
    s0 = a[0] & 1
    z0 = a[0] == 0
    s1 = a[1] & 1
    return s0 | (z0 and s1)


def f2_lex_largest(a) -> bool:
    """ZCash sort flag for Fp2: compare c1 first, c0 only when c1 == 0."""
    if a[1] % P != 0:
        return fp_lex_largest(a[1])
    return fp_lex_largest(a[0])


XI = (1, 1)

# ----------------------------------------------------------------------------------------
# Fp6 = Fp2[v]/(v^3 - xi); Fp12 = Fp6[w]/(w^2 - v)
# ----------------------------------------------------------------------------------------
F6_ZERO = (F2_ZERO, F2_ZERO, F2_ZERO)
F6_ONE = (F2_ONE, F2_ZERO, F2_ZERO)


def f6_add(a, b):
    return (f2_add(a[0], b[0]), f2_add(a[1], b[1]), f2_add(a[2], b[2]))


def f6_sub(a, b):
    return (f2_sub(a[0], b[0]), f2_sub(a[1], b[1]), f2_sub(a[2], b[2]))


def f6_neg(a):
    return (f2_neg(a[0]), f2_neg(a[1]), f2_neg(a[2]))


def f6_mul(a, b):
    a0, a1, a2 = a
    b0, b1, b2 = b
    t0 = f2_mul(a0, b0)
    t1 = f2_mul(a1, b1)
    t2 = f2_mul(a2, b2)
    c0 = f2_add(t0, f2_mul_xi(f2_sub(f2_mul(f2_add(a1, a2), f2_add(b1, b2)), f2_add(t1, t2))))
    c1 = f2_add(f2_sub(f2_mul(f2_add(a0, a1), f2_add(b0, b1)), f2_add(t0, t1)), f2_mul_xi(t2))
    c2 = f2_add(f2_sub(f2_mul(f2_add(a0, a2), f2_add(b0, b2)), f2_add(t0, t2)), t1)
    return (c0, c1, c2)


def f6_mul_v(a):
    """Multiply by v: (a0 + a1 v + a2 v^2) v = xi a2 + a0 v + a1 v^2."""
    return (f2_mul_xi(a[2]), a[0], a[1])


def f6_inv(a):
    a0, a1, a2 = a
    c0 = f2_sub(f2_sqr(a0), f2_mul_xi(f2_mul(a1, a2)))
    c1 = f2_sub(f2_mul_xi(f2_sqr(a2)), f2_mul(a0, a1))
    c2 = f2_sub(f2_sqr(a1), f2_mul(a0, a2))
    t = f2_add(f2_mul(a0, c0), f2_mul_xi(f2_add(f2_mul(a2, c1), f2_mul(a1, c2))))
    ti = f2_inv(t)
    return (f2_mul(c0, ti), f2_mul(c1, ti), f2_mul(c2, ti))


F12_ONE = (F6_ONE, F6_ZERO)


def f12_mul(a, b):
    a0, a1 = a
    b0, b1 = b
    t0 = f6_mul(a0, b0)
    t1 = f6_mul(a1, b1)
    c0 = f6_add(t0, f6_mul_v(t1))
    c1 = f6_sub(f6_mul(f6_add(a0, a1), f6_add(b0, b1)), f6_add(t0, t1))
    return (c0, c1)


def f12_sqr(a):
    return f12_mul(a, a)


def f12_conj(a):
    return (a[0], f6_neg(a[1]))


def f12_inv(a):
    a0, a1 = a
    t = f6_sub(f6_mul(a0, a0), f6_mul_v(f6_mul(a1, a1)))
    ti = f6_inv(t)
    return (f6_mul(a0, ti), f6_neg(f6_mul(a1, ti)))


def f12_eq(a, b) -> bool:
    return all(f2_eq(x, y) for x, y in zip(a[0] + a[1], b[0] + b[1]))


def f12_is_one(a) -> bool:
    return f12_eq(a, F12_ONE)


# Frobenius: element of Fp12 has coefficient of v^i w^j = w^(2i+j). (w^k)^p = gamma_k w^k with
# gamma_k = xi^(k(p-1)/6).
_GAMMA = [f2_pow(XI, k * (P - 1) // 6) for k in range(6)]


def f12_frob(a):
    (a0, a1, a2), (b0, b1, b2) = a
    coeffs = [a0, b0, a1, b1, a2, b2]  # index = power of w: 0,1,2,3,4,5
    out = [f2_mul(f2_conj(c), _GAMMA[k]) for k, c in enumerate(coeffs)]
    return ((out[0], out[2], out[4]), (out[1], out[3], out[5]))


def f12_pow(a, e: int):
    r = F12_ONE
    base = a
    while e > 0:
        if e & 1:
            r = f12_mul(r, base)
        base = f12_sqr(base)
        e >>= 1
    return r


# ----------------------------------------------------------------------------------------
# Curves. Points are affine tuples (x, y) or None for the point at infinity.
#   E1 : y^2 = x^3 + 4 over Fp          (G1, public keys)
#   E2 : y^2 = x^3 + 4(1+u) over Fp2    (G2, signatures; M-type sextic twist)
# ----------------------------------------------------------------------------------------
B1 = 4
B2 = (4, 4)

G1_GEN = (
    0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB,
    0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1,
)
G2_GEN = (
    (
        0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
        0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E,
    ),
    (
        0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
        0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE,
    ),
)


class FpOps:
    zero = 0
    one = 1
    b = B1

    @staticmethod
    def add(a, b):
        return (a + b) % P

    @staticmethod
    def sub(a, b):
        return (a - b) % P

    @staticmethod
    def mul(a, b):
        return a * b % P

    @staticmethod
    def sqr(a):
        return a * a % P

    @staticmethod
    def inv(a):
        return fp_inv(a)

    @staticmethod
    def neg(a):
        return (-a) % P

    @staticmethod
    def eq(a, b):
        return (a - b) % P == 0

    @staticmethod
    def is_zero(a):
        return a % P == 0

    @staticmethod
    def muls(a, s):
        return a * s % P


class Fp2Ops:
    zero = F2_ZERO
    one = F2_ONE
    b = B2
    add = staticmethod(f2_add)
    sub = staticmethod(f2_sub)
    mul = staticmethod(f2_mul)
    sqr = staticmethod(f2_sqr)
    inv = staticmethod(f2_inv)
    neg = staticmethod(f2_neg)
    eq = staticmethod(f2_eq)
    is_zero = staticmethod(f2_is_zero)
    muls = staticmethod(f2_muls)


def on_curve(F, pt) -> bool:
    if pt is None:
        return True
    x, y = pt
    return F.eq(F.sqr(y), F.add(F.mul(F.sqr(x), x), F.b))


def pt_neg(F, pt):
    if pt is None:
        return None
    return (pt[0], F.neg(pt[1]))


def pt_eq(F, p1, p2) -> bool:
    if p1 is None or p2 is None:
        return p1 is None and p2 is None
    return F.eq(p1[0], p2[0]) and F.eq(p1[1], p2[1])


# Jacobian (X, Y, Z): x = X/Z^2, y = Y/Z^3 (a = 0 curves). Used for scalar multiplication.
def _jac_from_aff(F, pt):
    if pt is None:
        return (F.one, F.one, F.zero)
    return (pt[0], pt[1], F.one)


def _jac_to_aff(F, J):
    X, Y, Z = J
    if F.is_zero(Z):
        return None
    zi = F.inv(Z)
    zi2 = F.sqr(zi)
    return (F.mul(X, zi2), F.mul(Y, F.mul(zi2, zi)))


def _jac_dbl(F, J):
    X, Y, Z = J
    if F.is_zero(Z) or F.is_zero(Y):
        return (F.one, F.one, F.zero)
    A = F.sqr(X)
    B = F.sqr(Y)
    C = F.sqr(B)
    D = F.muls(F.sub(F.sub(F.sqr(F.add(X, B)), A), C), 2)
    E = F.muls(A, 3)
    Fv = F.sqr(E)
    X3 = F.sub(Fv, F.muls(D, 2))
    Y3 = F.sub(F.mul(E, F.sub(D, X3)), F.muls(C, 8))
    Z3 = F.muls(F.mul(Y, Z), 2)
    return (X3, Y3, Z3)


def _jac_add(F, J1, J2):
    X1, Y1, Z1 = J1
    X2, Y2, Z2 = J2
    if F.is_zero(Z1):
        return J2
    if F.is_zero(Z2):
        return J1
    Z1Z1 = F.sqr(Z1)
    Z2Z2 = F.sqr(Z2)
    U1 = F.mul(X1, Z2Z2)
    U2 = F.mul(X2, Z1Z1)
    S1 = F.mul(Y1, F.mul(Z2, Z2Z2))
    S2 = F.mul(Y2, F.mul(Z1, Z1Z1))
    if F.eq(U1, U2):
        if F.eq(S1, S2):
            return _jac_dbl(F, J1)
        return (F.one, F.one, F.zero)
    H = F.sub(U2, U1)
    Rr = F.sub(S2, S1)
    H2 = F.sqr(H)
    H3 = F.mul(H2, H)
    U1H2 = F.mul(U1, H2)
    X3 = F.sub(F.sub(F.sqr(Rr), H3), F.muls(U1H2, 2))
    Y3 = F.sub(F.mul(Rr, F.sub(U1H2, X3)), F.mul(S1, H3))
    Z3 = F.mul(H, F.mul(Z1, Z2))
    return (X3, Y3, Z3)


def pt_add(F, p1, p2):
    return _jac_to_aff(F, _jac_add(F, _jac_from_aff(F, p1), _jac_from_aff(F, p2)))


def pt_mul(F, pt, k: int):
    """Scalar multiplication k*pt (k may be negative or exceed the group order)."""
    if pt is None or k == 0:
        return None
    if k < 0:
        pt = pt_neg(F, pt)
        k = -k
    acc = (F.one, F.one, F.zero)
    base = _jac_from_aff(F, pt)
    for bit in bin(k)[2:]:
        acc = _jac_dbl(F, acc)
        if bit == "1":
            acc = _jac_add(F, acc, base)
    return _jac_to_aff(F, acc)


def g1_in_subgroup(pt) -> bool:
    return pt_mul(FpOps, pt, R) is None


def g2_in_subgroup(pt) -> bool:
    return pt_mul(Fp2Ops, pt, R) is None


# psi endomorphism on E2: psi(x, y) = (conj(x) * PSI_CX, conj(y) * PSI_CY)
PSI_CX = f2_inv(f2_pow(XI, (P - 1) // 3))
PSI_CY = f2_inv(f2_pow(XI, (P - 1) // 2))


def g2_psi(pt):
    if pt is None:
        return None
    return (f2_mul(f2_conj(pt[0]), PSI_CX), f2_mul(f2_conj(pt[1]), PSI_CY))


# ----------------------------------------------------------------------------------------
# Serialization (ZCash format, as in blst POINTonE{1,2}_{Compress,Uncompress,Serialize,
# Deserialize}_BE). Errors mirror blst's BLST_ERROR numbering.
# ----------------------------------------------------------------------------------------
BLST_SUCCESS = 0
BLST_BAD_ENCODING = 1
BLST_POINT_NOT_ON_CURVE = 2
BLST_POINT_NOT_IN_GROUP = 3
BLST_AGGR_TYPE_MISMATCH = 4
BLST_VERIFY_FAIL = 5
BLST_PK_IS_INFINITY = 6
BLST_BAD_SCALAR = 7


class BlstError(Exception):
    def __init__(self, code: int):
        super().__init__(code)
        self.code = code


def _i2b(v: int, n: int) -> bytes:
    return int(v).to_bytes(n, "big")


def g1_compress(pt) -> bytes:
    if pt is None:
        return bytes([0xC0]) + bytes(47)
    out = bytearray(_i2b(pt[0], 48))
    out[0] |= 0x80 | (0x20 if fp_lex_largest(pt[1]) else 0)
    return bytes(out)


def g1_serialize(pt) -> bytes:
    if pt is None:
        return bytes([0x40]) + bytes(95)
    return _i2b(pt[0], 48) + _i2b(pt[1], 48)


def g2_compress(pt) -> bytes:
    if pt is None:
        return bytes([0xC0]) + bytes(95)
    (x0, x1), y = pt
    out = bytearray(_i2b(x1, 48) + _i2b(x0, 48))
    out[0] |= 0x80 | (0x20 if f2_lex_largest(y) else 0)
    return bytes(out)


def g2_serialize(pt) -> bytes:
    if pt is None:
        return bytes([0x40]) + bytes(191)
    (x0, x1), (y0, y1) = pt
    return _i2b(x1, 48) + _i2b(x0, 48) + _i2b(y1, 48) + _i2b(y0, 48)


def _g1_uncompress(b: bytes):
    b0 = b[0]
    if b0 & 0x40:
        if (b0 & 0x3F) == 0 and not any(b[1:]):
            return None
        raise BlstError(BLST_BAD_ENCODING)
    x = int.from_bytes(bytes([b0 & 0x1F]) + b[1:48], "big")
    if x >= P:
        raise BlstError(BLST_BAD_ENCODING)
    y = fp_sqrt(x * x * x + B1)
    if y is None:
        raise BlstError(BLST_POINT_NOT_ON_CURVE)
    if fp_lex_largest(y) != bool(b0 & 0x20):
        y = (-y) % P
    if x == 0:
        raise BlstError(BLST_POINT_NOT_IN_GROUP)
    return (x, y)


def _g1_deserialize(b: bytes):
    b0 = b[0]
    if b0 & 0x40:
        if (b0 & 0x3F) == 0 and not any(b[1:]):
            return None
        raise BlstError(BLST_BAD_ENCODING)
    if b0 & 0x20:
        raise BlstError(BLST_BAD_ENCODING)
    x = int.from_bytes(bytes([b0 & 0x1F]) + b[1:48], "big")
    y = int.from_bytes(b[48:96], "big")
    if x >= P or y >= P:
        raise BlstError(BLST_BAD_ENCODING)
    if not on_curve(FpOps, (x, y)):
        raise BlstError(BLST_POINT_NOT_ON_CURVE)
    if x == 0:
        raise BlstError(BLST_POINT_NOT_IN_GROUP)
    return (x, y)


def g1_from_bytes(b: bytes):
    """blst `PublicKey::from_bytes`: 48-byte compressed (0x80 set) or 96-byte uncompressed."""
    b = bytes(b)
    if len(b) == 48 and (b[0] & 0x80):
        return _g1_uncompress(b)
    if len(b) == 96 and not (b[0] & 0x80):
        return _g1_deserialize(b)
    raise BlstError(BLST_BAD_ENCODING)


def _g2_uncompress(b: bytes):
    b0 = b[0]
    if b0 & 0x40:
        if (b0 & 0x3F) == 0 and not any(b[1:]):
            return None
        raise BlstError(BLST_BAD_ENCODING)
    x1 = int.from_bytes(bytes([b0 & 0x1F]) + b[1:48], "big")
    x0 = int.from_bytes(b[48:96], "big")
    if x1 >= P or x0 >= P:
        raise BlstError(BLST_BAD_ENCODING)
    xx = (x0, x1)
    y = f2_sqrt(f2_add(f2_mul(f2_sqr(xx), xx), B2))
    if y is None:
        raise BlstError(BLST_POINT_NOT_ON_CURVE)
    if f2_lex_largest(y) != bool(b0 & 0x20):
        y = f2_neg(y)
    if f2_is_zero(xx):
        raise BlstError(BLST_POINT_NOT_IN_GROUP)
    return (xx, y)


def _g2_deserialize(b: bytes):
    b0 = b[0]
    if b0 & 0x40:
        if (b0 & 0x3F) == 0 and not any(b[1:]):
            return None
        raise BlstError(BLST_BAD_ENCODING)
    if b0 & 0x20:
        raise BlstError(BLST_BAD_ENCODING)
    x1 = int.from_bytes(bytes([b0 & 0x1F]) + b[1:48], "big")
    x0 = int.from_bytes(b[48:96], "big")
    y1 = int.from_bytes(b[96:144], "big")
    y0 = int.from_bytes(b[144:192], "big")
    if max(x0, x1, y0, y1) >= P:
        raise BlstError(BLST_BAD_ENCODING)
    pt = ((x0, x1), (y0, y1))
    if not on_curve(Fp2Ops, pt):
        raise BlstError(BLST_POINT_NOT_ON_CURVE)
    if f2_is_zero(pt[0]):
        raise BlstError(BLST_POINT_NOT_IN_GROUP)
    return pt


def g2_from_bytes(b: bytes):
    """blst `Signature::from_bytes`: 96-byte compressed or 192-byte uncompressed."""
    b = bytes(b)
    if len(b) == 96 and (b[0] & 0x80):
        return _g2_uncompress(b)
    if len(b) == 192 and not (b[0] & 0x80):
        return _g2_deserialize(b)
    raise BlstError(BLST_BAD_ENCODING)


# ----------------------------------------------------------------------------------------
# Hash to G2: RFC 9380 BLS12381G2_XMD:SHA-256_SSWU_RO_
# ----------------------------------------------------------------------------------------


def expand_message_xmd(msg: bytes, dst: bytes, len_in_bytes: int) -> bytes:
    b_in_bytes, s_in_bytes = 32, 64
    ell = (len_in_bytes + b_in_bytes - 1) // b_in_bytes
    if ell > 255 or len(dst) > 255 or len_in_bytes > 65535:
        raise ValueError("expand_message_xmd: bad lengths")
    dst_prime = dst + bytes([len(dst)])
    z_pad = bytes(s_in_bytes)
    l_i_b = len_in_bytes.to_bytes(2, "big")
    b0 = hashlib.sha256(z_pad + msg + l_i_b + b"\x00" + dst_prime).digest()
    b1 = hashlib.sha256(b0 + b"\x01" + dst_prime).digest()
    out = [b1]
    for i in range(2, ell + 1):
        prev = out[-1]
        out.append(hashlib.sha256(bytes(x ^ y for x, y in zip(b0, prev)) + bytes([i]) + dst_prime).digest())
    return b"".join(out)[:len_in_bytes]


def hash_to_field_fp2(msg: bytes, dst: bytes, count: int = 2):
    L = 64
    ub = expand_message_xmd(msg, dst, count * 2 * L)
    res = []
    for i in range(count):
        e = [int.from_bytes(ub[L * (j + i * 2): L * (j + i * 2 + 1)], "big") % P for j in range(2)]
        res.append((e[0], e[1]))
    return res


# E2' : y^2 = x^3 + A' x + B', A' = 240 u, B' = 1012 (1 + u); Z = -(2 + u)
SSWU_A = (0, 240)
SSWU_B = (1012, 1012)
SSWU_Z = f2(-2, -1)


def map_to_curve_sswu(u):
    """Simplified SWU for E2' (RFC 9380 section 6.6.2, non-constant-time form)."""
    A, B, Z = SSWU_A, SSWU_B, SSWU_Z
    u2 = f2_sqr(u)
    zu2 = f2_mul(Z, u2)
    tv1 = f2_add(f2_sqr(zu2), zu2)  # Z^2 u^4 + Z u^2
    if f2_is_zero(tv1):
        x1 = f2_mul(B, f2_inv(f2_mul(Z, A)))
    else:
        x1 = f2_mul(f2_mul(f2_neg(B), f2_inv(A)), f2_add(F2_ONE, f2_inv(tv1)))
    gx1 = f2_add(f2_add(f2_mul(f2_sqr(x1), x1), f2_mul(A, x1)), B)
    if f2_is_square(gx1):
        x, y = x1, f2_sqrt(gx1)
    else:
        x = f2_mul(zu2, x1)
        gx2 = f2_add(f2_add(f2_mul(f2_sqr(x), x), f2_mul(A, x)), B)
        y = f2_sqrt(gx2)
    if f2_sgn0(u) != f2_sgn0(y):
        y = f2_neg(y)
    return (x, y)


def _h(s: str) -> int:
    return int(s, 16)


# 3-isogeny E2' -> E2 constants (RFC 9380 appendix E.3). Pinned by tests: the map must
# carry E2' points onto E2, and hash_to_curve must reproduce the RFC's G2 test vectors.
ISO_XNUM = [
    (_h("5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6"),
     _h("5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6")),
    (0, _h("11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71a")),
    (_h("11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71e"),
     _h("8ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38d")),
    (_h("171d6541fa38ccfaed6dea691f5fb614cb14b4e7f4e810aa22d6108f142b85757098e38d0f671c7188e2aaaaaaaa5ed1"), 0),
]
ISO_XDEN = [
    (0, _h("1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaa63")),
    (0xC, _h("1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaa9f")),
    (1, 0),
]
ISO_YNUM = [
    (_h("1530477c7ab4113b59a4c18b076d11930f7da5d4a07f649bf54439d87d27e500fc8c25ebf8c92f6812cfc71c71c6d706"),
     _h("1530477c7ab4113b59a4c18b076d11930f7da5d4a07f649bf54439d87d27e500fc8c25ebf8c92f6812cfc71c71c6d706")),
    (0, _h("5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97be")),
    (_h("11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71c"),
     _h("8ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38f")),
    (_h("124c9ad43b6cf79bfbf7043de3811ad0761b0f37a1e26286b0e977c69aa274524e79097a56dc4bd9e1b371c71c718b10"), 0),
]
ISO_YDEN = [
    (_h("1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffa8fb"),
     _h("1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffa8fb")),
    (0, _h("1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffa9d3")),
    (0x12, _h("1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaa99")),
    (1, 0),
]


def _poly(coeffs, x):
    acc = F2_ZERO
    for c in reversed(coeffs):
        acc = f2_add(f2_mul(acc, x), c)
    return acc


def iso_map_g2(pt):
    if pt is None:
        return None
    x, y = pt
    xd = _poly(ISO_XDEN, x)
    yd = _poly(ISO_YDEN, x)
    if f2_is_zero(xd) or f2_is_zero(yd):
        return None
    xn = _poly(ISO_XNUM, x)
    yn = _poly(ISO_YNUM, x)
    return (f2_mul(xn, f2_inv(xd)), f2_mul(y, f2_mul(yn, f2_inv(yd))))


H_EFF_G2 = _h(
    "bc69f08f2ee75b3584c6a0ea91b352888e2a8e9145ad7689986ff031508ffe1329c2f178731db956d82bf015d1212b02"
    "ec0ec69d7477c1ae954cbc06689f6a359894c0adebbf6b4e8020005aaa95551"
)


def clear_cofactor_g2(pt):
    """h_eff * P (RFC 9380 section 8.8.2)."""
    return pt_mul(Fp2Ops, pt, H_EFF_G2)


def clear_cofactor_g2_psi(pt):
    """Equivalent endomorphism form (Budroni-Pintore):
    h_eff P = [x^2 - x - 1] P + [x - 1] psi(P) + psi^2(2P)."""
    F = Fp2Ops
    t1 = pt_mul(F, pt, X * X - X - 1)
    t2 = pt_mul(F, g2_psi(pt), X - 1)
    t3 = g2_psi(g2_psi(pt_mul(F, pt, 2)))
    return pt_add(F, pt_add(F, t1, t2), t3)


def hash_to_g2(msg: bytes, dst: bytes = DST_NUL):
    u0, u1 = hash_to_field_fp2(msg, dst, 2)
    q0 = iso_map_g2(map_to_curve_sswu(u0))
    q1 = iso_map_g2(map_to_curve_sswu(u1))
    return clear_cofactor_g2(pt_add(Fp2Ops, q0, q1))


# ----------------------------------------------------------------------------------------
# Pairing: optimal ate, Miller loop over |x| with affine line functions on the twist.
# Line through T (on E2) evaluated at P (on E1), scaled by w^3 (killed by the final exp):
#   l = (lambda*xT - yT) + (-lambda*xP) v + yP v w
# ----------------------------------------------------------------------------------------


def _line(lam, xT, yT, P1):
    xP, yP = P1
    c0 = (f2_sub(f2_mul(lam, xT), yT), f2_muls(lam, (-xP) % P), F2_ZERO)
    c1 = (F2_ZERO, (yP % P, 0), F2_ZERO)
    return (c0, c1)


def miller_loop(P1, Q2):
    """f_{|x|,Q}(P), conjugated because x < 0. P1 in E1 affine, Q2 in E2 affine (non-infinity)."""
    if P1 is None or Q2 is None:
        return F12_ONE
    f = F12_ONE
    T = Q2
    bits = bin(X_ABS)[3:]
    for bit in bits:
        xT, yT = T
        lam = f2_mul(f2_muls(f2_sqr(xT), 3), f2_inv(f2_muls(yT, 2)))
        f = f12_mul(f12_sqr(f), _line(lam, xT, yT, P1))
        x3 = f2_sub(f2_sqr(lam), f2_muls(xT, 2))
        T = (x3, f2_sub(f2_mul(lam, f2_sub(xT, x3)), yT))
        if bit == "1":
            xT, yT = T
            xQ, yQ = Q2
            lam = f2_mul(f2_sub(yQ, yT), f2_inv(f2_sub(xQ, xT)))
            f = f12_mul(f, _line(lam, xT, yT, P1))
            x3 = f2_sub(f2_sub(f2_sqr(lam), xT), xQ)
            T = (x3, f2_sub(f2_mul(lam, f2_sub(xT, x3)), yT))
    return f12_conj(f)


_FE_HARD = (P**4 - P**2 + 1) // R


def final_exponentiation(f):
    """f^((p^12 - 1)/r)."""
    # easy part: (p^6 - 1)(p^2 + 1)
    f = f12_mul(f12_conj(f), f12_inv(f))
    f = f12_mul(f12_frob(f12_frob(f)), f)
    return f12_pow(f, _FE_HARD)


def pairing(P1, Q2):
    return final_exponentiation(miller_loop(P1, Q2))


def multi_pairing_is_one(pairs) -> bool:
    f = F12_ONE
    for P1, Q2 in pairs:
        f = f12_mul(f, miller_loop(P1, Q2))
    return f12_is_one(final_exponentiation(f))


# ----------------------------------------------------------------------------------------
# BLS min-pk (what ophelia-blst exposes as BlsPrivateKey / BlsPublicKey / BlsSignature)
# ----------------------------------------------------------------------------------------


def hkdf_extract(salt: bytes, ikm: bytes) -> bytes:
    """RFC 5869 HKDF-Extract with SHA-256."""
    return hmac.new(salt, ikm, hashlib.sha256).digest()


def hkdf_expand(prk: bytes, info: bytes, length: int) -> bytes:
    """RFC 5869 HKDF-Expand with SHA-256."""
    t, okm, i = b"", b"", 1
    while len(okm) < length:
        t = hmac.new(prk, t + info + bytes([i]), hashlib.sha256).digest()
        okm += t
        i += 1
    return okm[:length]


def sk_keygen(ikm: bytes, key_info: bytes = b"") -> int:
    """blst `SecretKey::key_gen(ikm, key_info)` = IETF KeyGen (draft-irtf-cfrg-bls-signature-04
    section 2.3, identical to EIP-2333 HKDF_mod_r): what ophelia-blst's
    `BlsPrivateKey::try_from` [dep] must be, since the reference parses its own
    example/private_key (>= r) without error (src/consensus.rs:349-350)."""
    ikm = bytes(ikm)
    if len(ikm) < 32:
        raise BlstError(BLST_BAD_ENCODING)
    salt = b"BLS-SIG-KEYGEN-SALT-"
    sk = 0
    while sk == 0:
        salt = hashlib.sha256(salt).digest()
        okm = hkdf_expand(hkdf_extract(salt, ikm + b"\x00"), key_info + (48).to_bytes(2, "big"), 48)
        sk = int.from_bytes(okm, "big") % R
    return sk


def sk_from_bytes(b: bytes) -> int:
    """blst `SecretKey::from_bytes` (the OVH_FLAG_SK_RAW alternative): 32-byte big-endian
    scalar, 0 < sk < r."""
    b = bytes(b)
    if len(b) != 32:
        raise BlstError(BLST_BAD_ENCODING)
    v = int.from_bytes(b, "big")
    if v == 0 or v >= R:
        raise BlstError(BLST_BAD_ENCODING)
    return v


def sk_to_pk(sk: int):
    return pt_mul(FpOps, G1_GEN, sk)


def sign(sk: int, msg: bytes, dst: bytes = DST_NUL):
    """ConsensusCrypto::sign (src/consensus.rs:390-395): sigma = sk * H(msg)."""
    return pt_mul(Fp2Ops, hash_to_g2(msg, dst), sk)


def core_verify(pk, sig, msg: bytes, dst: bytes = DST_NUL) -> int:
    """blst core_verify (min-pk) with sig_groupcheck = true and pk_validate = true.
    Returns a BLST_ERROR code (0 on success)."""
    if sig is not None and not g2_in_subgroup(sig):
        return BLST_POINT_NOT_IN_GROUP
    if pk is None:
        return BLST_PK_IS_INFINITY
    if not g1_in_subgroup(pk):
        return BLST_POINT_NOT_IN_GROUP
    H = hash_to_g2(msg, dst)
    ok = multi_pairing_is_one([(pk, H), (pt_neg(FpOps, G1_GEN), sig)])
    return BLST_SUCCESS if ok else BLST_VERIFY_FAIL


def aggregate_g2(sigs, groupcheck: bool = True):
    """blst AggregateSignature::aggregate: empty -> AGGR_TYPE_MISMATCH; optional group check."""
    if len(sigs) == 0:
        raise BlstError(BLST_AGGR_TYPE_MISMATCH)
    acc = None
    for s in sigs:
        if groupcheck and s is not None and not g2_in_subgroup(s):
            raise BlstError(BLST_POINT_NOT_IN_GROUP)
        acc = pt_add(Fp2Ops, acc, s)
    return acc


def aggregate_g1(pks, validate: bool = False):
    """blst AggregatePublicKey::aggregate: empty -> AGGR_TYPE_MISMATCH."""
    if len(pks) == 0:
        raise BlstError(BLST_AGGR_TYPE_MISMATCH)
    acc = None
    for k in pks:
        if validate:
            if k is None:
                raise BlstError(BLST_PK_IS_INFINITY)
            if not g1_in_subgroup(k):
                raise BlstError(BLST_POINT_NOT_IN_GROUP)
        acc = pt_add(FpOps, acc, k)
    return acc


# ----------------------------------------------------------------------------------------
# "Fast-path" formulas, restated here so the C oracle and the HIP kernels can be checked
# against them. Each is validated in tests against the simple definitions above.
# ----------------------------------------------------------------------------------------
B2_PRIME = B2  # b' = 4 xi (M-type twist)
B2_3 = f2_muls(B2, 3)


def f12_mul_by_014(f, l0, l1, l4):
    """f * (l0 + l1 v + l4 v w) -- the sparse line shape produced by the M-type twist."""
    line = ((l0, l1, F2_ZERO), (F2_ZERO, l4, F2_ZERO))
    return f12_mul(f, line)


def miller_loop_proj(P1, Q2):
    """Same pairing as `miller_loop`, with T in homogeneous projective coordinates and
    lines scaled by Fp2 factors (removed by the final exponentiation).
    Doubling line:  (Y^2 - 3b'Z^2) + (-3X^2 xP) v + (2YZ yP) vw
    Addition line:  (theta xQ - lam yQ) + (-theta xP) v + (lam yP) vw,
                    theta = Y - yQ Z, lam = X - xQ Z."""
    if P1 is None or Q2 is None:
        return F12_ONE
    xP, yP = P1
    xQ, yQ = Q2
    X, Y, Z = xQ, yQ, F2_ONE
    f = F12_ONE
    first = True
    for bit in bin(X_ABS)[3:]:
        # doubling step
        XX = f2_sqr(X)
        YY = f2_sqr(Y)
        ZZ = f2_sqr(Z)
        E = f2_mul(B2_3, ZZ)                # 3 b' Z^2
        l0 = f2_sub(YY, E)
        l1 = f2_muls(XX, (-3 * xP) % P)
        l4 = f2_muls(f2_mul(Y, Z), (2 * yP) % P)
        # T = 2T  (x = X/Z, y = Y/Z)
        A = f2_mul(X, Y)                    # XY
        Fv = f2_muls(E, 3)                  # 9 b' Z^2
        X3 = f2_muls(f2_mul(A, f2_sub(YY, Fv)), 2)          # 2XY(Y^2 - 9b'Z^2)
        G = f2_add(YY, Fv)
        Y3 = f2_sub(f2_sqr(G), f2_muls(f2_sqr(E), 12))      # (Y^2+9b'Z^2)^2 - 108 b'^2 Z^4
        Z3 = f2_muls(f2_mul(YY, f2_mul(Y, Z)), 8)          # 8 Y^3 Z
        X, Y, Z = X3, Y3, Z3
        f = f12_mul_by_014(F12_ONE if first else f12_sqr(f), l0, l1, l4)
        first = False
        if bit == "1":
            theta = f2_sub(Y, f2_mul(yQ, Z))
            lam = f2_sub(X, f2_mul(xQ, Z))
            l0 = f2_sub(f2_mul(theta, xQ), f2_mul(lam, yQ))
            l1 = f2_muls(theta, (-xP) % P)
            l4 = f2_muls(lam, yP)
            C = f2_sqr(theta)
            D = f2_sqr(lam)
            Ee = f2_mul(D, lam)
            Fz = f2_mul(Z, C)
            G = f2_mul(X, D)
            H = f2_sub(f2_add(Ee, Fz), f2_muls(G, 2))
            X3 = f2_mul(lam, H)
            Y3 = f2_sub(f2_mul(theta, f2_sub(G, H)), f2_mul(Y, Ee))
            Z3 = f2_mul(Z, Ee)
            X, Y, Z = X3, Y3, Z3
            f = f12_mul_by_014(f, l0, l1, l4)
    return f12_conj(f)


def f12_cyc_exp_xabs(f):
    """f^|x| by square-and-multiply over |x| = 0xd201000000010000."""
    r = f
    for bit in bin(X_ABS)[3:]:
        r = f12_sqr(r)
        if bit == "1":
            r = f12_mul(r, f)
    return r


def f12_cyc_exp_x(f):
    """f^x for f in the cyclotomic subgroup (x < 0: inverse = conjugate)."""
    return f12_conj(f12_cyc_exp_xabs(f))


def final_exponentiation_x_chain(f):
    """f^(3 (p^12-1)/r), via 3 Phi12(p)/r = (x-1)^2 (x+p) (x^2+p^2-1) + 3
    (Hayashida-Hayasaka-Teruya). Equals final_exponentiation(f)^3."""
    f = f12_mul(f12_conj(f), f12_inv(f))
    f = f12_mul(f12_frob(f12_frob(f)), f)
    # t = f^(x-1)^2
    t = f12_mul(f12_cyc_exp_x(f), f12_conj(f))
    t = f12_mul(f12_cyc_exp_x(t), f12_conj(t))
    # t = t^(x+p)
    t = f12_mul(f12_cyc_exp_x(t), f12_frob(t))
    # t = t^(x^2 + p^2 - 1)
    t = f12_mul(f12_mul(f12_cyc_exp_x(f12_cyc_exp_x(t)), f12_frob(f12_frob(t))), f12_conj(t))
    # * f^3
    return f12_mul(t, f12_mul(f12_sqr(f), f))


# G1 endomorphism phi(x, y) = (beta x, y), beta a cube root of unity in Fp. Fast subgroup
# check (Scott 2021): P in G1 <=> phi(P) == -x^2 P, for the beta selected below.
_BETA_CANDIDATES = [b for b in (pow(2, (P - 1) // 3, P), pow(pow(2, (P - 1) // 3, P), 2, P))]


def _select_beta():
    for b in _BETA_CANDIDATES:
        phi = (G1_GEN[0] * b % P, G1_GEN[1])
        if pt_eq(FpOps, phi, pt_mul(FpOps, G1_GEN, -(X * X))):
            return b
    raise AssertionError("no beta")


BETA_G1 = _select_beta()


def g1_in_subgroup_fast(pt) -> bool:
    if pt is None:
        return True
    phi = (pt[0] * BETA_G1 % P, pt[1])
    return pt_eq(FpOps, phi, pt_mul(FpOps, pt, -(X * X)))


def g2_in_subgroup_fast(pt) -> bool:
    """Scott 2021: Q in G2 <=> psi(Q) == [x] Q."""
    if pt is None:
        return True
    return pt_eq(Fp2Ops, g2_psi(pt), pt_mul(Fp2Ops, pt, X))
