"""The MSM schedule of consensus_overlord_amd/csrc/msm.hpp (digits, counting sort, level pair
lists, bucket trees in the A array, bit-plane sums, window combination), restated step by step
over the oracle's G2 arithmetic and checked against sum r_i sigma_i computed directly. The
device kernels run exactly these index formulas; the point additions themselves are the
Fp-VM programs (gen.check_msm, test_vm_host.test_msm_programs_on_interpreter)."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle", "py"))

import bls12_381 as bls  # noqa: E402

F = bls.Fp2Ops
NBW, NB, NT, TM = 255, 4 * 255, 32, 64
LAMBDA_NEG = bls.X * bls.X   # -lambda = x^2 ; tau = -psi^2(sigma) = [lambda] sigma


def add(a, b):
    return bls.pt_add(F, a, b)


def model_msm(points, scalars64, valid):
    """msm.hpp on 2n points: point 2i = sigma_i (scalar = low half), 2i + 1 = tau_i (high half)."""
    n = len(points)
    tau = [bls.pt_neg(F, bls.g2_psi(bls.g2_psi(p))) for p in points]
    pt = lambda pid: (points if pid % 2 == 0 else tau)[pid // 2]   # noqa: E731
    half = lambda r, h: (r >> 32) & 0xFFFFFFFF if h else r & 0xFFFFFFFF   # noqa: E731
    # k_msm_count
    cnt = [0] * NB
    for i in range(n):
        if not valid[i]:
            continue
        for h in range(2):
            s = half(scalars64[i], h)
            for w in range(4):
                d = (s >> (8 * w)) & 255
                if d:
                    cnt[w * NBW + d - 1] += 1
    nlev = 1
    while (1 << nlev) < 2 * n:
        nlev += 1
    # k_msm_scan
    off, acc = [], 0
    for c in cnt:
        off.append(acc)
        acc += c
    off.append(acc)
    pf = []
    for lv in range(nlev):
        hh = 1 << lv
        row, acc = [], 0
        for c in cnt:
            row.append(acc)
            acc += (c + 1) // 2 if lv == 0 else ((c - hh + 2 * hh - 1) >> (lv + 1) if c > hh else 0)
        row.append(acc)
        pf.append(row)
    # k_msm_scatter (any order within a bucket)
    cur = list(off)
    ent = [None] * off[-1]
    order = list(range(n))
    random.Random(7).shuffle(order)   # the device's atomics order is arbitrary
    for i in order:
        if not valid[i]:
            continue
        for h in range(2):
            s = half(scalars64[i], h)
            for w in range(4):
                d = (s >> (8 * w)) & 255
                if d:
                    b = w * NBW + d - 1
                    ent[cur[b]] = 2 * i + h
                    cur[b] += 1

    def find(row, q):
        lo, hi = 0, NB
        while hi - lo > 1:
            mid = (lo + hi) >> 1
            if row[mid] <= q:
                lo = mid
            else:
                hi = mid
        return lo
    A = {}
    # level 0 (madd)
    for q in range(pf[0][NB]):
        b = find(pf[0], q)
        j = q - pf[0][b]
        k = 2 * j
        e = off[b] + k
        other = pt(ent[e + 1]) if k + 1 < cnt[b] else None
        A[pf[0][b] + j] = add(other, pt(ent[e]))
    for lv in range(1, nlev):
        row = pf[lv]
        for q in range(row[NB]):
            b = find(row, q)
            j = q - row[b]
            k = j << (lv + 1)
            ia = pf[0][b] + (k >> 1)
            ib = pf[0][b] + ((k + (1 << lv)) >> 1)
            A[ia] = add(A[ia], A[ib])

    def member(j, k):
        return ((j >> k) << (k + 1)) | (1 << k) | (j & ((1 << k) - 1))
    U = {}
    for q in range(NT * TM):
        t, i = q // TM, q % TM
        w, k = t >> 3, t & 7
        b0 = w * NBW + member(2 * i, k) - 1
        b1 = w * NBW + member(2 * i + 1, k) - 1
        U[q] = add(A[pf[0][b0]] if cnt[b0] else None, A[pf[0][b1]] if cnt[b1] else None)
    for lv in range(1, 7):
        per = TM >> lv
        for q in range(NT * per):
            t, i = q // per, q % per
            e = t * TM + (i << lv)
            U[e] = add(U[e], U[e + (1 << (lv - 1))])
    for h in range(1, 6):
        m = 1 << (h - 1)
        for q in range(NT >> h):
            e = 2 * m * q * TM
            U[e] = add(U[e], bls.pt_mul(F, U[e + m * TM], 1 << m))
    return U[0]


def direct(points, scalars64, valid):
    acc = None
    for p, r, v in zip(points, scalars64, valid):
        if v:
            a, b = r & 0xFFFFFFFF, r >> 32
            acc = add(acc, bls.pt_mul(F, p, (a + b * (-LAMBDA_NEG)) % bls.R))
    return acc


def _points(k):
    g2 = bls.pt_mul(F, bls.G2, 1) if hasattr(bls, "G2") else None
    rng = random.Random(0xC17A)
    base = g2 if g2 is not None else bls.hash_to_g2(b"\x00" * 32)
    return [bls.pt_mul(F, base, rng.randrange(1, bls.R)) for _ in range(k)]


def test_msm_schedule_matches_direct_sum():
    rng = random.Random(11)
    pts = _points(6)
    scal = [rng.getrandbits(64) for _ in pts]
    scal[1] = 0x00000001_000000FF           # one digit per window edge case
    scal[2] = 0xFFFFFFFF_FFFFFFFF           # every digit 255
    valid = [True, True, True, False, True, True]
    assert model_msm(pts, scal, valid) == direct(pts, scal, valid)


def test_msm_schedule_crowded_buckets():
    """many points in the same buckets (several tree levels), and a batch of one vote"""
    rng = random.Random(12)
    pts = _points(9)
    scal = [0x01010101_02020202 if k % 3 else rng.getrandbits(64) for k in range(len(pts))]
    valid = [True] * len(pts)
    assert model_msm(pts, scal, valid) == direct(pts, scal, valid)
    assert model_msm(pts[:1], scal[:1], [True]) == direct(pts[:1], scal[:1], [True])
    assert model_msm(pts[:2], scal[:2], [False, False]) is None
