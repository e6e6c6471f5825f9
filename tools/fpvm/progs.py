"""The Fp-VM programs of the batch verifier (built from alg.py), with their input / output
layouts. Input and output names are listed in the order the HIP side addresses them.

  vote     one vote of ovh_verify_batch: pk decompress + G1 subgroup
           check, sig decompress + G2 subgroup check, hash_to_G2 from (u0, u1), the RLC
           scalar product r pk (projective), f = Miller(r pk, H); stores f, sigma and
           tau = -psi^2(sigma) (affine) for the Pippenger MSM of sum r_i sigma_i
  vote_t   the same for a public key taken from the device validator table (ovh_set_validators:
           already decompressed and group-checked, projective) or a QC's aggregated key.
  vote1    a standalone vote (ovh_verify, n = 1, scalar 1): f = Miller(pk, H) Miller(-G1, sigma)
           as one two-pair Miller loop, so its check is final1 alone (no MSM, no partials)
  vote_t1  the same from a table / aggregated key (a QC's verify_aggregated_signature)
  final1   final exponentiation of f == 1
  rs       bisection only: r sigma = [a] sigma + [b] tau for one vote (the per-vote term the MSM
           sums), 32-step joint chain
  madd     MSM bucket level 0: B (projective) + A (affine)
  padd     MSM bucket levels >= 1 and the bit-plane sums: A + B (projective)
  hdbl<m>  MSM window combination: A + [2^m] B (projective), m = 1, 2, 4, 8, 16
  sigchk   aggregate_signatures: one signature's decompression + G2 subgroup check (the vote's
           "sig" section on its own), affine sigma out for the padd tree that sums them
  pkchk    a public key's decompression + G1 subgroup check (the validator table and the keys of
           verify_aggregated_signature), affine key out
  g1padd   A + B in G1 (projective): the pairwise tree that sums an aggregated key
  signg0   Crypto::sign, first part: H = hash_to_G2(u0, u1), the 15 sums of [|x|^i] H (GLS),
           the first 16 steps of the 4-digit chain (selb on the launch's scalar: the schedule
           does not depend on the secret)
  signg1   the next 16 chain steps (run three times)
  pkgen    acc -> [2^64] acc + [k] G1 over a 64-bit chunk k of a secret scalar (run four times)
  fold     4 partials (F_i in Fp12, S_i projective G2) -> (prod F_i, sum S_i)
  final    up to 4 partials -> prod F * Miller(-G1, sum S) -> final exponentiation == 1; also
           the bisection checks of the fallback (one group's partial, or one vote's (f, r sigma):
           e(r pk, H) e(-G1, r sigma) = (e(pk, H) / e(G1, sigma))^r == 1 iff the vote verifies).
"""
from __future__ import annotations

import os


from alg import G1X, G1Y, Alg
from ir import P, Prog

USE_SOP = False   # Fp2 products as sum-of-products ops (two lanes, no post-adds)

R_MONT = pow(2, 384, P)


def f12_names(prefix):
    return ["%s%d" % (prefix, j) for j in range(12)]


def g2p_names(prefix):
    return ["%s%d" % (prefix, j) for j in range(6)]


def flat12(f):
    return [c for f6 in f for f2 in f6 for c in f2]


def unflat12(v):
    return ((tuple(v[0:2]), tuple(v[2:4]), tuple(v[4:6])), (tuple(v[6:8]), tuple(v[8:10]), tuple(v[10:12])))


def flat_g2p(pt):
    return [c for f2 in pt for c in f2]


def unflat_g2p(v):
    return (tuple(v[0:2]), tuple(v[2:4]), tuple(v[4:6]))


# HBM state planes of a vote (ovhip.hip reads them through VM_S_* in vm_progs.inc):
# u0, u1 | sigma affine | tau = -psi^2(sigma) affine | f | r sigma (bisection only)
S_U, S_SIG, S_TAU, S_F, S_RS, S_TOTAL = 0, 4, 8, 12, 24, 30
# square roots by one Yao exponentiation (alg.Alg fast_sqrt) in the batch vote programs too:
# vote 2,985 -> 2,824 phases, vote_t 2,972 -> 2,629 (cost estimate -4% / -11%)
FAST_SQRT_BATCH = os.environ.get("OVH_FAST_SQRT_BATCH", "1") == "1"

VOTE_IN = ["pk_x", "pk_sort", "sig_x0", "sig_x1", "sig_sort", "u00", "u01", "u10", "u11"]
VOTE_OUT = ["pk_ok", "pk_grp", "sig_ok", "sig_grp", "h_inf"]
# stored straight to HBM planes by `st` ops as soon as they are final
VOTE_ST = [(n, S_F + k) for k, n in enumerate(f12_names("f"))] + \
    [("q%d" % k, S_SIG + k) for k in range(4)] + [("t%d" % k, S_TAU + k) for k in range(4)]


def affine_pair(a, Q):
    """sigma (affine) and tau = -psi^2(sigma) (affine: psi^2 keeps Z = 1) as 8 Fp values."""
    T = a.g2_neg_psi2(Q)
    return [Q[0][0], Q[0][1], Q[1][0], Q[1][1], T[0][0], T[0][1], T[1][0], T[1][1]]


def build_vote():
    p = Prog("vote")
    a = Alg(p, use_sop=USE_SOP, fast_sqrt=FAST_SQRT_BATCH)
    R = p.const(R_MONT)
    pkx = p.input("pk_x") * R
    sx = (p.input("sig_x0") * R, p.input("sig_x1") * R)
    u0 = (p.input("u00"), p.input("u01"))
    u1 = (p.input("u10"), p.input("u11"))
    pk_ok, (px, py) = a.g1_decompress(pkx, p.input("pk_sort"))
    Pp = (px, py, p.one)
    pk_grp, _ = a.g1_in_group(Pp)
    p.section = "sig"   # the signature's decompression + subgroup check (gen.py SEC_BIAS)
    sig_ok, (qx, qy) = a.g2_decompress(sx, p.input("sig_sort"))
    Qs = (qx, qy, (p.one, p.zero))
    sig_grp = a.g2_in_group(Qs)
    p.section = None
    H = a.hash_to_g2(u0, u1)
    h_inf = a.f2_is_zero(H[2])
    rP = a.pt_mul_glv("fp", Pp, a.g1_phi(Pp))          # projective: no inversion
    f = a.miller_loop(rP, H)
    for name, v in zip(VOTE_OUT, [pk_ok, pk_grp, sig_ok, sig_grp, h_inf]):
        p.output(name, v)
    for (name, plane), v in zip(VOTE_ST, flat12(f) + affine_pair(a, Qs)):
        p.store(name, v, plane)
    return p


VOTE_T_IN = ["pk_X", "pk_Y", "pk_Z", "sig_x0", "sig_x1", "sig_sort", "u00", "u01", "u10", "u11"]
VOTE_T_OUT = ["sig_ok", "sig_grp", "h_inf"]


def build_vote_t():
    p = Prog("vote_t")
    a = Alg(p, use_sop=USE_SOP, fast_sqrt=FAST_SQRT_BATCH)
    R = p.const(R_MONT)
    Pp = (p.input("pk_X"), p.input("pk_Y"), p.input("pk_Z"))
    sx = (p.input("sig_x0") * R, p.input("sig_x1") * R)
    u0 = (p.input("u00"), p.input("u01"))
    u1 = (p.input("u10"), p.input("u11"))
    p.section = "sig"   # the signature's decompression + subgroup check (gen.py SEC_BIAS)
    sig_ok, (qx, qy) = a.g2_decompress(sx, p.input("sig_sort"))
    Qs = (qx, qy, (p.one, p.zero))
    sig_grp = a.g2_in_group(Qs)
    p.section = None
    H = a.hash_to_g2(u0, u1)
    h_inf = a.f2_is_zero(H[2])
    rP = a.pt_mul_glv("fp", Pp, a.g1_phi(Pp))
    f = a.miller_loop(rP, H)
    for name, v in zip(VOTE_T_OUT, [sig_ok, sig_grp, h_inf]):
        p.output(name, v)
    for (name, plane), v in zip(VOTE_ST, flat12(f) + affine_pair(a, Qs)):
        p.store(name, v, plane)
    return p


VOTE1_ST = [(n, S_F + k) for k, n in enumerate(f12_names("f"))]


def build_vote1(table: bool):
    def build():
        p = Prog("vote_t1" if table else "vote1")
        a = Alg(p, use_sop=USE_SOP, fast_sqrt=True)
        R = p.const(R_MONT)
        if table:
            Pa = (p.input("pk_X"), p.input("pk_Y"), p.input("pk_Z"))
        else:
            pk_ok, (px, py) = a.g1_decompress(p.input("pk_x") * R, p.input("pk_sort"))
            pk_grp, _ = a.g1_in_group((px, py, p.one))
            Pa = (px, py)
        sx = (p.input("sig_x0") * R, p.input("sig_x1") * R)
        u0 = (p.input("u00"), p.input("u01"))
        u1 = (p.input("u10"), p.input("u11"))
        p.section = "sig"
        sig_ok, (qx, qy) = a.g2_decompress(sx, p.input("sig_sort"))
        Qs = (qx, qy, (p.one, p.zero))
        sig_grp = a.g2_in_group(Qs)
        p.section = None
        H = a.hash_to_g2(u0, u1)
        h_inf = a.f2_is_zero(H[2])
        # two single-pair Miller loops multiplied at the end, not one shared-f loop: the
        # signature's pair then runs beside hash_to_G2 (it needs sigma only), and the key's pair
        # after H is one line per step (vote1 critical path 2,452 -> 2,051 ops; the extra f
        # squarings fill idle lanes of the one wave)
        f = a.f12_mul(a.miller_loop_multi([(Pa, H)]), a.miller_loop_multi([((p.const(G1X), p.const(-G1Y)), Qs)]))
        flags = [sig_ok, sig_grp, h_inf] if table else [pk_ok, pk_grp, sig_ok, sig_grp, h_inf]
        for name, v in zip(VOTE_T_OUT if table else VOTE_OUT, flags):
            p.output(name, v)
        for (name, plane), v in zip(VOTE1_ST, flat12(f)):
            p.store(name, v, plane)
        # H (projective) for the message cache (ovhip.hip verify_one_locked): the next vote on
        # the same hash runs vote1h without hash_to_G2
        for (name, plane), v in zip(VOTE1H_ST, flat_g2p(H)):
            p.store(name, v, plane)
        return p
    return build


VOTE1H_ST = [(n, S_RS + k) for k, n in enumerate(g2p_names("h"))]
VOTE1H_IN = ["pk_x", "pk_sort", "sig_x0", "sig_x1", "sig_sort"] + g2p_names("h")
VOTE1H_OUT = ["pk_ok", "pk_grp", "sig_ok", "sig_grp"]
VOTE_T1H_IN = ["pk_X", "pk_Y", "pk_Z", "sig_x0", "sig_x1", "sig_sort"] + g2p_names("h")
VOTE_T1H_OUT = ["sig_ok", "sig_grp"]


def build_vote1h(table: bool):
    """vote1h / vote_t1h: vote1 / vote_t1 with H = hash_to_G2(hash) from the message cache (a
    vote on a hash already seen by this context: every vote of a round signs the same hash).
    Critical path: the key's decompression and Miller loop, beside the signature's (1,250 levels
    instead of hash_to_G2's 1,203 plus the Miller loop)."""
    def build():
        p = Prog("vote_t1h" if table else "vote1h")
        a = Alg(p, use_sop=USE_SOP, fast_sqrt=True)
        R = p.const(R_MONT)
        if table:
            Pa = (p.input("pk_X"), p.input("pk_Y"), p.input("pk_Z"))
        else:
            pk_ok, (px, py) = a.g1_decompress(p.input("pk_x") * R, p.input("pk_sort"))
            pk_grp, _ = a.g1_in_group((px, py, p.one))
            Pa = (px, py)
        sx = (p.input("sig_x0") * R, p.input("sig_x1") * R)
        H = unflat_g2p([p.input(n) for n in g2p_names("h")])
        sig_ok, (qx, qy) = a.g2_decompress(sx, p.input("sig_sort"))
        Qs = (qx, qy, (p.one, p.zero))
        sig_grp = a.g2_in_group(Qs)
        f = a.f12_mul(a.miller_loop_multi([(Pa, H)]), a.miller_loop_multi([((p.const(G1X), p.const(-G1Y)), Qs)]))
        flags = [sig_ok, sig_grp] if table else [pk_ok, pk_grp, sig_ok, sig_grp]
        for name, v in zip(VOTE_T1H_OUT if table else VOTE1H_OUT, flags):
            p.output(name, v)
        for (name, plane), v in zip(VOTE1_ST, flat12(f)):
            p.store(name, v, plane)
        return p
    return build


def build_votew(table: bool):
    """votew / votew_t: one vote of a small batch (n <= 1024, ovhip.hip k_vm_votew) on a whole
    64-lane wave: the vote's checks and H(m) as in vote1 / vote_t1, the RLC products r pk
    (projective, [a] pk + [b] phi(pk)) and r sigma ([a] sigma + [b] tau, the rs chain), and
    f = Miller(r pk, H) Miller(-G1, r sigma), so that FE(f) = (e(pk, H) / e(G1, sigma))^r: the
    batch's combined check is FE(prod f_i) == 1 with no MSM and no Miller loop in the final, and a
    vote's own check is FE(f_i) == 1. The sigma side (decompression, r sigma, its Miller loop)
    runs beside hash_to_G2 on the wave's idle lanes."""
    def build():
        p = Prog("votew_t" if table else "votew")
        a = Alg(p, use_sop=USE_SOP, fast_sqrt=True)
        R = p.const(R_MONT)
        if table:
            Pp = (p.input("pk_X"), p.input("pk_Y"), p.input("pk_Z"))
        else:
            pk_ok, (px, py) = a.g1_decompress(p.input("pk_x") * R, p.input("pk_sort"))
            Pp = (px, py, p.one)
            pk_grp, _ = a.g1_in_group(Pp)
        sx = (p.input("sig_x0") * R, p.input("sig_x1") * R)
        u0 = (p.input("u00"), p.input("u01"))
        u1 = (p.input("u10"), p.input("u11"))
        p.section = "sig"
        sig_ok, (qx, qy) = a.g2_decompress(sx, p.input("sig_sort"))
        Qs = (qx, qy, (p.one, p.zero))
        sig_grp = a.g2_in_group(Qs)
        rS = a.pt_mul_glv("f2", Qs, a.g2_neg_psi2(Qs))
        p.section = None
        H = a.hash_to_g2(u0, u1)
        h_inf = a.f2_is_zero(H[2])
        rP = a.pt_mul_glv("fp", Pp, a.g1_phi(Pp))
        f = a.f12_mul(a.miller_loop_multi([(rP, H)]), a.miller_loop_multi([((p.const(G1X), p.const(-G1Y)), rS)]))
        flags = [sig_ok, sig_grp, h_inf] if table else [pk_ok, pk_grp, sig_ok, sig_grp, h_inf]
        for name, v in zip(VOTE_T_OUT if table else VOTE_OUT, flags):
            p.output(name, v)
        for (name, plane), v in zip(VOTE1_ST, flat12(f)):
            p.store(name, v, plane)
        return p
    return build


QCPRE_IN = ["sig_x0", "sig_x1", "sig_sort", "u00", "u01", "u10", "u11"]
QCPRE_OUT = ["sig_ok", "sig_grp", "h_inf"]
QCPRE_ST = [(n, S_RS + k) for k, n in enumerate(g2p_names("h"))] + [(n, S_F + k) for k, n in enumerate(f12_names("g"))]
QCMIL_IN = ["pk_X", "pk_Y", "pk_Z"] + g2p_names("h") + f12_names("g")


def build_qcpre():
    """verify_aggregated_signature, the part that does not need the aggregated key (it runs on a
    side stream beside the keys' decompression, subgroup checks and tree sum): the signature's
    decompression + G2 subgroup check, H = hash_to_G2(u0, u1) and g = Miller(-G1, sigma); H
    (projective) and g go to HBM planes for qcmil."""
    p = Prog("qcpre")
    a = Alg(p, use_sop=USE_SOP, fast_sqrt=True)
    R = p.const(R_MONT)
    sx = (p.input("sig_x0") * R, p.input("sig_x1") * R)
    u0 = (p.input("u00"), p.input("u01"))
    u1 = (p.input("u10"), p.input("u11"))
    sig_ok, (qx, qy) = a.g2_decompress(sx, p.input("sig_sort"))
    Qs = (qx, qy, (p.one, p.zero))
    sig_grp = a.g2_in_group(Qs)
    H = a.hash_to_g2(u0, u1)
    h_inf = a.f2_is_zero(H[2])
    g = a.miller_loop_multi([((p.const(G1X), p.const(-G1Y)), Qs)])
    for name, v in zip(QCPRE_OUT, [sig_ok, sig_grp, h_inf]):
        p.output(name, v)
    for (name, plane), v in zip(QCPRE_ST, flat_g2p(H) + flat12(g)):
        p.store(name, v, plane)
    return p


def build_qcmil():
    """verify_aggregated_signature, the rest: f = Miller(apk, H) * g (apk projective, from the
    key tree), then final1."""
    p = Prog("qcmil")
    a = Alg(p, use_sop=USE_SOP)
    P = (p.input("pk_X"), p.input("pk_Y"), p.input("pk_Z"))
    H = unflat_g2p([p.input(n) for n in g2p_names("h")])
    g = unflat12([p.input(n) for n in f12_names("g")])
    f = a.f12_mul(a.miller_loop_multi([(P, H)]), g)
    for (name, plane), v in zip(VOTE1_ST, flat12(f)):
        p.store(name, v, plane)
    return p


def build_final1():
    p = Prog("final1")
    a = Alg(p, inv_op=True, use_sop=USE_SOP)
    F = unflat12([p.input(n) for n in f12_names("f")])
    p.output("ok", a.f12_eq_one(a.final_exp(F)))
    return p


RS_IN = ["q%d" % k for k in range(4)] + ["t%d" % k for k in range(4)]
RS_OUT = []
RS_ST = [(n, S_RS + k) for k, n in enumerate(g2p_names("s"))]


def build_rs():
    """[a] sigma + [b] tau for the vote's RLC value (a, b its 32-bit halves): the vote's r sigma,
    recomputed by the bisection when the batch's combined check failed."""
    p = Prog("rs")
    a = Alg(p, use_sop=USE_SOP)
    one = (p.one, p.zero)
    Q = ((p.input("q0"), p.input("q1")), (p.input("q2"), p.input("q3")), one)
    T = ((p.input("t0"), p.input("t1")), (p.input("t2"), p.input("t3")), one)
    rS = a.pt_mul_glv("f2", Q, T)
    for (name, plane), v in zip(RS_ST, flat_g2p(rS)):
        p.store(name, v, plane)
    return p


# ---- Pippenger MSM of sum r_i sigma_i (ovhip.hip k_msm_*): points are projective (X : Y : Z)
AFF_IN = ["a%d" % k for k in range(4)]
PA_IN = ["a%d" % k for k in range(6)]
PB_IN = ["b%d" % k for k in range(6)]
PT_OUT = ["s%d" % k for k in range(6)]


def _pt_in(p, names):
    v = [p.input(n) for n in names]
    return unflat_g2p(v) if len(v) == 6 else ((v[0], v[1]), (v[2], v[3]), (p.one, p.zero))


def build_madd():
    """bucket level 0: B + A, A affine (a point of the sorted entry list), B projective (the
    pair's other point with Z = 1, or the identity (0 : 1 : 0) for a bucket's odd last entry)."""
    p = Prog("madd")
    a = Alg(p, use_sop=USE_SOP)
    A = _pt_in(p, AFF_IN)
    B = _pt_in(p, PB_IN)
    for name, v in zip(PT_OUT, flat_g2p(a.pt_add("f2", B, A))):
        p.output(name, v)
    return p


def build_padd():
    p = Prog("padd")
    a = Alg(p, use_sop=USE_SOP)
    S = a.pt_add("f2", _pt_in(p, PA_IN), _pt_in(p, PB_IN))
    for name, v in zip(PT_OUT, flat_g2p(S)):
        p.output(name, v)
    return p


HDBL_M = (1, 2, 4, 8, 16)


def build_hdbl(m):
    """A + [2^m] B: one level of the MSM's window combination sum_t 2^t T_t (pairs of levels
    2^(2^(h-1)) apart)."""
    def build():
        p = Prog("hdbl%d" % m)
        a = Alg(p, use_sop=USE_SOP)
        B = _pt_in(p, PB_IN)
        for _ in range(m):
            B = a.pt_dbl("f2", B)
        for name, v in zip(PT_OUT, flat_g2p(a.pt_add("f2", _pt_in(p, PA_IN), B))):
            p.output(name, v)
        return p
    return build


SIGCHK_IN = ["sig_x0", "sig_x1", "sig_sort"]
SIGCHK_OUT = ["sig_ok", "sig_grp", "q0", "q1", "q2", "q3"]


def build_sigchk():
    p = Prog("sigchk")
    a = Alg(p, use_sop=USE_SOP, fast_sqrt=True)
    R = p.const(R_MONT)
    sx = (p.input("sig_x0") * R, p.input("sig_x1") * R)
    sig_ok, (qx, qy) = a.g2_decompress(sx, p.input("sig_sort"))
    sig_grp = a.g2_in_group((qx, qy, (p.one, p.zero)))
    for name, v in zip(SIGCHK_OUT, [sig_ok, sig_grp, qx[0], qx[1], qy[0], qy[1]]):
        p.output(name, v)
    return p


PKCHK_IN = ["pk_x", "pk_sort"]
PKCHK_OUT = ["pk_ok", "pk_grp", "p0", "p1"]


def build_pkchk():
    p = Prog("pkchk")
    a = Alg(p, use_sop=USE_SOP, fast_sqrt=True)
    R = p.const(R_MONT)
    pk_ok, (px, py) = a.g1_decompress(p.input("pk_x") * R, p.input("pk_sort"))
    pk_grp, _ = a.g1_in_group((px, py, p.one))
    for name, v in zip(PKCHK_OUT, [pk_ok, pk_grp, px, py]):
        p.output(name, v)
    return p


PKDEC_OUT = ["pk_ok"]
G1GRP_IN = ["pk_X", "pk_Y", "pk_Z"]
G1GRP_OUT = ["pk_grp"]


def build_g1grp():
    """verify_aggregated_signature with keys outside G1 (BlsPublicKey::aggregate does not
    group-check, blst's verify checks the SUM, consensus.rs:371,378-380): the G1 subgroup check of
    the aggregated key (projective)."""
    p = Prog("g1grp")
    a = Alg(p, use_sop=USE_SOP)
    grp, _ = a.g1_in_group((p.input("pk_X"), p.input("pk_Y"), p.input("pk_Z")))
    p.output("pk_grp", grp)
    return p



def build_pkdec():
    """aggregate_signatures' key validation (consensus.rs:435-436: the keys are only parsed):
    the 48-byte key's decompression alone -- x^3 + 4 a square -- with no subgroup check."""
    p = Prog("pkdec")
    a = Alg(p, use_sop=USE_SOP, fast_sqrt=True)
    R = p.const(R_MONT)
    pk_ok, _ = a.g1_decompress(p.input("pk_x") * R, p.input("pk_sort"))
    p.output("pk_ok", pk_ok)
    return p


G1A_IN = ["a%d" % k for k in range(3)]
G1B_IN = ["b%d" % k for k in range(3)]
G1_OUT = ["s%d" % k for k in range(3)]


def build_g1padd():
    p = Prog("g1padd")
    a = Alg(p, use_sop=USE_SOP)
    S = a.pt_add("fp", tuple(p.input(n) for n in G1A_IN), tuple(p.input(n) for n in G1B_IN))
    for name, v in zip(G1_OUT, S):
        p.output(name, v)
    return p


def _smul64(a, acc, T, F="fp"):
    """acc -> [2^64] acc + [k] H over the launch scalar's 64 bits k, 2-bit windows MSB first:
    two doublings and one complete addition of T[v] (T = H, 2H, 3H; v = 0 adds the identity,
    picked by two selb levels off the doubling chain). F: "fp" (G1, pkgen) or "f2" (G2)."""
    H, H2, H3 = T
    O = a.pt_inf(F)
    for w in range(31, -1, -1):
        # the window's addend is selected once the previous window's sum exists
        dep = acc[2] if F == "fp" else acc[2][0]
        lo = a.pt_selb(F, 2 * w, O, H, dep)
        hi = a.pt_selb(F, 2 * w, H2, H3, dep)
        ad = a.pt_selb(F, 2 * w + 1, lo, hi, dep)
        acc = a.pt_dbl(F, a.pt_dbl(F, acc))
        acc = a.pt_add(F, acc, ad)
    return acc


SIGNG_T = ["t%d" % k for k in range(90)]   # T[b] = sum of B_i over the set bits i of b, b = 1..15


def _signg_steps(a, acc, T, first=False):
    """16 steps of the 4-dimensional GLS chain acc -> 2 acc + T[b], b = the step's 4 selb bits
    (bit 4t + i of the launch scalar: digit i at this step), MSB first; T[0] = O."""
    tab = [a.pt_inf("f2")] + T
    for t in range(15, -1, -1):
        dep = None if (first and t == 15) else acc[2][0]
        lv = tab
        for i in range(4):   # selb tree: digit i picks between the entries with bit i clear / set
            lv = [a.pt_selb("f2", 4 * t + i, lv[2 * m], lv[2 * m + 1], dep) for m in range(len(lv) // 2)]
        ad = lv[0]
        acc = ad if (first and t == 15) else a.pt_add("f2", a.pt_dbl("f2", acc), ad)
    return acc


def _gls_table(a, H):
    """B_i = [|x|^i] H = (-psi)^i (H) on G2 (psi acts as x < 0), and T[b] = sum_{i in b} B_i."""
    B1 = a.pt_neg("f2", a.g2_psi(H))
    B2 = a.g2_psi(a.g2_psi(H))
    B3 = a.pt_neg("f2", a.g2_psi(B2))
    B = [H, B1, B2, B3]
    T = {0: None}
    for b in range(1, 16):
        low = b & (b - 1)          # b without its top set bit
        top = B[(b ^ low).bit_length() - 1]
        T[b] = top if low == 0 else a.pt_add("f2", T[low], top)
    return [T[b] for b in range(1, 16)]


def build_signg0():
    """Crypto::sign by the 4-dimensional GLS decomposition k = sum k_i |x|^i (k_i < 2^64): H =
    hash_to_G2(u0, u1), the 15-entry table of sums of [|x|^i] H, and the first 16 of the 64 chain
    steps (digit bits 63..48); the secret enters only as selb bits."""
    p = Prog("signg0")
    a = Alg(p, use_sop=USE_SOP)
    H = a.hash_to_g2((p.input("u00"), p.input("u01")), (p.input("u10"), p.input("u11")))
    T = _gls_table(a, H)
    acc = _signg_steps(a, None, T, first=True)
    flat_t = [c for pt in T for c in flat_g2p(pt)]
    for name, v in zip(SIGN_ACC + SIGNG_T, flat_g2p(acc) + flat_t):
        p.output(name, v)
    return p


def build_signg1():
    """The next 16 GLS chain steps (run three times)."""
    p = Prog("signg1")
    a = Alg(p, use_sop=USE_SOP)
    acc = _pt_in(p, SIGN_ACC)
    T = [unflat_g2p([p.input(n) for n in SIGNG_T[6 * j:6 * j + 6]]) for j in range(15)]
    for name, v in zip(SIGN_ACC, flat_g2p(_signg_steps(a, acc, T))):
        p.output(name, v)
    return p


PKGEN_ACC = ["c0", "c1", "c2"]


def build_pkgen():
    """Public key from a secret scalar (ConsensusCrypto::new, ovh_sk_to_pk): acc -> [2^64] acc +
    [k] G1 over the launch scalar's 64 bits, 2-bit windows over the constants G1, 2 G1, 3 G1;
    run four times from the identity (k the scalar's 64-bit chunks, most significant first), the
    secret only as selb bits."""
    p = Prog("pkgen")
    a = Alg(p, use_sop=USE_SOP)
    G = (p.const(G1X), p.const(G1Y), p.one)
    G2 = a.pt_dbl("fp", G)        # constants: the IR folds operations on constants
    G3 = a.pt_add("fp", G2, G)
    acc = tuple(p.input(n) for n in PKGEN_ACC)
    for name, v in zip(PKGEN_ACC, _smul64(a, acc, (G, G2, G3), F="fp")):
        p.output(name, v)
    return p


SIGN0_IN = ["u00", "u01", "u10", "u11"]
SIGN_ACC = ["c%d" % k for k in range(6)]


FOLD_K = 4
FOLD_IN = [n for k in range(FOLD_K) for n in f12_names("F%d_" % k) + g2p_names("S%d_" % k)]
FOLD_OUT = f12_names("F") + g2p_names("S")


def build_fold():
    p = Prog("fold")
    a = Alg(p, use_sop=USE_SOP)
    Fs, Ss = [], []
    for k in range(FOLD_K):
        Fs.append(unflat12([p.input(n) for n in f12_names("F%d_" % k)]))
        Ss.append(unflat_g2p([p.input(n) for n in g2p_names("S%d_" % k)]))
    F01 = a.f12_mul(Fs[0], Fs[1])
    F23 = a.f12_mul(Fs[2], Fs[3])
    S01 = a.pt_add("f2", Ss[0], Ss[1])
    S23 = a.pt_add("f2", Ss[2], Ss[3])
    F = a.f12_mul(F01, F23)
    S = a.pt_add("f2", S01, S23)
    for name, v in zip(FOLD_OUT, flat12(F) + flat_g2p(S)):
        p.output(name, v)
    return p


FINAL_IN = FOLD_IN
FINAL_OUT = ["ok"]


def build_final():
    p = Prog("final")
    a = Alg(p, inv_op=True, use_sop=USE_SOP)
    Fs, Ss = [], []
    for k in range(FOLD_K):
        Fs.append(unflat12([p.input(n) for n in f12_names("F%d_" % k)]))
        Ss.append(unflat_g2p([p.input(n) for n in g2p_names("S%d_" % k)]))
    F = a.f12_mul(a.f12_mul(Fs[0], Fs[1]), a.f12_mul(Fs[2], Fs[3]))
    S = a.pt_add("f2", a.pt_add("f2", Ss[0], Ss[1]), a.pt_add("f2", Ss[2], Ss[3]))
    s_inf = a.f2_is_zero(S[2])
    ng1 = (p.const(G1X), p.const(-G1Y))
    m = a.miller_loop(ng1, S)
    one = a.f12_one()
    m = unflat12([p.sel(s_inf, x, y) for x, y in zip(flat12(m), flat12(one))])
    fe = a.final_exp(a.f12_mul(F, m))
    p.output("ok", a.f12_eq_one(fe))
    return p


PROGRAMS = {
    "vote": (build_vote, VOTE_IN, VOTE_OUT),
    "vote_t": (build_vote_t, VOTE_T_IN, VOTE_T_OUT),
    "fold": (build_fold, FOLD_IN, FOLD_OUT),
    "final": (build_final, FINAL_IN, FINAL_OUT),
    "rs": (build_rs, RS_IN, RS_OUT),
    "madd": (build_madd, AFF_IN + PB_IN, PT_OUT),
    "padd": (build_padd, PA_IN + PB_IN, PT_OUT),
}
for _m in HDBL_M:
    PROGRAMS["hdbl%d" % _m] = (build_hdbl(_m), PA_IN + PB_IN, PT_OUT)
PROGRAMS["sigchk"] = (build_sigchk, SIGCHK_IN, SIGCHK_OUT)
PROGRAMS["pkchk"] = (build_pkchk, PKCHK_IN, PKCHK_OUT)
PROGRAMS["vote1"] = (build_vote1(False), VOTE_IN, VOTE_OUT)
PROGRAMS["vote_t1"] = (build_vote1(True), VOTE_T_IN, VOTE_T_OUT)
PROGRAMS["final1"] = (build_final1, f12_names("f"), ["ok"])
PROGRAMS["pkgen"] = (build_pkgen, PKGEN_ACC, PKGEN_ACC)
PROGRAMS["signg0"] = (build_signg0, SIGN0_IN, SIGN_ACC + SIGNG_T)
PROGRAMS["signg1"] = (build_signg1, SIGN_ACC + SIGNG_T, SIGN_ACC)
PROGRAMS["vote1h"] = (build_vote1h(False), VOTE1H_IN, VOTE1H_OUT)
PROGRAMS["vote_t1h"] = (build_vote1h(True), VOTE_T1H_IN, VOTE_T1H_OUT)
PROGRAMS["qcpre"] = (build_qcpre, QCPRE_IN, QCPRE_OUT)
PROGRAMS["qcmil"] = (build_qcmil, QCMIL_IN, [])
PROGRAMS["votew"] = (build_votew(False), VOTE_IN, VOTE_OUT)
PROGRAMS["votew_t"] = (build_votew(True), VOTE_T_IN, VOTE_T_OUT)
PROGRAMS["g1padd"] = (build_g1padd, G1A_IN + G1B_IN, G1_OUT)

# ---------------------------------------------------------------- same-message batches (r04)
# Every vote of a round signs the same hash (consensus.rs:169-175: Vote has no voter field), so
# a batch of n votes over G distinct hashes checks
#   prod_g e(sum_{i in g} r_i pk_i, H_g) * e(-G1, sum_i r_i sigma_i) == 1
# with one hash_to_G2 and one Miller loop per hash: per vote only the key / signature checks and
# r_i pk_i (ovhip.hip verify_samemsg_locked).
VSAME_IN = ["pk_x", "pk_sort", "sig_x0", "sig_x1", "sig_sort"]
VSAME_OUT = ["pk_ok", "pk_grp", "sig_ok", "sig_grp"]
VSAME_T_IN = ["pk_X", "pk_Y", "pk_Z", "sig_x0", "sig_x1", "sig_sort"]
VSAME_T_OUT = ["sig_ok", "sig_grp"]
# sigma / tau for the MSM (as the vote program), r pk (homogeneous projective) in the first three
# f planes (the batch's f planes are free on this path until the bisection)
VSAME_ST = [("q%d" % k, S_SIG + k) for k in range(4)] + [("t%d" % k, S_TAU + k) for k in range(4)] + \
    [("r%d" % k, S_F + k) for k in range(3)]
# group slab planes (per distinct hash): u0, u1 | H projective | f = Miller(apk, H)
G_U, G_H, G_F, G_PLANES = 0, 4, 10, 22
H2G_IN = ["u00", "u01", "u10", "u11"]
H2G_OUT = ["h_inf"]
GMIL_IN = ["pk_X", "pk_Y", "pk_Z"] + g2p_names("h")


def build_vsame(table: bool):
    def build():
        """vsame / vsame_t: one vote of a same-message batch -- the key's decompression + G1
        subgroup check (vsame; vsame_t takes a validator-table point), the signature's
        decompression + G2 subgroup check, r pk = [a] pk + [b] phi(pk) with the vote's RLC value;
        stores sigma, tau (the MSM's terms) and r pk."""
        p = Prog("vsame_t" if table else "vsame")
        a = Alg(p, use_sop=USE_SOP, fast_sqrt=FAST_SQRT_BATCH)
        R = p.const(R_MONT)
        outs = []
        if table:
            Pp = (p.input("pk_X"), p.input("pk_Y"), p.input("pk_Z"))
        else:
            pk_ok, (px, py) = a.g1_decompress(p.input("pk_x") * R, p.input("pk_sort"))
            Pp = (px, py, p.one)
            pk_grp, _ = a.g1_in_group(Pp)
            outs = [pk_ok, pk_grp]
        p.section = "sig"
        sx = (p.input("sig_x0") * R, p.input("sig_x1") * R)
        sig_ok, (qx, qy) = a.g2_decompress(sx, p.input("sig_sort"))
        Qs = (qx, qy, (p.one, p.zero))
        sig_grp = a.g2_in_group(Qs)
        p.section = None
        rP = a.pt_mul_glv("fp", Pp, a.g1_phi(Pp))
        for name, v in zip(VSAME_T_OUT if table else VSAME_OUT, outs + [sig_ok, sig_grp]):
            p.output(name, v)
        for (name, plane), v in zip(VSAME_ST, affine_pair(a, Qs) + list(rP)):
            p.store(name, v, plane)
        return p
    return build


def build_h2g():
    """H = hash_to_G2(u0, u1) of one distinct hash of a same-message batch -> the group slab's H
    planes, and the H-is-infinity flag."""
    p = Prog("h2g")
    a = Alg(p, use_sop=USE_SOP, fast_sqrt=True)
    H = a.hash_to_g2((p.input("u00"), p.input("u01")), (p.input("u10"), p.input("u11")))
    p.output("h_inf", a.f2_is_zero(H[2]))
    for k, v in enumerate(flat_g2p(H)):
        p.store("h%d" % k, v, G_H + k)
    return p


def build_gmil():
    """f_g = Miller(apk_g, H_g) of one distinct hash (apk_g = sum of its votes' r pk, projective)
    -> the group slab's f planes."""
    p = Prog("gmil")
    a = Alg(p, use_sop=USE_SOP)
    P = (p.input("pk_X"), p.input("pk_Y"), p.input("pk_Z"))
    H = unflat_g2p([p.input(n) for n in g2p_names("h")])
    f = a.miller_loop_multi([(P, H)])
    for k, v in enumerate(flat12(f)):
        p.store("f%d" % k, v, G_F + k)
    return p


PROGRAMS["pkdec"] = (build_pkdec, PKCHK_IN, PKDEC_OUT)
PROGRAMS["g1grp"] = (build_g1grp, G1GRP_IN, G1GRP_OUT)
GFIN_IN = f12_names("F") + ["pk_X", "pk_Y", "pk_Z"] + g2p_names("h") + g2p_names("S")


def build_gfin():
    """The combined check of a same-message batch: F (the other hashes' Miller values, folded) x
    Miller(apk_0, H_0) x Miller(-G1, S) as one two-pair Miller loop, then the final
    exponentiation == 1 (apk_0 and S not the identity: the kernel decides otherwise)."""
    p = Prog("gfin")
    a = Alg(p, inv_op=True, use_sop=USE_SOP)
    F = unflat12([p.input(n) for n in f12_names("F")])
    P0 = (p.input("pk_X"), p.input("pk_Y"), p.input("pk_Z"))
    H = unflat_g2p([p.input(n) for n in g2p_names("h")])
    S = unflat_g2p([p.input(n) for n in g2p_names("S")])
    ng1 = (p.const(G1X), p.const(-G1Y))
    m = a.miller_loop_multi([(P0, H), (ng1, S)])
    p.output("ok", a.f12_eq_one(a.final_exp(a.f12_mul(F, m))))
    return p


PROGRAMS["gfin"] = (build_gfin, GFIN_IN, ["ok"])
PROGRAMS["vsame"] = (build_vsame(False), VSAME_IN, VSAME_OUT)
PROGRAMS["vsame_t"] = (build_vsame(True), VSAME_T_IN, VSAME_T_OUT)
PROGRAMS["h2g"] = (build_h2g, H2G_IN, H2G_OUT)
PROGRAMS["gmil"] = (build_gmil, GMIL_IN, [])
# the same vote programs on 8-lane slices (eight votes per wave) for large same-message batches:
# 1,504 phases per eight votes against 1,288 per four (per vote -40% on gen.py's cost model);
# the 16-lane form keeps the shorter per-vote latency for small batches (ovhip.hip VSAME8_MIN)
PROGRAMS["vsame8"] = (build_vsame(False), VSAME_IN, VSAME_OUT)
PROGRAMS["vsame8_t"] = (build_vsame(True), VSAME_T_IN, VSAME_T_OUT)
