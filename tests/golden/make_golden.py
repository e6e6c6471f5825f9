#!/usr/bin/env python3
"""Generate tests/golden/golden_v1.json from the CPU oracle (oracle/py).

The reference (Rust + un-vendored blst) cannot be built or imported here,
so these vectors come from the from-scratch Python oracle, which is itself pinned by
published known-answer values (tests/test_oracle_kat.py: RFC 9380 expand_message_xmd and
hash_to_curve G2 vectors, GB/T 32905 SM3 vectors, the BLS12-381 generators).

Run:  python tests/golden/make_golden.py      (takes ~1-2 minutes)
"""
from __future__ import annotations

import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle", "py"))

import bls12_381 as bls  # noqa: E402
import overlord_oracle as ov  # noqa: E402

F1, F2 = bls.FpOps, bls.Fp2Ops


def hx(b: bytes) -> str:
    return bytes(b).hex()


def rnd_e1(rng):
    while True:
        x = rng.randrange(bls.P)
        y = bls.fp_sqrt(x ** 3 + 4)
        if y is not None:
            return (x, y)


def rnd_e2(rng):
    while True:
        x = (rng.randrange(bls.P), rng.randrange(bls.P))
        y = bls.f2_sqrt(bls.f2_add(bls.f2_mul(bls.f2_sqr(x), x), bls.B2))
        if y is not None:
            return (x, y)


def non_square_x_g1(rng):
    while True:
        x = rng.randrange(bls.P)
        if bls.fp_sqrt(x ** 3 + 4) is None:
            return x


def non_square_x_g2(rng):
    while True:
        x = (rng.randrange(bls.P), rng.randrange(bls.P))
        if bls.f2_sqrt(bls.f2_add(bls.f2_mul(bls.f2_sqr(x), x), bls.B2)) is None:
            return x


def main():
    rng = random.Random(0xC17A)
    out = {"version": 1, "dst": bls.DST_NUL.decode(), "generator": "tests/golden/make_golden.py"}

    # ---- keys, votes, signatures (synthetic workload definition) ----
    nkeys = 8
    keys, votes = [], []
    for i in range(nkeys):
        sk = ov.synth_sk(i)
        pk = bls.sk_to_pk(sk)
        keys.append({"i": i, "sk": "%064x" % sk, "pk": hx(bls.g1_compress(pk)), "pk_uncompressed": hx(bls.g1_serialize(pk))})
        bh = ov.synth_block_hash(i)
        rlp = ov.rlp_vote(1 + i // 64, i % 3, ov.PRECOMMIT, bh)
        digest = ov.sm3(rlp)
        _, sig = ov.sign(sk, digest)
        votes.append({"i": i, "block_hash": hx(bh), "rlp": hx(rlp), "digest": hx(digest), "sig": hx(sig)})
    out["keys"] = keys
    out["votes"] = votes

    # ---- hash_to_g2 on digests (uncompressed, c1||c0 per coordinate) ----
    out["hash_to_g2"] = [{"msg": v["digest"], "point": hx(bls.g2_serialize(bls.hash_to_g2(bytes.fromhex(v["digest"]))))} for v in votes[:4]]

    # ---- verify cases ----
    sig = lambda i: bytes.fromhex(votes[i]["sig"])  # noqa: E731
    dig = lambda i: bytes.fromhex(votes[i]["digest"])  # noqa: E731
    pk = lambda i: bytes.fromhex(keys[i]["pk"])  # noqa: E731
    cases = []

    def add(name, s, h, p):
        code = ov.verify_signature(s, h, p)
        cases.append({"name": name, "sig": hx(s), "hash": hx(h), "pk": hx(p), "code": code})

    for i in range(nkeys):
        add("valid_%d" % i, sig(i), dig(i), pk(i))
    add("wrong_msg", sig(0), dig(1), pk(0))
    add("wrong_pk", sig(0), dig(0), pk(1))
    add("swapped_sig", sig(1), dig(0), pk(0))
    add("pk_uncompressed", sig(2), dig(2), bytes.fromhex(keys[2]["pk_uncompressed"]))
    s_un = bls.g2_serialize(bls.g2_from_bytes(sig(3)))
    add("sig_uncompressed", s_un, dig(3), pk(3))
    # sigma + G2 generator (valid point, wrong signature) -- the config-5 corruption
    bad = bls.g2_compress(bls.pt_add(F2, bls.g2_from_bytes(sig(4)), bls.G2_GEN))
    add("sig_plus_g2", bad, dig(4), pk(4))
    # wrong lengths
    add("hash_31", sig(0), dig(0)[:31], pk(0))
    add("hash_33", sig(0), dig(0) + b"\x00", pk(0))
    add("pk_47", sig(0), dig(0), pk(0)[:47])
    add("sig_95", sig(0)[:95], dig(0), pk(0))
    add("empty_all", b"", dig(0), b"")
    # flag errors
    p_noflag = bytearray(pk(0)); p_noflag[0] &= 0x7F
    add("pk_compressed_bit_clear", sig(0), dig(0), bytes(p_noflag))
    s_noflag = bytearray(sig(0)); s_noflag[0] &= 0x7F
    add("sig_compressed_bit_clear", bytes(s_noflag), dig(0), pk(0))
    p_inf_dirty = bytearray(bls.g1_compress(None)); p_inf_dirty[47] = 1
    add("pk_infinity_dirty", sig(0), dig(0), bytes(p_inf_dirty))
    s_inf_dirty = bytearray(bls.g2_compress(None)); s_inf_dirty[0] |= 0x20
    add("sig_infinity_sortflag", bytes(s_inf_dirty), dig(0), pk(0))
    add("pk_infinity", sig(0), dig(0), bls.g1_compress(None))
    add("sig_infinity", bls.g2_compress(None), dig(0), pk(0))
    # x >= p
    xp = bytearray(bls.P.to_bytes(48, "big")); xp[0] |= 0x80
    add("pk_x_eq_p", sig(0), dig(0), bytes(xp))
    sx = bytearray(bls.P.to_bytes(48, "big") + bytes(48)); sx[0] |= 0x80
    add("sig_x1_eq_p", bytes(sx), dig(0), pk(0))
    sx0 = bytearray(bytes(48) + bls.P.to_bytes(48, "big")); sx0[0] |= 0x80; sx0[47] = 1
    add("sig_x0_eq_p", bytes(sx0), dig(0), pk(0))
    # not on curve
    x = non_square_x_g1(rng); b = bytearray(x.to_bytes(48, "big")); b[0] |= 0x80
    add("pk_not_on_curve", sig(0), dig(0), bytes(b))
    x2 = non_square_x_g2(rng); b2 = bytearray(x2[1].to_bytes(48, "big") + x2[0].to_bytes(48, "big")); b2[0] |= 0x80
    add("sig_not_on_curve", bytes(b2), dig(0), pk(0))
    # on curve, not in subgroup
    add("pk_not_in_g1", sig(0), dig(0), bls.g1_compress(rnd_e1(rng)))
    add("sig_not_in_g2", bls.g2_compress(rnd_e2(rng)), dig(0), pk(0))
    # x = 0 (G1: (0, +-2) on curve, rejected by blst at parse)
    z = bytearray(48); z[0] = 0x80
    add("pk_x_zero", sig(0), dig(0), bytes(z))
    # uncompressed with sort flag set -> bad encoding
    pu = bytearray(bytes.fromhex(keys[0]["pk_uncompressed"])); pu[0] |= 0x20
    add("pk_uncompressed_sortflag", sig(0), dig(0), bytes(pu))
    # uncompressed off-curve
    pu2 = bytearray(bytes.fromhex(keys[0]["pk_uncompressed"])); pu2[95] ^= 1
    add("pk_uncompressed_off_curve", sig(0), dig(0), bytes(pu2))
    out["verify"] = cases

    # ---- aggregation (configs 1 and 2) ----
    agg = []
    sigs4 = [sig(i) for i in range(4)]
    pks4 = [pk(i) for i in range(4)]
    code, a = ov.aggregate_signatures(sigs4, pks4)
    agg.append({"name": "agg4", "sigs": [hx(s) for s in sigs4], "pks": [hx(p) for p in pks4], "code": code, "out": hx(a) if a else None})
    code, a = ov.aggregate_signatures([], [])
    agg.append({"name": "agg_empty", "sigs": [], "pks": [], "code": code, "out": None})
    code, a = ov.aggregate_signatures(sigs4, pks4[:3])
    agg.append({"name": "agg_len_mismatch", "sigs": [hx(s) for s in sigs4], "pks": [hx(p) for p in pks4[:3]], "code": code, "out": None})
    badsig = bls.g2_compress(rnd_e2(rng))
    code, a = ov.aggregate_signatures(sigs4[:2] + [badsig], pks4[:3])
    agg.append({"name": "agg_not_in_g2", "sigs": [hx(s) for s in sigs4[:2] + [badsig]], "pks": [hx(p) for p in pks4[:3]], "code": code, "out": None})
    code, a = ov.aggregate_signatures(sigs4[:2], [pks4[0], pks4[1][:47]])
    agg.append({"name": "agg_bad_pk", "sigs": [hx(s) for s in sigs4[:2]], "pks": [hx(pks4[0]), hx(pks4[1][:47])], "code": code, "out": None})
    # sigma and -sigma sum to infinity
    neg = bls.g2_compress(bls.pt_neg(F2, bls.g2_from_bytes(sig(0))))
    code, a = ov.aggregate_signatures([sig(0), neg], [pk(0), pk(0)])
    agg.append({"name": "agg_to_infinity", "sigs": [hx(sig(0)), hx(neg)], "pks": [hx(pk(0))] * 2, "code": code, "out": hx(a)})
    out["aggregate"] = agg

    pkagg = []
    for name, voters in (("pkagg4", pks4), ("pkagg_empty", []), ("pkagg1", pks4[:1])):
        code, a = ov.aggregate_public_keys(voters)
        pkagg.append({"name": name, "pks": [hx(p) for p in voters], "code": code, "out": hx(a) if a else None})
    out["aggregate_pks"] = pkagg

    # ---- QC: 100 validators, first 67 sign the same precommit (config 2) ----
    nval, nq = 100, 67
    qc_hash = ov.vote_hash(7, 0, ov.PRECOMMIT, ov.synth_block_hash(9999))
    qsks = [ov.synth_sk(1000 + i) for i in range(nval)]
    qpks = [bls.g1_compress(bls.sk_to_pk(s)) for s in qsks]
    H = bls.hash_to_g2(qc_hash)
    qsigs = [bls.g2_compress(bls.pt_mul(F2, H, s)) for s in qsks[:nq]]
    code, qagg = ov.aggregate_signatures(qsigs, qpks[:nq])
    assert code == 0
    _, qaggpk = ov.aggregate_public_keys(qpks[:nq])
    qc = {"hash": hx(qc_hash), "pks": [hx(p) for p in qpks], "sigs": [hx(s) for s in qsigs], "agg_sig": hx(qagg), "agg_pk": hx(qaggpk)}
    qc["verify_ok"] = ov.verify_aggregated_signature(qagg, qc_hash, qpks[:nq])
    qc["verify_missing_one"] = ov.verify_aggregated_signature(qagg, qc_hash, qpks[:nq - 1])
    qc["verify_wrong_hash"] = ov.verify_aggregated_signature(qagg, ov.sm3(b"x"), qpks[:nq])
    qc["verify_empty"] = ov.verify_aggregated_signature(qagg, qc_hash, [])
    qc["verify_hash_31"] = ov.verify_aggregated_signature(qagg, qc_hash[:31], qpks[:nq])
    qc["verify_bad_pk"] = ov.verify_aggregated_signature(qagg, qc_hash, qpks[:nq - 1] + [qpks[0][:40]])
    out["qc"] = qc

    # ---- a GT value: x-chain final exponentiation of e(G1,G2)'s Miller output (for kernel-level checks) ----
    f = bls.miller_loop(bls.G1_GEN, bls.G2_GEN)
    e3 = bls.final_exponentiation_x_chain(f)
    flat = [c for f6 in e3 for f2_ in f6 for c in f2_]
    out["gt_e_g1_g2_cubed"] = ["%096x" % c for c in flat]

    path = os.path.join(HERE, "golden_v1.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
