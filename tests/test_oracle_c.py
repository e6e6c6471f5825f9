"""The C restatement of the oracle (oracle/c/bls_oracle.c) against the golden fixtures (made by
the Python oracle, itself pinned to RFC 9380 / generator KATs in test_oracle_kat.py) and
against the Python oracle on seeded random cases: verdict codes, signatures, aggregates and
hash-to-G2 points must be bit-exact."""
import random

import numpy as np
import pytest

import bls12_381 as bls
import orc
import overlord_oracle as ov


def _b(h):
    return bytes.fromhex(h)


def test_gt_value(golden):
    assert orc.gt_g1g2() == golden["gt_e_g1_g2_cubed"]


def test_hash_to_g2_golden(golden):
    dst = golden["dst"].encode()
    for h in golden["hash_to_g2"]:
        assert orc.hash_to_g2(_b(h["msg"]), dst).hex() == h["point"]


def test_hash_to_g2_rfc9380():
    from test_oracle_kat import RFC9380_G2_DST, RFC9380_G2_RO
    for msg, (x0, x1, y0, y1) in RFC9380_G2_RO.items():
        out = orc.hash_to_g2(msg, RFC9380_G2_DST)
        want = b"".join(v.to_bytes(48, "big") for v in (x1, x0, y1, y0))
        assert out == want


def test_keys_and_signatures(golden):
    for k, v in zip(golden["keys"], golden["votes"]):
        c, pk = orc.sk_to_pk(_b(k["sk"]))
        assert c == 0 and pk.hex() == k["pk"]
        c, sig = orc.sign(_b(k["sk"]), _b(v["digest"]))
        assert c == 0 and sig.hex() == v["sig"]


def test_verify_codes(golden):
    for c in golden["verify"]:
        assert orc.verify(_b(c["sig"]), _b(c["hash"]), _b(c["pk"])) == c["code"], c["name"]


def test_aggregates(golden):
    for c in golden["aggregate"]:
        code, out = orc.aggregate_sigs([_b(s) for s in c["sigs"]], [_b(p) for p in c["pks"]])
        assert code == c["code"], c["name"]
        if code == 0:
            assert out.hex() == c["out"], c["name"]
    for c in golden["aggregate_pks"]:
        code, out = orc.aggregate_pks([_b(p) for p in c["pks"]])
        assert code == c["code"], c["name"]
        if code == 0:
            assert out.hex() == c["out"], c["name"]


def test_qc(golden):
    q = golden["qc"]
    pks = [_b(p) for p in q["pks"]]
    h = _b(q["hash"])
    agg = _b(q["agg_sig"])
    assert orc.aggregate_sigs([_b(s) for s in q["sigs"]], pks[:67]) == (0, agg)
    assert orc.aggregate_pks(pks[:67]) == (0, _b(q["agg_pk"]))
    assert orc.verify_aggregated(agg, h, pks[:67]) == q["verify_ok"]
    assert orc.verify_aggregated(agg, h, pks[:66]) == q["verify_missing_one"]
    assert orc.verify_aggregated(agg, h, []) == q["verify_empty"]
    assert orc.verify_aggregated(agg, h[:31], pks[:67]) == q["verify_hash_31"]
    assert orc.verify_aggregated(agg, h, pks[:66] + [pks[0][:40]]) == q["verify_bad_pk"]


def test_random_vs_python_oracle():
    rng = random.Random(1234)
    for _ in range(3):
        sk = rng.randrange(1, bls.R)
        msg = bytes(rng.randrange(256) for _ in range(32))
        skb = sk.to_bytes(32, "big")
        _, want = ov.sign(sk, msg)
        assert orc.sign(skb, msg) == (0, want)
        pk = bls.g1_compress(bls.sk_to_pk(sk))
        assert orc.sk_to_pk(skb) == (0, pk)
        assert orc.verify(want, msg, pk) == 0
        bad = bytes(rng.randrange(256) for _ in range(32))
        assert orc.verify(want, bad, pk) == ov.verify_signature(want, bad, pk) == 5


@pytest.mark.parametrize("threads", [1, 4])
def test_batch_rlc_matches_per_vote(golden, threads):
    cases = [c for c in golden["verify"] if len(_b(c["sig"])) == 96 and len(_b(c["hash"])) == 32
             and len(_b(c["pk"])) == 48]
    sigs = np.array([list(_b(c["sig"])) for c in cases], dtype=np.uint8)
    hs = np.array([list(_b(c["hash"])) for c in cases], dtype=np.uint8)
    pks = np.array([list(_b(c["pk"])) for c in cases], dtype=np.uint8)
    want = [c["code"] for c in cases]
    assert list(orc.verify_many(sigs, hs, pks, threads)) == want
    codes, ok = orc.verify_batch_rlc(sigs, hs, pks, seed=5, threads=threads)
    assert list(codes) == want and not ok
    good = [i for i, c in enumerate(cases) if c["code"] == 0]
    codes, ok = orc.verify_batch_rlc(sigs[good], hs[good], pks[good], seed=6, threads=threads)
    assert ok and (codes == 0).all()


def test_mulx_product_matches_portable_cios():
    """the oracle's Montgomery product runs as BMI2 mulx + ADX adcx / adox asm
    (oracle/c/mont_mulx.h, tools/gen_mulx.py) when the CPU has them -- only to make the timed CPU
    baseline closer to what blst would do. It must agree with the portable u128 CIOS bit for bit:
    200,000 random canonical operand pairs plus the edge values 0, 1, p - 1, and (the golden
    tests above) every verdict and byte the oracle produces."""
    assert orc.load().orc_mulx_selftest(0xC17A, 200000) == 0
