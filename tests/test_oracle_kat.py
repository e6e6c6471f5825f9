"""Pin the CPU oracle against published known-answer values.

The reference's own tests hold no crypto vectors (src/config.rs:58-72 is its only test),
so the oracle is pinned by published standards instead:
  * RFC 9380 Appendix K.1 expand_message_xmd(SHA-256) vectors,
  * RFC 9380 Appendix J.10.1 BLS12381G2_XMD:SHA-256_SSWU_RO_ hash_to_curve vectors,
  * GB/T 32905-2016 SM3 vectors,
  * the BLS12-381 generators (ZCash compressed encodings) and group orders.
"""
import random

import bls12_381 as bls
import overlord_oracle as ov

F1, F2 = bls.FpOps, bls.Fp2Ops

RFC9380_G2_DST = b"QUUX-V01-CS02-with-BLS12381G2_XMD:SHA-256_SSWU_RO_"
RFC9380_G2_RO = {
    b"": (
        0x0141EBFBDCA40EB85B87142E130AB689C673CF60F1A3E98D69335266F30D9B8D4AC44C1038E9DCDD5393FAF5C41FB78A,
        0x05CB8437535E20ECFFAEF7752BADDF98034139C38452458BAEEFAB379BA13DFF5BF5DD71B72418717047F5B0F37DA03D,
        0x0503921D7F6A12805E72940B963C0CF3471C7B2A524950CA195D11062EE75EC076DAF2D4BC358C4B190C0C98064FDD92,
        0x12424AC32561493F3FE3C260708A12B7C620E7BE00099A974E259DDC7D1F6395C3C811CDD19F1E8DBF3E9ECFDCBAB8D6,
    ),
    b"abc": (
        0x02C2D18E033B960562AAE3CAB37A27CE00D80CCD5BA4B7FE0E7A210245129DBEC7780CCC7954725F4168AFF2787776E6,
        0x139CDDBCCDC5E91B9623EFD38C49F81A6F83F175E80B06FC374DE9EB4B41DFE4CA3A230ED250FBE3A2ACF73A41177FD8,
        0x1787327B68159716A37440985269CF584BCB1E621D3A7202BE6EA05C4CFE244AEB197642555A0645FB87BF7466B2BA48,
        0x00AA65DAE3C8D732D10ECD2C50F8A1BAF3001578F71C694E03866E9F3D49AC1E1CE70DD94A733534F106D4CEC0EDDD16,
    ),
}


def test_generators():
    assert bls.on_curve(F1, bls.G1_GEN) and bls.on_curve(F2, bls.G2_GEN)
    assert bls.pt_mul(F1, bls.G1_GEN, bls.R) is None
    assert bls.pt_mul(F2, bls.G2_GEN, bls.R) is None
    assert bls.g1_compress(bls.G1_GEN).hex() == (
        "97f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb")
    assert bls.g2_compress(bls.G2_GEN).hex().startswith("93e02b6052719f607dacd3a088274f65")
    assert (bls.X - 1) ** 2 * bls.R // 3 + bls.X == bls.P
    assert bls.X ** 4 - bls.X ** 2 + 1 == bls.R


def test_sm3_kat():
    assert ov.sm3(b"abc").hex() == "66c7f0f462eeedd9d1f2d46bdc10e4e24167c4875cf2f7a2297da02b8f4ba8e0"
    assert ov.sm3(b"abcd" * 16).hex() == "debe9ff92275b8a138604889c18e5a4d6fdb70e5387e5765293dcba39c0c5732"


def test_expand_message_xmd_kat():
    dst = b"QUUX-V01-CS02-with-expander-SHA256-128"
    assert bls.expand_message_xmd(b"", dst, 0x20).hex() == "68a985b87eb6b46952128911f2a4412bbc302a9d759667f87f7a21d803f07235"
    assert bls.expand_message_xmd(b"abc", dst, 0x20).hex() == "d8ccab23b5985ccea865c6c97b6e5b8350e794e603b4b97902f53a8a0d605615"


def test_hash_to_g2_rfc9380():
    for msg, (x0, x1, y0, y1) in RFC9380_G2_RO.items():
        H = bls.hash_to_g2(msg, RFC9380_G2_DST)
        assert H == ((x0, x1), (y0, y1))


def test_iso_map_and_cofactor():
    rng = random.Random(5)
    for _ in range(3):
        while True:
            x = (rng.randrange(bls.P), rng.randrange(bls.P))
            g = bls.f2_add(bls.f2_add(bls.f2_mul(bls.f2_sqr(x), x), bls.f2_mul(bls.SSWU_A, x)), bls.SSWU_B)
            y = bls.f2_sqrt(g)
            if y is not None:
                break
        q = bls.iso_map_g2((x, y))
        assert bls.on_curve(F2, q)
        assert bls.pt_eq(F2, bls.clear_cofactor_g2(q), bls.clear_cofactor_g2_psi(q))


def test_pairing_bilinear_and_fast_paths():
    rng = random.Random(9)
    a, b = rng.randrange(1, bls.R), rng.randrange(1, bls.R)
    Pa = bls.pt_mul(F1, bls.G1_GEN, a)
    Qb = bls.pt_mul(F2, bls.G2_GEN, b)
    e = bls.pairing(bls.G1_GEN, bls.G2_GEN)
    assert not bls.f12_is_one(e)
    assert bls.f12_is_one(bls.f12_pow(e, bls.R))
    eab = bls.pairing(Pa, Qb)
    assert bls.f12_eq(eab, bls.f12_pow(e, a * b % bls.R))
    fp = bls.miller_loop_proj(Pa, Qb)
    assert bls.f12_eq(bls.final_exponentiation(fp), eab)
    e3 = bls.final_exponentiation_x_chain(bls.miller_loop(Pa, Qb))
    assert bls.f12_eq(e3, bls.f12_mul(bls.f12_sqr(eab), eab))


def test_fast_subgroup_checks_match_naive():
    rng = random.Random(11)
    for _ in range(3):
        while True:
            x = rng.randrange(bls.P)
            y = bls.fp_sqrt(x ** 3 + 4)
            if y is not None:
                break
        p1 = (x, y)
        assert bls.g1_in_subgroup_fast(p1) == bls.g1_in_subgroup(p1)
        cleared = bls.pt_mul(F1, p1, (bls.X - 1) ** 2 // 3)
        assert bls.g1_in_subgroup_fast(cleared) and bls.g1_in_subgroup(cleared)
        while True:
            x2 = (rng.randrange(bls.P), rng.randrange(bls.P))
            y2 = bls.f2_sqrt(bls.f2_add(bls.f2_mul(bls.f2_sqr(x2), x2), bls.B2))
            if y2 is not None:
                break
        q = (x2, y2)
        assert bls.g2_in_subgroup_fast(q) == bls.g2_in_subgroup(q)
        assert bls.g2_in_subgroup_fast(bls.clear_cofactor_g2(q))


def test_vote_rlp_fixture():
    # SURVEY.md Appendix B illustrative fixture (overlord 0.4 Vote RLP, [dep])
    rlp = ov.rlp_vote(1, 0, ov.PRECOMMIT, ov.sm3(b""))
    assert rlp.hex() == "e4018001a01ab21d8355cfa17f8e61194831e81a8f22bec8c728fefb747ed035eb5082aa2b"
    assert ov.sm3(rlp).hex() == "b879a90276edf81f09f6f5577740dd6e9d4a6ce799f7cedd2a7c46bd1e231325"


def test_sign_verify_roundtrip_and_golden(golden):
    # the committed fixtures are reproducible from the oracle
    k = golden["keys"][0]
    v = golden["votes"][0]
    sk = int(k["sk"], 16)
    assert bls.g1_compress(bls.sk_to_pk(sk)).hex() == k["pk"]
    code, sig = ov.sign(sk, bytes.fromhex(v["digest"]))
    assert code == 0 and sig.hex() == v["sig"]
    assert ov.verify_signature(sig, bytes.fromhex(v["digest"]), bytes.fromhex(k["pk"])) == 0
    h = golden["hash_to_g2"][0]
    assert bls.g2_serialize(bls.hash_to_g2(bytes.fromhex(h["msg"]))).hex() == h["point"]


def test_golden_verify_codes(golden):
    for c in golden["verify"][:12]:
        code = ov.verify_signature(bytes.fromhex(c["sig"]), bytes.fromhex(c["hash"]), bytes.fromhex(c["pk"]))
        assert code == c["code"], c["name"]


# ---- private-key parse: IETF KeyGen (ophelia-blst BlsPrivateKey::try_from [dep]) ----
def test_hkdf_sha256_rfc5869_case1():
    """RFC 5869 Appendix A.1 (the HKDF under KeyGen)."""
    prk = bls.hkdf_extract(bytes(range(13)), b"\x0b" * 22)
    assert prk.hex() == "077709362c2e32df0ddc3f0dc47bba6390b6c73bb50f9c3122ec844ad7c2b3e5"
    okm = bls.hkdf_expand(prk, bytes(range(0xF0, 0xFA)), 42)
    assert okm.hex() == ("3cb25f25faacd57a90434f64d0362f2a2d2d0a90cf1a5a4c5db02d56ecc4c5bf"
                         "34007208d5b887185865")


def test_keygen_eip2333_master_key():
    """EIP-2333 test case 0: derive_master_SK(seed) = HKDF_mod_r(seed) = KeyGen(seed, "")."""
    seed = bytes.fromhex("c55257c360c07c72029aebc1b53c05ed0362ada38ead3e3e9efa3708e53495531f09a6987599d182"
                         "64c1e1c92f2cf141630c7a3c4ab7c81b2f001698e7463b04")
    assert bls.sk_keygen(seed) == 6083874454709270928345386274498605044986640685124978867557563392430687146096
    import orc
    assert orc.sk_keygen(seed) == (0, bls.sk_keygen(seed).to_bytes(32, "big"))


def test_example_private_key_fixture():
    """The reference's example/private_key (>= r) parses by KeyGen; the fixture's name and
    signatures follow from the oracle (tests/golden/make_example_key.py)."""
    import json
    import os
    import orc
    with open(os.path.join(os.path.dirname(__file__), "golden", "example_key.json")) as fh:
        ex = json.load(fh)
    key = bytes.fromhex(ex["key_hex"])
    assert int.from_bytes(key, "big") >= bls.R
    sk = bls.sk_keygen(key)
    assert "%064x" % sk == ex["scalar"]
    assert orc.sk_keygen(key) == (0, bytes.fromhex(ex["scalar"]))
    assert bls.g1_compress(bls.sk_to_pk(sk)).hex() == ex["name"]
    assert orc.sk_to_pk(sk.to_bytes(32, "big")) == (0, bytes.fromhex(ex["name"]))
    for s in ex["signatures"]:
        assert orc.sign(sk.to_bytes(32, "big"), bytes.fromhex(s["digest"])) == (0, bytes.fromhex(s["sig"]))
    try:
        bls.sk_from_bytes(key)
        raise AssertionError("strict parse accepted a key >= r")
    except bls.BlstError as e:
        assert e.code == ex["raw_parse_code"]
    assert orc.sk_keygen(key[:31])[0] == 1     # KeyGen needs >= 32 bytes of key material
