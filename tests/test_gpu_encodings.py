"""GPU parity of ovh_verify on encodings other than compressed 96 / 48 bytes (ovhip.hip
k_canon_one: uncompressed points, other lengths, flag errors, re-encoded into one compressed
vote for the vote1 + final1 path; consensus.rs:406-410 with blst's from_bytes semantics, a [dep]
assumption). Every case's code == the C oracle's, on golden votes turned
into uncompressed encodings and corrupted field by field."""
import pytest

pytestmark = pytest.mark.gpu

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB


@pytest.fixture(scope="module")
def cc():
    import consensus_overlord_amd as coa
    return coa.ConsensusCrypto(bytes.fromhex("12" * 32))


def _b(h):
    return bytes.fromhex(h)


def _cases(golden):
    import bls12_381 as bls
    v, k = golden["votes"], golden["keys"]
    named = {c["name"]: c for c in golden["verify"]}
    out = []
    for j in range(3):
        h = _b(v[j]["digest"])
        sig_c, pk_c = _b(v[j]["sig"]), _b(k[j]["pk"])
        sig_u = bls.g2_serialize(bls.g2_from_bytes(sig_c))
        pk_u = bls.g1_serialize(bls.g1_from_bytes(pk_c))
        other_u = bls.g2_serialize(bls.g2_from_bytes(_b(v[(j + 1) % len(v)]["sig"])))
        out += [("u_sig", sig_u, h, pk_c), ("u_pk", sig_c, h, pk_u), ("u_both", sig_u, h, pk_u),
                ("u_wrong_sig", other_u, h, pk_u)]
    h, sig_c, pk_c = _b(v[0]["digest"]), _b(v[0]["sig"]), _b(k[0]["pk"])
    sig_u = bytearray(bls.g2_serialize(bls.g2_from_bytes(sig_c)))
    pk_u = bytearray(bls.g1_serialize(bls.g1_from_bytes(pk_c)))

    def mod(buf, pos, val):
        b = bytearray(buf)
        b[pos] = val
        return bytes(b)
    out += [
        ("u_sig_off_curve", mod(sig_u, 191, sig_u[191] ^ 1), h, pk_c),
        ("u_sig_sortflag", mod(sig_u, 0, sig_u[0] | 0x20), h, pk_c),
        ("u_sig_compflag", mod(sig_u, 0, sig_u[0] | 0x80), h, pk_c),
        ("u_sig_inf", bytes([0x40]) + bytes(191), h, pk_c),
        ("u_sig_inf_dirty", bytes([0x40]) + bytes(190) + b"\x01", h, pk_c),
        ("u_sig_y_ge_p", bytes(sig_u[:96]) + P.to_bytes(48, "big") + bytes(sig_u[144:]), h, pk_c),
        ("u_sig_x_ge_p", bytes(sig_u[:48]) + P.to_bytes(48, "big") + bytes(sig_u[96:]), h, pk_c),
        ("u_pk_off_curve", sig_c, h, mod(pk_u, 95, pk_u[95] ^ 1)),
        ("u_pk_inf", sig_c, h, bytes([0x40]) + bytes(95)),
        ("u_pk_y_ge_p", sig_c, h, bytes(pk_u[:48]) + P.to_bytes(48, "big")),
        ("u_pk_bad_and_sig_bad", bytes(sig_u[:100]), h, bytes(pk_u[:50])),
        ("len_0_0", b"", h, b""),
        ("sig_191", bytes(sig_u[:191]), h, pk_c),
        ("sig_193", bytes(sig_u) + b"\x00", h, pk_c),
        ("pk_97", sig_c, h, bytes(pk_u) + b"\x00"),
    ]
    nig = bls._g2_uncompress(_b(named["sig_not_in_g2"]["sig"]))
    out.append(("u_sig_not_in_g2", bls.g2_serialize(nig), _b(named["sig_not_in_g2"]["hash"]),
                _b(named["sig_not_in_g2"]["pk"])))
    nig1 = bls._g1_uncompress(_b(named["pk_not_in_g1"]["pk"]))
    out.append(("u_pk_not_in_g1", _b(named["pk_not_in_g1"]["sig"]), _b(named["pk_not_in_g1"]["hash"]),
                bls.g1_serialize(nig1)))
    # every golden case whose encodings are not compressed 96 / 48 (uncompressed, other lengths)
    out += [(c["name"], _b(c["sig"]), _b(c["hash"]), _b(c["pk"])) for c in golden["verify"]
            if len(_b(c["hash"])) == 32 and (len(_b(c["sig"])) != 96 or len(_b(c["pk"])) != 48)]
    return out


def test_other_encodings_match_oracle(cc, golden):
    import orc
    cases = _cases(golden)
    want_codes = set()
    for name, sig, h, pk in cases:
        want = orc.verify(sig, h, pk)
        got = cc.lib.ovh_verify(cc.ctx.ptr, sig, len(sig), h, len(h), pk, len(pk))
        assert got == want, (name, got, want)
        want_codes.add(want)
    # the set covers success, a failed pairing, parse / curve / group failures and the key error
    assert {0, 1, 2, 3, 5, 102} <= want_codes, want_codes


def test_other_encodings_golden_codes(cc, golden):
    """The golden file's own codes for its uncompressed / odd-length cases."""
    for c in golden["verify"]:
        sig, h, pk = _b(c["sig"]), _b(c["hash"]), _b(c["pk"])
        if len(h) != 32 or (len(sig) == 96 and len(pk) == 48):
            continue
        assert cc.lib.ovh_verify(cc.ctx.ptr, sig, len(sig), h, len(h), pk, len(pk)) == c["code"], c["name"]


def _agg(cc, sigs, pks):
    import ctypes
    import orc
    sd, sl = orc._lens(sigs)
    pd, pl = orc._lens(pks)
    out = ctypes.create_string_buffer(96)
    c = cc.lib.ovh_aggregate_sigs(cc.ctx.ptr, sd, sl, len(sigs), pd, pl, len(pks), out)
    return c, (out.raw if c == 0 else None)


def _vagg(cc, agg, h, pks):
    import orc
    pd, pl = orc._lens(pks)
    return cc.lib.ovh_verify_aggregated(cc.ctx.ptr, agg, len(agg), h, len(h), pd, pl, len(pks))


def test_aggregate_and_qc_other_encodings(cc, golden):
    """aggregate_signatures over lists mixing compressed and uncompressed signatures (and keys),
    with an off-curve, a bad-length and a non-subgroup item; verify_aggregated_signature with an
    uncompressed aggregate and uncompressed / odd keys (k_canon_sig_list, k_canon_qc): codes and
    bytes == the C oracle's."""
    import bls12_381 as bls
    import orc
    q = golden["qc"]
    pks = [_b(p) for p in q["pks"][:67]]
    sigs = [_b(s) for s in q["sigs"][:67]]
    h = _b(q["hash"])
    su = [bls.g2_serialize(bls.g2_from_bytes(s)) if i % 3 == 0 else s for i, s in enumerate(sigs)]
    pu = [bls.g1_serialize(bls.g1_from_bytes(p)) if i % 4 == 1 else p for i, p in enumerate(pks)]
    named = {c["name"]: c for c in golden["verify"]}
    nig = bls.g2_serialize(bls._g2_uncompress(_b(named["sig_not_in_g2"]["sig"])))
    off = bytearray(su[0])
    off[191] ^= 1
    lists = [(su, pks), (su, pu), (sigs, pu), (su[:5] + [bytes(off)] + su[6:], pks), (su[:6] + [su[6][:100]] + su[7:], pks),
             (su[:9] + [nig] + su[10:], pks), ([su[0]], [pu[1]])]
    for s_, p_ in lists:
        want = orc.aggregate_sigs(s_, p_)
        assert _agg(cc, s_, p_) == want, want[0]
    agg = _b(q["agg_sig"])
    agg_u = bls.g2_serialize(bls.g2_from_bytes(agg))
    bad_u = bytearray(agg_u)
    bad_u[191] ^= 1
    cases = [(agg_u, h, pks), (agg_u, h, pu), (agg, h, pu), (agg_u, h, pu[:66]), (agg_u, _b("00" * 32), pu),
             (bytes(bad_u), h, pu), (agg_u[:150], h, pu), (agg_u, h, pu[:66] + [pu[1][:60]]),
             (agg_u, h, pu[:66] + [bls.g1_serialize(None)])]
    for a, hh, p_ in cases:
        assert _vagg(cc, a, hh, p_) == orc.verify_aggregated(a, hh, p_), (len(a), len(p_))
