"""Validator keys on the Fp-VM (k_vm_pkchk: decompression + G1 subgroup check, a g1padd tree
for an aggregated key, the workgroup-parallel QC key sums) against the C oracle: every
48-byte golden key in the table and as a one-key aggregate, and verify_aggregated_signature /
aggregate_public_keys over sizes 1 .. 300 with repeated keys and a key next to its negation."""
import ctypes
import json
import os

import pytest

import synth_votes as sv

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def golden():
    with open(os.path.join(ROOT, "tests", "golden", "golden_v1.json")) as fh:
        return json.load(fh)


def test_verify_aggregated_key_tree_matches_oracle(golden):
    import consensus_overlord_amd as coa
    import orc
    c = coa.ConsensusCrypto(bytes.fromhex("3c" * 32))
    sigs, hs, pks = sv.make(c.ctx, 300, lo=50000)
    sigs, pks = [bytes(s) for s in sigs], [bytes(p) for p in pks]
    h = bytes(hs[0])
    neg = sv.bls.g1_compress(sv.bls.pt_neg(sv.bls.FpOps, sv.bls.g1_from_bytes(pks[3])))
    cases = []
    for n in (1, 2, 3, 67, 100, 129, 300):
        agg = orc.aggregate_sigs(sigs[:n], pks[:n])[1]
        cases.append((agg, h, pks[:n]))
    # every signer signed its own digest: only the one-signer QC over hs[0] verifies; the others
    # must fail exactly as the oracle says, whatever the key sum
    cases.append((sigs[0], h, pks[:1] + pks[:1]))
    cases.append((sigs[0], h, pks[:40] + pks[:40] + [pks[0]]))
    cases.append((sigs[0], h, pks[:5] + [neg] + pks[5:9]))
    for x in golden["verify"]:
        if len(x["pk"]) == 96:
            cases.append((sigs[0], h, [bytes.fromhex(x["pk"])]))
            cases.append((sigs[0], h, pks[:3] + [bytes.fromhex(x["pk"])]))
    for agg, hh, voters in cases:
        want = orc.verify_aggregated(agg, hh, voters)
        got = c.lib.ovh_verify_aggregated(c.ctx.ptr, agg, 96, hh, 32, b"".join(voters),
                                          (ctypes.c_size_t * len(voters))(*[len(v) for v in voters]), len(voters))
        assert got == want, (len(voters), got, want)
    assert c.lib.ovh_verify_aggregated(c.ctx.ptr, sigs[0], 96, h, 32, pks[0], (ctypes.c_size_t * 1)(48), 1) == 0


def test_validator_table_golden_keys(golden):
    """update_pubkeys with all 48-byte golden keys (+ 100 valid ones) -> QC batch codes equal the
    oracle's verify_aggregated for single-key and mixed QCs."""
    import consensus_overlord_amd as coa
    import orc
    c = coa.ConsensusCrypto(bytes.fromhex("3d" * 32))
    sigs, hs, pks = sv.make(c.ctx, 100, lo=51000)
    sigs, pks = [bytes(s) for s in sigs], [bytes(p) for p in pks]
    gk = sorted(set(bytes.fromhex(x["pk"]) for x in golden["verify"] if len(x["pk"]) == 96))
    table = pks + [k for k in gk if k not in pks]
    c.update_pubkeys(table)
    skeys = sorted(table)
    nb = (len(table) + 7) // 8

    def bm(voters):
        b = bytearray(nb)
        for v in voters:
            i = skeys.index(v)
            b[i // 8] |= 0x80 >> (i % 8)
        return bytes(b)
    qcs = [(sigs[0], bytes(hs[0]), [pks[0]]), (sigs[0], bytes(hs[0]), pks[:67]), (sigs[1], bytes(hs[1]), [pks[1]])]
    qcs += [(sigs[0], bytes(hs[0]), [k]) for k in gk] + [(sigs[0], bytes(hs[0]), [pks[0], k]) for k in gk]
    got = c.verify_qc_batch([q[0] for q in qcs], [q[1] for q in qcs], [bm(q[2]) for q in qcs])
    want = [orc.verify_aggregated(s, hh, v) for s, hh, v in qcs]
    assert got.tolist() == want
    assert want[0] == 0 and want[2] == 0


def test_aggregate_pks_vm_matches_oracle(golden):
    """BlsPublicKey::aggregate on the VM (pkchk + g1padd tree + compression): sizes 1 .. 300,
    repeated keys, a key and its negation, every 48-byte golden key case (infinity, outside G1,
    unparseable -> 102) alone and inside a list, against the C oracle (bytes and codes)."""
    import consensus_overlord_amd as coa
    import orc
    c = coa.ConsensusCrypto(bytes.fromhex("3d" * 32))
    _, _, pks = sv.make(c.ctx, 300, lo=60000)
    pks = [bytes(p) for p in pks]
    neg = sv.bls.g1_compress(sv.bls.pt_neg(sv.bls.FpOps, sv.bls.g1_from_bytes(pks[3])))
    lists = [pks[:n] for n in (1, 2, 3, 67, 100, 129, 300)]
    lists += [pks[:1] + pks[:1], pks[:40] + pks[:40], pks[:5] + [neg] + pks[3:4]]
    for x in golden["verify"]:
        if len(x["pk"]) == 96:
            lists.append([bytes.fromhex(x["pk"])])
            lists.append(pks[:3] + [bytes.fromhex(x["pk"])] + pks[3:5])
    for voters in lists:
        code, want = orc.aggregate_pks(voters)
        out = ctypes.create_string_buffer(48)
        got = c.lib.ovh_aggregate_pks(c.ctx.ptr, b"".join(voters),
                                      (ctypes.c_size_t * len(voters))(*[len(v) for v in voters]), len(voters), out)
        assert got == code, (len(voters), got, code)
        if code == 0:
            assert out.raw == want, len(voters)


def _order11_point():
    """A point of order 11 on E(Fp) (11 divides the G1 cofactor (x - 1)^2 / 3): outside G1, and
    its x is not 0 (the order-3 points (0, +-2) do not parse, DESIGN.md assumption 5)."""
    import bls12_381 as bls
    h1 = (bls.X - 1) ** 2 // 3
    assert h1 % 121 == 0   # the 11-part of E(Fp) has exponent 11: [h1 / 121 r] P has order 1 or 11
    x = 5
    while True:
        y = bls.fp_sqrt((x ** 3 + 4) % bls.P)
        if y is not None:
            T = bls.pt_mul(bls.FpOps, (x, y), h1 // 121 * bls.R)
            if T is not None:
                assert bls.pt_mul(bls.FpOps, T, 11) is None
                return T
        x += 1


def test_aggregated_key_outside_g1_checked_on_the_sum():
    """verify_aggregated_signature checks the SUM of the keys (BlsPublicKey::aggregate does not
    group-check, blst's verify checks the aggregated key: consensus.rs:371,378-380): keys A + T
    and B - T (T of order 11, both outside G1) sum into G1 and verify; either alone, or with B,
    does not (POINT_NOT_IN_GROUP) -- on the VM (k_vm_g1grp), per call and in a QC batch, as the
    C oracle."""
    import bls12_381 as bls
    import orc
    import consensus_overlord_amd as coa
    F = bls.FpOps
    cc = coa.ConsensusCrypto(bytes.fromhex("4d" * 32))
    h = bytes.fromhex("5e" * 32)
    sa, sb = 0x1234567 * 0x9E3779B97F4A7C15 % bls.R, 0x7654321 * 0xC2B2AE3D27D4EB4F % bls.R
    A, B = bls.sk_to_pk(sa), bls.sk_to_pk(sb)
    T = _order11_point()
    K1 = bls.g1_compress(bls.pt_add(F, A, T))
    K2 = bls.g1_compress(bls.pt_add(F, B, bls.pt_neg(F, T)))
    Bc = bls.g1_compress(B)
    agg = orc.aggregate_sigs([orc.sign(sa.to_bytes(32, "big"), h)[1], orc.sign(sb.to_bytes(32, "big"), h)[1]],
                             [bls.g1_compress(A), Bc])[1]
    cases = [[K1, K2], [K1], [K1, Bc], [K2, K1]]
    want = [orc.verify_aggregated(agg, h, ks) for ks in cases]
    assert want == [0, 3, 3, 0]

    def vagg(ks):
        lens = (ctypes.c_size_t * len(ks))(*[48] * len(ks))
        return cc.lib.ovh_verify_aggregated(cc.ctx.ptr, agg, 96, h, 32, b"".join(ks), lens, len(ks))
    assert [vagg(ks) for ks in cases] == want
    # the same QCs through the validator table (ovh_verify_qc_batch)
    table = [K1, K2, Bc, bls.g1_compress(A)]
    cc.update_pubkeys(table)
    skeys = sorted(table)
    bms = []
    for ks in cases:
        bm = bytearray(1)
        for k in ks:
            i = skeys.index(k)
            bm[0] |= 0x80 >> i
        bms.append(bytes(bm))
    got = cc.verify_qc_batch([agg] * len(cases), [h] * len(cases), bms)
    assert got.tolist() == want
