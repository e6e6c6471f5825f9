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
