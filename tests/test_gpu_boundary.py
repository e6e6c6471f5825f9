"""The drop-in boundary on the GPU (include/ovhip.h): thread safety of one context, the
vote-batching verdict cache (ovh_prefetch -> ovh_verify), the device validator table
(ovh_set_validators -> vote_t path) and batched QC verification (ovh_verify_qc_batch), each
checked against the oracle / golden codes."""
import json
import os
import threading

import numpy as np
import pytest

import synth_votes as sv

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def golden():
    with open(os.path.join(ROOT, "tests", "golden", "golden_v1.json")) as fh:
        return json.load(fh)


def _fixed(golden):
    return [c for c in golden["verify"] if len(c["sig"]) == 192 and len(c["hash"]) == 64 and len(c["pk"]) == 96]


def _b(h):
    return bytes.fromhex(h)


def test_two_threads_one_context(golden):
    """overlord's serial verify_signature and a gRPC-side batch on the same context at once
    (main.rs:107-127): every call returns its exact codes."""
    import consensus_overlord_amd as coa
    c = coa.ConsensusCrypto(bytes.fromhex("55" * 32))
    cases = _fixed(golden)
    n = 512
    sigs, hs, pks = sv.make(c.ctx, n, lo=90000)
    for k, i in enumerate(range(0, n, 97)):
        sigs[i] = np.frombuffer(sv.add_g2(bytes(sigs[i])), dtype=np.uint8)
    want = sv.oracle_codes(sigs, hs, pks)
    errors = []

    def serial():
        try:
            for _ in range(2):
                for cs in cases:
                    got = c.lib.ovh_verify(c.ctx.ptr, _b(cs["sig"]), 96, _b(cs["hash"]), 32, _b(cs["pk"]), 48)
                    if got != cs["code"]:
                        errors.append(("verify", cs["name"], got))
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    def batch():
        try:
            for _ in range(3):
                got = c.verify_batch(list(map(bytes, sigs)), list(map(bytes, hs)), list(map(bytes, pks)))
                if got.tolist() != want.tolist():
                    errors.append(("batch", got))
        except Exception as e:  # noqa: BLE001
            errors.append(e)
    th = [threading.Thread(target=serial), threading.Thread(target=batch)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errors, errors[:3]


def test_prefetch_then_serial_verify_hits_cache(golden):
    import consensus_overlord_amd as coa
    from consensus_overlord_amd.crypto import CryptoErr, Other
    c = coa.ConsensusCrypto(bytes.fromhex("66" * 32))
    cases = _fixed(golden)
    sigs, hs, pks = [_b(x["sig"]) for x in cases], [_b(x["hash"]) for x in cases], [_b(x["pk"]) for x in cases]
    c.prefetch(sigs, hs, pks)
    h0, m0, e0 = c.cache_stats()
    assert e0 == len(set(zip(sigs, hs, pks)))
    for cs, s, h, p in zip(cases, sigs, hs, pks):
        try:
            c.verify_signature(s, h, p)
            got = 0
        except CryptoErr as e:
            got = e.code
        except Other as e:
            got = {"lose public key": 102}[str(e)]
        assert got == cs["code"], cs["name"]
    h1, m1, _ = c.cache_stats()
    assert h1 - h0 == len(cases) and m1 == m0
    # a triple not prefetched is a miss and still exact
    import orc
    v = [x for x in cases if x["name"].startswith("valid_")]
    s2, h3, p4 = _b(v[2]["sig"]), _b(v[3]["hash"]), _b(v[4]["pk"])
    assert (s2, h3, p4) not in set(zip(sigs, hs, pks))
    assert c.lib.ovh_verify(c.ctx.ptr, s2, 96, h3, 32, p4, 48) == orc.verify(s2, h3, p4) == 5
    assert c.cache_stats()[1] == m1 + 1


def test_validator_table_path_matches_golden(golden):
    """update_pubkeys with every fixed-size golden key (including keys that do not parse, the
    infinity key and a non-G1 key): verify_batch then runs the table (vote_t) path."""
    import consensus_overlord_amd as coa
    c = coa.ConsensusCrypto(bytes.fromhex("77" * 32))
    cases = _fixed(golden)
    keys = sorted(set(_b(x["pk"]) for x in cases))
    c.update_pubkeys(keys)
    got = c.verify_batch([_b(x["sig"]) for x in cases], [_b(x["hash"]) for x in cases], [_b(x["pk"]) for x in cases])
    for cs, g in zip(cases, got):
        assert g == cs["code"], cs["name"]
    # per call through the table too
    for cs in cases[:12]:
        assert c.lib.ovh_verify(c.ctx.ptr, _b(cs["sig"]), 96, _b(cs["hash"]), 32, _b(cs["pk"]), 48) == cs["code"]


def _bitmap(sorted_keys, voters, nbytes):
    bm = bytearray(nbytes)
    pos = {k: i for i, k in enumerate(sorted_keys)}
    for v in voters:
        i = pos[v]
        bm[i // 8] |= 0x80 >> (i % 8)
    return bytes(bm)


def test_qc_batch_matches_verify_aggregated(golden):
    """check_block's QC check (consensus.rs:143-207) batched over QCs: voters from the bitmap
    over the key-sorted validator table (extract_voters)."""
    import consensus_overlord_amd as coa
    import orc
    c = coa.ConsensusCrypto(bytes.fromhex("88" * 32))
    q = golden["qc"]
    pks = [_b(p) for p in q["pks"]]
    bad_parse = _b([x for x in golden["verify"] if x["name"] == "pk_x_eq_p"][0]["pk"])
    not_g1 = _b([x for x in golden["verify"] if x["name"] == "pk_not_in_g1"][0]["pk"])
    table = pks + [bad_parse, not_g1]
    c.update_pubkeys(table)
    skeys = sorted(table)
    nb = (len(table) + 7) // 8
    agg, h = _b(q["agg_sig"]), _b(q["hash"])
    qcs = [
        (agg, h, pks[:67]),                 # valid QC (config 2)
        (agg, h, pks[:66]),                 # one signer missing
        (agg, bytes(32), pks[:67]),         # wrong vote hash
        (agg, h, []),                       # empty bitmap -> AGGR_TYPE_MISMATCH
        (agg, h, pks[:67] + [bad_parse]),   # a voter key that does not parse -> 102
        (agg, h, pks[:66] + [not_g1]),      # a voter key outside G1 (exact single-QC path)
        (_b(q["sigs"][0]), h, [pks[0]]),    # single-signer QC
    ]
    sigs = [x[0] for x in qcs]
    hashes = [x[1] for x in qcs]
    bitmaps = [_bitmap(skeys, x[2], nb) for x in qcs]
    got = c.verify_qc_batch(sigs, hashes, bitmaps)
    want = [orc.verify_aggregated(s, hh, list(v)) for s, hh, v in qcs]
    assert got.tolist() == want
    assert want[:4] == [0, 5, 5, 4] and want[4] == 102 and want[6] == 0


def test_table_split_mixed_batch(golden):
    """A batch whose voters are partly in the validator table: the table votes run vote_t, the
    rest the vote program (two combined checks), and every code still equals the oracle's --
    unknown voters, invalid signatures and keys that do not parse included; the same through a
    two-device context, whose shards split the same way."""
    import consensus_overlord_amd as coa
    from consensus_overlord_amd.crypto import Context
    c = coa.ConsensusCrypto(bytes.fromhex("99" * 32))
    n = 300
    sigs, hs, pks = sv.make(c.ctx, n, lo=70000)
    for i in range(0, n, 37):
        sigs[i] = np.frombuffer(sv.add_g2(bytes(sigs[i])), dtype=np.uint8)
    bad_parse = _b([x for x in golden["verify"] if x["name"] == "pk_x_eq_p"][0]["pk"])
    pks[5] = np.frombuffer(bad_parse, dtype=np.uint8)     # in the table, does not parse
    pks[6] = np.frombuffer(bad_parse, dtype=np.uint8)
    table = [bytes(pks[i]) for i in range(0, n, 2)] + [bad_parse]
    c.update_pubkeys(table)
    want = sv.oracle_codes(sigs, hs, pks)
    args = (list(map(bytes, sigs)), list(map(bytes, hs)), list(map(bytes, pks)))
    assert c.verify_batch(*args).tolist() == want.tolist()
    multi = coa.ConsensusCrypto(bytes.fromhex("99" * 32), ctx=Context(devices=[0, 0]))
    multi.update_pubkeys(table)
    assert multi.verify_batch(*args).tolist() == want.tolist()
    # per call: a table voter and an unknown voter
    for i in (1, 2, 37, 74):
        assert c.lib.ovh_verify(c.ctx.ptr, bytes(sigs[i]), 96, bytes(hs[i]), 32, bytes(pks[i]), 48) == want[i]


def test_oversized_encodings_keep_reference_precedence(golden):
    """consensus.rs:403-414 order for encodings of any length: hash length, then the key parse
    (102), then the signature parse (BAD_ENCODING) -- also past the staging limit."""
    import consensus_overlord_amd as coa
    c = coa.ConsensusCrypto(bytes.fromhex("aa" * 32))
    v = [x for x in golden["verify"] if x["name"].startswith("valid_")][0]
    s, h, p = _b(v["sig"]), _b(v["hash"]), _b(v["pk"])
    big = bytes(5000)
    L = c.lib
    assert L.ovh_verify(c.ctx.ptr, s, 96, h, 32, p, 48) == 0
    assert L.ovh_verify(c.ctx.ptr, s, 96, h, 32, big, len(big)) == 102
    assert L.ovh_verify(c.ctx.ptr, big, len(big), h, 32, p, 48) == 1
    assert L.ovh_verify(c.ctx.ptr, big, len(big), h, 32, big, len(big)) == 102
    assert L.ovh_verify(c.ctx.ptr, big, len(big), h, 31, big, len(big)) == 100


def test_peer_matrix_of_contexts():
    """ovh_multi_peer_matrix: a one-device context is its own peer; a context over {0, 0} has
    every pair on one device (no host staging anywhere); with two GPUs visible, the matrix
    follows what the runtime reports for the pair."""
    from consensus_overlord_amd.crypto import Context
    c = Context()
    assert c.peer_matrix() == [[True]]
    m = Context(devices=[0, 0])
    assert m.peer_matrix() == [[True, True], [True, True]]
    import torch
    if torch.cuda.device_count() > 1:   # distinct devices: the matrix is what the runtime allows
        d = Context(devices=[0, 1])
        pm = d.peer_matrix()
        can = torch.cuda.can_device_access_peer(0, 1) and torch.cuda.can_device_access_peer(1, 0)
        assert pm[0][0] and pm[1][1] and pm[0][1] == torch.cuda.can_device_access_peer(0, 1)
        assert pm[1][0] == torch.cuda.can_device_access_peer(1, 0) or not can
