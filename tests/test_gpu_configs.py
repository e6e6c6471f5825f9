"""GPU parity at BASELINE.json's configuration sizes (SURVEY.md 8(d) synthetic votes), through
the C ABI, against the C oracle's per-vote verdicts (test infrastructure):

  config 3  4096 distinct-message precommit votes, RLC batch, with injected invalid votes
  config 5  1024 votes, 1% sigma + G2 at seeded positions: every one flagged by the bisection
  config 4  the multi-device split (ovh_create_multi over {0, 0} on the one-GPU box): shards,
            peer-copied partials, one combined check, per-device bisection
  soundness the cancellation pair built for a known seed: flagged under the library's
            getrandom seeds, accepted only with the test-only OVH_FLAG_TEST_RLC (same seed)."""
import json
import os

import numpy as np
import pytest

import synth_votes as sv

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def cc():
    import consensus_overlord_amd as coa
    return coa.ConsensusCrypto(bytes.fromhex("22" * 32))


@pytest.fixture(scope="module")
def golden_cases():
    with open(os.path.join(ROOT, "tests", "golden", "golden_v1.json")) as fh:
        g = json.load(fh)
    return [c for c in g["verify"] if len(c["sig"]) == 192 and len(c["hash"]) == 64 and len(c["pk"]) == 96]


def _inject(sigs, hs, pks, golden_cases, positions):
    """Overwrite votes at `positions` with the fixed-size golden negative cases (bad encodings,
    off-curve, non-subgroup, infinity, wrong message ...), cycling through them."""
    neg = [c for c in golden_cases if c["code"] != 0]
    for k, i in enumerate(positions):
        c = neg[k % len(neg)]
        sigs[i] = np.frombuffer(bytes.fromhex(c["sig"]), dtype=np.uint8)
        hs[i] = np.frombuffer(bytes.fromhex(c["hash"]), dtype=np.uint8)
        pks[i] = np.frombuffer(bytes.fromhex(c["pk"]), dtype=np.uint8)


def test_config3_4096_votes_exact_codes(cc, golden_cases):
    n = 4096
    sigs, hs, pks = sv.make(cc.ctx, n)
    codes = cc.verify_batch(list(map(bytes, sigs)), list(map(bytes, hs)), list(map(bytes, pks)))
    assert (codes == 0).all()
    # invalid votes of every kind at seeded positions, plus sigma + G2 and swapped digests
    bad = sv.seeded_positions(n, 0.01, 3)
    _inject(sigs, hs, pks, golden_cases, bad[: len(bad) // 2])
    for i in bad[len(bad) // 2:]:
        sigs[i] = np.frombuffer(sv.add_g2(bytes(sigs[i])), dtype=np.uint8)
    hs[[10, 20]] = hs[[20, 10]]
    want = sv.oracle_codes(sigs, hs, pks)
    got = cc.verify_batch(list(map(bytes, sigs)), list(map(bytes, hs)), list(map(bytes, pks)))
    assert got.tolist() == want.tolist()
    assert sorted(set(np.nonzero(want)[0].tolist())) == sorted(set(bad) | {10, 20})


def test_config5_1024_one_percent_flagged(cc):
    import torch
    from consensus_overlord_amd import device as dev
    n = 1024
    sigs, hs, pks = sv.make(cc.ctx, n, lo=50000)
    bad = sv.seeded_positions(n, 0.01, 5)
    for i in bad:
        sigs[i] = np.frombuffer(sv.add_g2(bytes(sigs[i])), dtype=np.uint8)
    d = [torch.from_numpy(x.copy()).cuda() for x in (sigs, hs, pks)]
    torch.cuda.synchronize()
    codes = dev.verify_batch(cc.ctx, *d).cpu().numpy()
    assert [i for i in range(n) if codes[i]] == bad
    assert all(codes[i] == 5 for i in bad)
    assert codes.tolist() == sv.oracle_codes(sigs, hs, pks).tolist()


def test_config4_multi_device_split(golden_cases):
    """ovh_create_multi({0, 0}): two shards of 1024 with invalid votes in both."""
    import consensus_overlord_amd as coa
    from consensus_overlord_amd.crypto import Context
    ctx = Context(devices=[0, 0])
    assert ctx.device_count == 2
    c = coa.ConsensusCrypto(bytes.fromhex("33" * 32), ctx=ctx)
    n = 2048
    one = coa.ConsensusCrypto(bytes.fromhex("33" * 32))
    sigs, hs, pks = sv.make(one.ctx, n, lo=70000)
    got = c.verify_batch(list(map(bytes, sigs)), list(map(bytes, hs)), list(map(bytes, pks)))
    assert (got == 0).all()
    bad = [5, 700, 1030, 2000]
    _inject(sigs, hs, pks, golden_cases, bad[:2])
    for i in bad[2:]:
        sigs[i] = np.frombuffer(sv.add_g2(bytes(sigs[i])), dtype=np.uint8)
    got = c.verify_batch(list(map(bytes, sigs)), list(map(bytes, hs)), list(map(bytes, pks)))
    assert got.tolist() == sv.oracle_codes(sigs, hs, pks).tolist()
    # single calls rotate over the devices and agree
    for i in (0, 5, 1030):
        assert c.lib.ovh_verify(ctx.ptr, bytes(sigs[i]), 96, bytes(hs[i]), 32, bytes(pks[i]), 48) == got[i]


def test_rlc_cancellation_needs_known_seed():
    import consensus_overlord_amd as coa
    from consensus_overlord_amd.crypto import FLAG_TEST_RLC, Context
    from rlc_attack import cancel_pair
    with open(os.path.join(ROOT, "tests", "golden", "golden_v1.json")) as fh:
        g = json.load(fh)
    sigs = [bytes.fromhex(x["sig"]) for x in g["votes"][:4]]
    hs = [bytes.fromhex(x["digest"]) for x in g["votes"][:4]]
    pks = [bytes.fromhex(x["pk"]) for x in g["keys"][:4]]
    seed = 0x1234
    sigs[0], sigs[2] = cancel_pair(sigs[0], sigs[2], seed, 0, 2)
    c = coa.ConsensusCrypto(bytes.fromhex("44" * 32))
    for _ in range(3):    # fresh getrandom coefficients every batch
        assert c.verify_batch(sigs, hs, pks).tolist() == [5, 0, 5, 0]
    t = coa.ConsensusCrypto(bytes.fromhex("44" * 32), ctx=Context(flags=FLAG_TEST_RLC))
    t.ctx.set_test_rlc(seed, 0)
    # same coefficients as the oracle's SplitMix64 / GLV derivation: the forged pair cancels
    assert t.verify_batch(sigs, hs, pks).tolist() == [0, 0, 0, 0]
    t.ctx.set_test_rlc(seed + 1, 0)
    assert t.verify_batch(sigs, hs, pks).tolist() == [5, 0, 5, 0]


def test_unit_scalar_only_for_a_standalone_vote():
    """A batch of one vote checks its own pairing equation with scalar 1 (ovhip.hip
    vote_scalar / k_sig_as_S); a one-vote shard of a larger combined check must keep its random
    coefficient: sigma_0 + T and sigma_1 - T (cancelling under unit scalars) split over a
    two-device context are both flagged, and each alone verifies to 5."""
    import consensus_overlord_amd as coa
    from consensus_overlord_amd.crypto import Context
    from rlc_attack import bls
    with open(os.path.join(ROOT, "tests", "golden", "golden_v1.json")) as fh:
        g = json.load(fh)
    sigs = [bytes.fromhex(x["sig"]) for x in g["votes"][:2]]
    hs = [bytes.fromhex(x["digest"]) for x in g["votes"][:2]]
    pks = [bytes.fromhex(x["pk"]) for x in g["keys"][:2]]
    F, T = bls.Fp2Ops, bls.G2_GEN
    forged = [bls.g2_compress(bls.pt_add(F, bls.g2_from_bytes(sigs[0]), T)),
              bls.g2_compress(bls.pt_add(F, bls.g2_from_bytes(sigs[1]), bls.pt_neg(F, T)))]
    one = coa.ConsensusCrypto(bytes.fromhex("55" * 32))
    assert one.verify_batch(sigs[:1], hs[:1], pks[:1]).tolist() == [0]
    for k in range(2):
        assert one.verify_batch(forged[k:k + 1], hs[k:k + 1], pks[k:k + 1]).tolist() == [5]
        assert one.lib.ovh_verify(one.ctx.ptr, forged[k], 96, hs[k], 32, pks[k], 48) == 5
    multi = coa.ConsensusCrypto(bytes.fromhex("55" * 32), ctx=Context(devices=[0, 0]))
    for _ in range(3):
        assert multi.verify_batch(forged, hs, pks).tolist() == [5, 5]
        assert multi.verify_batch(sigs, hs, pks).tolist() == [0, 0]
