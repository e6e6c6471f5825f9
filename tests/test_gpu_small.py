"""GPU parity of the small-batch path (ovhip.hip verify_small_locked: batches of 2 .. 1024 votes,
one vote per wave, f_i = Miller(r pk, H) Miller(-G1, r sigma), one final exponentiation of the
folded product, per-vote FE(f_i) when it fails) against the golden codes, the C oracle and the
standard batch path (a context created with OVH_SMALL_MAX=0: vote kernel + MSM + final)."""
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _b(h):
    return bytes.fromhex(h)


def _ctx(small: bool, **kw):
    """A ConsensusCrypto whose context takes (small) or skips (not small) the small-batch path."""
    import consensus_overlord_amd as coa
    from consensus_overlord_amd.crypto import Context
    old = os.environ.get("OVH_SMALL_MAX")
    if not small:
        os.environ["OVH_SMALL_MAX"] = "0"
    try:
        return coa.ConsensusCrypto(bytes.fromhex("66" * 32), ctx=Context(**kw))
    finally:
        if old is None:
            os.environ.pop("OVH_SMALL_MAX", None)
        else:
            os.environ["OVH_SMALL_MAX"] = old


@pytest.fixture(scope="module")
def pair():
    return _ctx(True), _ctx(False)


def test_small_path_golden_codes(pair, golden):
    """Every fixed-size golden verify case in one batch (parse failures, subgroup failures,
    infinity, wrong message / key / signature) on both paths == the golden per-vote code."""
    cases = [c for c in golden["verify"] if len(_b(c["sig"])) == 96 and len(_b(c["hash"])) == 32
             and len(_b(c["pk"])) == 48]
    assert 2 <= len(cases) <= 1024
    want = [c["code"] for c in cases]
    for cc in pair:
        got = cc.verify_batch([_b(c["sig"]) for c in cases], [_b(c["hash"]) for c in cases],
                              [_b(c["pk"]) for c in cases])
        assert list(got) == want


def test_small_path_sizes_and_invalid_positions(pair, golden):
    """Batches of 2, 3, 5, 64 and 1024 golden votes (repeated) with sigma + G2 and swapped
    signatures at seeded positions: the small path flags exactly the votes the C oracle flags,
    as the standard path does."""
    import bls12_381 as bls
    import orc
    v, k = golden["votes"], golden["keys"]
    rng = random.Random(11)
    for n in (2, 3, 5, 64, 1024):
        idx = [i % len(v) for i in range(n)]
        sigs = [_b(v[j]["sig"]) for j in idx]
        hs = [_b(v[j]["digest"]) for j in idx]
        pks = [_b(k[j]["pk"]) for j in idx]
        for i in rng.sample(range(n), max(1, n // 50)):
            if rng.random() < 0.5:
                pt = bls.g2_from_bytes(sigs[i])
                sigs[i] = bls.g2_compress(bls.pt_add(bls.Fp2Ops, pt, bls.G2_GEN))
            else:
                sigs[i] = sigs[(i + 1) % n] if idx[(i + 1) % n] != idx[i] else _b(v[(idx[i] + 1) % len(v)]["sig"])
        cat = [np.frombuffer(b"".join(x), dtype=np.uint8) for x in (sigs, hs, pks)]
        want = orc.verify_many(*cat, threads=8)
        for cc in pair:
            assert list(cc.verify_batch(sigs, hs, pks)) == list(want), n


def test_small_path_validator_table(pair, golden):
    """Table votes (votew_t) and key-byte votes (votew) of one mixed batch on the small path
    (the table / other split), against the standard path and the golden codes."""
    cases = [c for c in golden["verify"] if len(_b(c["sig"])) == 96 and len(_b(c["hash"])) == 32
             and len(_b(c["pk"])) == 48]
    keys = [_b(x["pk"]) for x in golden["keys"]]
    for cc in pair:
        cc.update_pubkeys(keys)
        try:
            got = cc.verify_batch([_b(c["sig"]) for c in cases], [_b(c["hash"]) for c in cases],
                                  [_b(c["pk"]) for c in cases])
            assert list(got) == [c["code"] for c in cases]
        finally:
            cc.update_pubkeys([])


def test_small_path_device_batch_config5(pair):
    """Config 5 at its size through the device entry point on both paths: 1024 synthetic votes,
    1% sigma + G2 at seeded positions, every position flagged and the rest Ok."""
    import torch
    import bls12_381 as bls
    from consensus_overlord_amd import device as dev
    from test_gpu_parity import _synth
    cc = pair[0]
    n = 1024
    sks, hs = _synth(n, seed=0xC5)
    pks = dev.sk_to_pk_batch(cc.ctx, sks)
    sigs = dev.sign_batch(cc.ctx, sks, hs)
    bad = sorted(random.Random(5).sample(range(n), n // 100))
    s_host = sigs.cpu().numpy().copy()
    for i in bad:
        pt = bls.g2_from_bytes(bytes(s_host[i]))
        s_host[i] = np.frombuffer(bls.g2_compress(bls.pt_add(bls.Fp2Ops, pt, bls.G2_GEN)), dtype=np.uint8)
    sigs2 = torch.from_numpy(s_host).cuda()
    torch.cuda.synchronize()
    for c in pair:
        codes = dev.verify_batch(c.ctx, sigs2, hs, pks).cpu().numpy()
        assert [i for i in range(n) if codes[i] != 0] == bad
        assert all(codes[i] == 5 for i in bad)
        assert (dev.verify_batch(c.ctx, sigs, hs, pks).cpu().numpy() == 0).all()
