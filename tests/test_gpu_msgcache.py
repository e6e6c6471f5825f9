"""GPU parity of the per-call message cache (ovhip.hip verify_one_locked: H = hash_to_G2(hash)
kept for the last 256 hashes verified per call; a later vote on a cached hash runs vote1h /
vote_t1h without hash_to_G2). Codes against the golden fixtures and the C oracle, on hits,
misses, the validator-table variant and after eviction."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _b(h):
    return bytes.fromhex(h)


def _stats(cc):
    st = (ctypes.c_uint64 * 2)()
    assert cc.lib.ovh_msg_cache_stats(cc.ctx.ptr, st) == 0
    return st[0], st[1]


def _verify(cc, sig, h, pk):
    return cc.lib.ovh_verify(cc.ctx.ptr, sig, len(sig), h, len(h), pk, len(pk))


def test_same_hash_votes_hit_the_cache(golden):
    """Four golden keys sign one hash (library signing, checked against the oracle elsewhere):
    the first verify misses, the rest hit; valid votes verify, swapped signatures fail with 5,
    and every golden verify case on that hash keeps its exact code on the hit path."""
    import consensus_overlord_amd as coa
    from consensus_overlord_amd.crypto import FLAG_SK_RAW, Context
    import orc
    raw = Context(flags=FLAG_SK_RAW)
    keys = golden["keys"][:4]
    cc = coa.ConsensusCrypto(bytes.fromhex("77" * 32))
    h = _b(golden["votes"][0]["digest"])
    sigs = [coa.ConsensusCrypto(_b(k["sk"]), ctx=raw).sign(h) for k in keys]
    pks = [_b(k["pk"]) for k in keys]
    h0, m0 = _stats(cc)
    assert _verify(cc, sigs[0], h, pks[0]) == 0
    h1, m1 = _stats(cc)
    assert (h1 - h0, m1 - m0) == (0, 1)
    for k in range(1, 4):
        assert _verify(cc, sigs[k], h, pks[k]) == 0
        assert _verify(cc, sigs[k], h, pks[k - 1]) == 5 == orc.verify(sigs[k], h, pks[k - 1])
    h2, m2 = _stats(cc)
    assert (h2 - h1, m2 - m1) == (6, 0)
    # golden cases on the cached hash: parse / subgroup / infinity failures on the vote1h path
    same = [c for c in golden["verify"] if _b(c["hash"]) == h and len(_b(c["sig"])) == 96 and len(_b(c["pk"])) == 48]
    assert len(same) >= 5
    for c in same:
        assert _verify(cc, _b(c["sig"]), h, _b(c["pk"])) == c["code"], c["name"]
    assert _stats(cc)[1] == m2


def test_table_votes_on_cached_hash(golden):
    """vote_t1h: voters in the validator table, on a cached hash, == the golden codes."""
    import consensus_overlord_amd as coa
    cc = coa.ConsensusCrypto(bytes.fromhex("78" * 32))
    cc.update_pubkeys([_b(k["pk"]) for k in golden["keys"]])
    v, k = golden["votes"], golden["keys"]
    for rep in range(2):
        for j in range(len(v)):
            assert _verify(cc, _b(v[j]["sig"]), _b(v[j]["digest"]), _b(k[j]["pk"])) == 0, (rep, j)
            other = _b(v[(j + 1) % len(v)]["sig"])
            assert _verify(cc, other, _b(v[j]["digest"]), _b(k[j]["pk"])) == 5, (rep, j)
    hits, misses = _stats(cc)
    assert misses == len(v) and hits == 3 * len(v)


def test_eviction_keeps_codes():
    """300 distinct hashes through a 256-entry cache, then the first ones again (evicted:
    misses) and the last ones (still cached: hits): every vote verifies, a swapped one fails."""
    import hashlib
    import torch
    import consensus_overlord_amd as coa
    from consensus_overlord_amd import device as dev
    cc = coa.ConsensusCrypto(bytes.fromhex("79" * 32))
    n = 300
    sk = (1234567).to_bytes(32, "big")
    sks = torch.from_numpy(np.tile(np.frombuffer(sk, dtype=np.uint8), (n, 1))).cuda()
    hs_h = np.stack([np.frombuffer(hashlib.sha256(b"msg%d" % i).digest(), dtype=np.uint8) for i in range(n)])
    sigs = dev.sign_batch(cc.ctx, sks, torch.from_numpy(hs_h).cuda()).cpu().numpy()
    pk = bytes(dev.sk_to_pk_batch(cc.ctx, sks[:1]).cpu().numpy()[0])
    for i in range(n):
        assert _verify(cc, bytes(sigs[i]), bytes(hs_h[i]), pk) == 0, i
    h0, m0 = _stats(cc)
    assert m0 == n
    for i in (0, 1, 2):
        assert _verify(cc, bytes(sigs[i]), bytes(hs_h[i]), pk) == 0
    for i in (n - 1, n - 2):
        assert _verify(cc, bytes(sigs[i]), bytes(hs_h[i]), pk) == 0
        assert _verify(cc, bytes(sigs[i - 1]), bytes(hs_h[i]), pk) == 5
    h1, m1 = _stats(cc)
    assert (h1 - h0, m1 - m0) == (4, 3)
