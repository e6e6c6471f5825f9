"""Same-message batches on the GPU (ovhip.hip verify_samemsg_locked): the
votes of a round all sign one hash (consensus.rs:169-175: Vote has no voter field), and a batch
over few distinct hashes is checked with one hash_to_G2 and one Miller loop per hash. Every code
is compared with the C oracle's per-vote verify (orc.verify / verify_many), with invalid votes
(sigma + G2, a signature outside G2, a key that does not parse), validator-table and other
voters mixed, several hashes per batch and a hash whose every vote fails."""
import json
import os

import numpy as np
import pytest

import orc
import synth_votes as sv

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def golden():
    with open(os.path.join(ROOT, "tests", "golden", "golden_v1.json")) as fh:
        return json.load(fh)


def _round(ctx, lo, n, digest):
    """n validators (synthetic keys lo..) signing one digest on the device -> sigs, pks (numpy)."""
    import torch
    from consensus_overlord_amd import device as dev
    sks = torch.from_numpy(sv.scalars(lo, n)).cuda()
    pks = dev.sk_to_pk_batch(ctx, sks).cpu().numpy()
    hs = torch.from_numpy(np.tile(np.frombuffer(digest, dtype=np.uint8), (n, 1))).cuda()
    sigs = dev.sign_batch(ctx, sks, hs).cpu().numpy()
    k = n // 2
    assert orc.sign(bytes(sv.scalars(lo + k, 1)[0]), digest) == (0, bytes(sigs[k])), "device signature"
    return sigs, pks


def _cc(key_hex, mode="2"):
    """A context whose batches take the same-message path at any size (OVH_SAMEMSG=2; by default
    only batches above the small-batch size do, include/ovhip.h)."""
    import consensus_overlord_amd as coa
    os.environ["OVH_SAMEMSG"] = mode
    try:
        return coa.ConsensusCrypto(bytes.fromhex(key_hex * 32))
    finally:
        del os.environ["OVH_SAMEMSG"]


def _named(golden, name, field):
    return np.frombuffer(bytes.fromhex([c for c in golden["verify"] if c["name"] == name][0][field]), dtype=np.uint8)


def test_relayer_round_99_of_100_prefetch_then_hits(golden):
    """The ingress case: a relayer receives 99 of the 100 precommits of a round (its own never
    crosses the network), 1% sigma + G2 and two golden negatives among them; one prefetch takes
    the same-message path, and every later verify_signature is a cache hit equal to orc.verify."""
    import consensus_overlord_amd as coa
    from consensus_overlord_amd.crypto import ConsensusError, CryptoErr
    cc = _cc("6b")
    digest = sv.sha(b"samemsg round 7")
    sigs, pks = _round(cc.ctx, 81000, 100, digest)
    cc.update_pubkeys([bytes(p) for p in pks])
    sigs, pks = sigs[1:].copy(), pks[1:].copy()          # validator 0 is this node
    sigs[17] = np.frombuffer(sv.add_g2(bytes(sigs[17])), dtype=np.uint8)
    sigs[40] = _named(golden, "sig_not_in_g2", "sig")     # -> POINT_NOT_IN_GROUP
    pks[63] = _named(golden, "pk_x_eq_p", "pk")           # -> lose public key (102)
    hs = np.tile(np.frombuffer(digest, dtype=np.uint8), (99, 1))
    want = sv.oracle_codes(sigs, hs, pks)
    assert sorted(set(want.tolist())) == [0, 3, 5, 102]
    b0 = cc.samemsg_stats()
    args = (list(map(bytes, sigs)), list(map(bytes, hs)), list(map(bytes, pks)))
    cc.prefetch(*args)
    b1 = cc.samemsg_stats()
    assert (b1[0] - b0[0], b1[1] - b0[1], b1[2] - b0[2]) == (1, 99, 1)
    h0, m0, _ = cc.cache_stats()
    for i in range(99):
        try:
            cc.verify_signature(*(a[i] for a in args))
            got = 0
        except CryptoErr as e:
            got = e.code
        except ConsensusError:
            got = 102
        assert got == want[i], i
    h1, m1, _ = cc.cache_stats()
    assert h1 - h0 == 99 and m1 == m0


def test_mixed_table_and_keys_three_hashes():
    """A backlog of prevotes, precommits and chokes (three hashes) whose voters are partly in the
    validator table: codes equal the oracle's, one same-message batch, both key sources."""
    import consensus_overlord_amd as coa
    cc = _cc("6c")
    ds = [sv.sha(b"prevote 9"), sv.sha(b"precommit 9"), sv.sha(b"choke 9")]
    S, H, K = [], [], []
    for d, n in zip(ds, (60, 60, 10)):
        sg, pk = _round(cc.ctx, 82000, n, d)
        S.append(sg)
        K.append(pk)
        H.append(np.tile(np.frombuffer(d, dtype=np.uint8), (n, 1)))
    sigs, hs, pks = np.concatenate(S), np.concatenate(H), np.concatenate(K)
    order = np.random.default_rng(9).permutation(len(sigs))
    sigs, hs, pks = sigs[order].copy(), hs[order].copy(), pks[order].copy()
    for i in (3, 77, 101):
        sigs[i] = np.frombuffer(sv.add_g2(bytes(sigs[i])), dtype=np.uint8)
    sigs[5] = sigs[6]                                      # another voter's signature on the same hash
    cc.update_pubkeys([bytes(p) for p in K[0][::2]])       # half of the validators in the table
    want = sv.oracle_codes(sigs, hs, pks)
    assert (want != 0).sum() == 4
    b0 = cc.samemsg_stats()
    got = cc.verify_batch(list(map(bytes, sigs)), list(map(bytes, hs)), list(map(bytes, pks)))
    b1 = cc.samemsg_stats()
    assert got.tolist() == want.tolist()
    assert (b1[0] - b0[0], b1[2] - b0[2]) == (1, 3)


def test_hash_whose_every_vote_fails_and_all_valid_batches():
    """A hash whose every vote fails contributes e(O, H) = 1 (its key sum is the identity): the
    other hash's votes still pass without bisection; an all-valid round passes as a whole."""
    import consensus_overlord_amd as coa
    cc = _cc("6d")
    da, db = sv.sha(b"round a"), sv.sha(b"round b")
    sa, pa = _round(cc.ctx, 83000, 40, da)
    sb, pb = _round(cc.ctx, 83100, 24, db)
    sb = np.stack([np.frombuffer(sv.add_g2(bytes(x)), dtype=np.uint8) for x in sb])
    sigs, pks = np.concatenate([sa, sb]), np.concatenate([pa, pb])
    hs = np.concatenate([np.tile(np.frombuffer(da, dtype=np.uint8), (40, 1)),
                         np.tile(np.frombuffer(db, dtype=np.uint8), (24, 1))])
    want = sv.oracle_codes(sigs, hs, pks)
    assert want[:40].tolist() == [0] * 40 and want[40:].tolist() == [5] * 24
    got = cc.verify_batch(list(map(bytes, sigs)), list(map(bytes, hs)), list(map(bytes, pks)))
    assert got.tolist() == want.tolist()
    # the failing hash first: its pair cannot join the final's loop (k_vm_gfin: verdict 0), the
    # per-vote bisection decides
    rev = np.concatenate([np.arange(40, 64), np.arange(40)])
    got = cc.verify_batch(list(map(bytes, sigs[rev])), list(map(bytes, hs[rev])), list(map(bytes, pks[rev])))
    assert got.tolist() == want[rev].tolist()
    got = cc.verify_batch(list(map(bytes, sa)), [da] * 40, list(map(bytes, pa)))
    assert got.tolist() == [0] * 40
    # one vote per hash on average is not a same-message batch
    b0 = cc.samemsg_stats()
    s2, h2, p2 = sv.make(cc.ctx, 6, lo=83200)
    assert cc.verify_batch(list(map(bytes, s2)), list(map(bytes, h2)), list(map(bytes, p2))).tolist() == [0] * 6
    assert cc.samemsg_stats() == b0


def test_samemsg_4096_one_hash_with_invalid_votes():
    """Config-3 keys all signing one hash (4,096 votes: the default routing takes the same-message
    path above the small-batch size): 1% sigma + G2 at seeded positions, every position flagged
    and the rest Ok, as the oracle on a sample; a 99-vote round on the default context takes the
    small-batch path (the lower latency) with the same codes."""
    import consensus_overlord_amd as coa
    cc = coa.ConsensusCrypto(bytes.fromhex("6e" * 32))
    n = 4096
    d = sv.sha(b"samemsg 4096")
    sigs, pks = _round(cc.ctx, 0, n, d)
    bad = sv.seeded_positions(n, 0.01, 44)
    for i in bad:
        sigs[i] = np.frombuffer(sv.add_g2(bytes(sigs[i])), dtype=np.uint8)
    hs = [d] * n
    b0 = cc.samemsg_stats()
    got = cc.verify_batch(list(map(bytes, sigs)), hs, list(map(bytes, pks)))
    assert cc.samemsg_stats()[0] == b0[0] + 1
    assert [i for i in range(n) if got[i] != 0] == bad
    assert set(got[bad].tolist()) == {5}
    for i in bad[:3] + [1, 2000, 4095]:
        assert orc.verify(bytes(sigs[i]), d, bytes(pks[i])) == got[i]
    small = cc.verify_batch(list(map(bytes, sigs[:99])), hs[:99], list(map(bytes, pks[:99])))
    assert small.tolist() == got[:99].tolist() and cc.samemsg_stats()[0] == b0[0] + 1


def test_device_async_pipeline_codes_equal_oracle():
    """ovh_verify_samemsg_device_async: five batches in flight over two hashes and two sizes (the
    one-hash plan is rebuilt when n changes), invalid votes (sigma + G2, another voter's
    signature, a key that does not parse) in some of them; after batch_wait every code equals the
    oracle's per-vote verify."""
    import torch
    import consensus_overlord_amd as coa
    from consensus_overlord_amd import device as dev
    cc = coa.ConsensusCrypto(bytes.fromhex("6f" * 32))
    da, db = sv.sha(b"pipelined a"), sv.sha(b"pipelined b")
    sa, pa = _round(cc.ctx, 84000, 300, da)
    sb, pb = _round(cc.ctx, 84000, 300, db)
    bad = sa.copy()
    bad[7] = np.frombuffer(sv.add_g2(bytes(bad[7])), dtype=np.uint8)
    bad[150] = bad[151]
    badk = pa.copy()
    badk[299] = np.frombuffer(bytes.fromhex("ff" * 48), dtype=np.uint8)
    jobs = [(sa, da, pa), (bad, da, badk), (sb, db, pb), (sb[:129], db, pb[:129]), (bad, da, pa)]
    codes = [torch.full((len(s),), -1, dtype=torch.int32, device="cuda") for s, _, _ in jobs]
    # the device inputs stay referenced until batch_wait (the library reads them on its own stream)
    dins = [(torch.from_numpy(s).cuda(), torch.from_numpy(p).cuda()) for s, _, p in jobs]
    torch.cuda.synchronize()
    for (_, d, _), (s_d, p_d), c in zip(jobs, dins, codes):
        dev.verify_samemsg_async(cc.ctx, s_d, d, p_d, c)
    dev.batch_wait(cc.ctx)
    for (s, d, p), c in zip(jobs, codes):
        want = sv.oracle_codes(s, np.tile(np.frombuffer(d, dtype=np.uint8), (len(s), 1)), p)
        assert c.cpu().numpy().tolist() == want.tolist()
    assert codes[1].cpu().numpy()[[7, 150, 299]].tolist() != [0, 0, 0]


def test_first_hash_all_malformed_takes_no_bisection():
    """a fresh hash whose only votes are malformed (96 bytes that do not
    parse), arriving first, must not make the combined check degenerate. Its key sum is the
    identity, so the device picks the next hash as the head of the final's two-pair loop
    (k_pick_head): the codes equal the oracle's and the batch's bisection stage does no per-vote
    work (stage time, OVH_FLAG_PROFILE context) -- with hash 0 as the fixed head every valid vote
    went through a per-vote Miller loop and final exponentiation."""
    import ctypes
    import consensus_overlord_amd as coa
    from consensus_overlord_amd.crypto import Context, FLAG_PROFILE
    os.environ["OVH_SAMEMSG"] = "2"
    try:
        ctx = Context(0, flags=FLAG_PROFILE)
    finally:
        del os.environ["OVH_SAMEMSG"]
    cc = coa.ConsensusCrypto(bytes.fromhex("71" * 32), ctx=ctx)
    da, db = sv.sha(b"fresh hash, malformed votes"), sv.sha(b"round 12 precommit")
    sb, pb = _round(cc.ctx, 85000, 48, db)
    junk = np.frombuffer(bytes.fromhex("ff" * 96), dtype=np.uint8)
    sa, pa = np.stack([junk] * 3), pb[:3].copy()
    sigs, pks = np.concatenate([sa, sb]), np.concatenate([pa, pb])
    hs = np.concatenate([np.tile(np.frombuffer(da, dtype=np.uint8), (3, 1)),
                         np.tile(np.frombuffer(db, dtype=np.uint8), (48, 1))])
    want = sv.oracle_codes(sigs, hs, pks)
    assert want[:3].tolist() == [1, 1, 1] and want[3:].tolist() == [0] * 48
    b0 = cc.samemsg_stats()
    got = cc.verify_batch(list(map(bytes, sigs)), list(map(bytes, hs)), list(map(bytes, pks)))
    assert got.tolist() == want.tolist()
    assert cc.samemsg_stats()[0] == b0[0] + 1
    names = [ctx.lib.ovh_stage_name(k).decode() for k in range(6)]
    ms = (ctypes.c_float * 6)()
    assert ctx.lib.ovh_stage_times(ctx.ptr, ms, 6) == 6
    # the per-vote bisection of 48 votes is milliseconds of Miller loops and final
    # exponentiations; skipped, its kernels exit at their first instruction
    assert ms[names.index("bisect")] < 0.5, list(ms)
