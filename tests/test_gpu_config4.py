"""Config 4 at its size (BASELINE.json configs[3]): 65,536 SURVEY 8(d) votes
split into 8 shards of 8,192, invalid votes in two different shards (sigma + G2 in shard 1, the
golden negative cases in shard 6), codes compared with the C oracle's per-vote verify
(orc.verify_many, 16 threads; consensus.rs:397-416 vote by vote). Two forms of the split:

  * one process, eight devices: ovh_create_multi({0} x 8) on the one-GPU box -- eight device
    pipelines, partials peer-copied to devices[0], one combined check, per-device bisection;
  * eight "ranks" in one process: eight contexts, each ovh_batch_partial_device on its shard,
    the 8 x 864-byte partials gathered into one buffer (the all-gather of shard.py), then every
    context's ovh_combine_partials_device_async + bisection of its own shard."""
import json
import os

import numpy as np
import pytest

import synth_votes as sv

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, SHARDS = 65536, 8
SH = N // SHARDS


@pytest.fixture(scope="module")
def workload():
    import consensus_overlord_amd as coa
    with open(os.path.join(ROOT, "tests", "golden", "golden_v1.json")) as fh:
        g = json.load(fh)
    neg = [c for c in g["verify"] if len(c["sig"]) == 192 and len(c["hash"]) == 64 and len(c["pk"]) == 96
           and c["code"] != 0]
    one = coa.ConsensusCrypto(bytes.fromhex("c4" * 32))
    sigs, hs, pks = sv.make(one.ctx, N, lo=0)
    one.ctx.close()
    g2 = [SH + k for k in (0, 17, 4095, 8191)]                       # shard 1: sigma + G2
    for i in g2:
        sigs[i] = np.frombuffer(sv.add_g2(bytes(sigs[i])), dtype=np.uint8)
    gn = [6 * SH + 3 + 97 * k for k in range(len(neg))]               # shard 6: golden negatives
    for c, i in zip(neg, gn):
        sigs[i] = np.frombuffer(bytes.fromhex(c["sig"]), dtype=np.uint8)
        hs[i] = np.frombuffer(bytes.fromhex(c["hash"]), dtype=np.uint8)
        pks[i] = np.frombuffer(bytes.fromhex(c["pk"]), dtype=np.uint8)
    want = sv.oracle_codes(sigs, hs, pks, threads=16)
    assert sorted(np.nonzero(want)[0].tolist()) == sorted(g2 + gn)
    return sigs, hs, pks, want


def test_config4_65536_votes_eight_device_context(workload):
    import consensus_overlord_amd as coa
    from consensus_overlord_amd.crypto import Context
    sigs, hs, pks, want = workload
    ctx = Context(devices=[0] * SHARDS)
    assert ctx.device_count == SHARDS
    c = coa.ConsensusCrypto(bytes.fromhex("c4" * 32), ctx=ctx)
    got = c.verify_batch(list(map(bytes, sigs)), list(map(bytes, hs)), list(map(bytes, pks)))
    assert got.tolist() == want.tolist()
    ctx.close()


def test_config4_65536_votes_eight_shard_partials(workload):
    import torch
    from consensus_overlord_amd import device as dev
    from consensus_overlord_amd.crypto import Context
    sigs, hs, pks, want = workload
    ctxs = [Context(0) for _ in range(SHARDS)]
    st = torch.cuda.Stream()
    d = [torch.from_numpy(x.copy()).cuda() for x in (sigs, hs, pks)]
    codes = torch.full((N,), -1, dtype=torch.int32, device="cuda")
    parts = torch.zeros((SHARDS, 864), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    with torch.cuda.stream(st):
        for r, cx in enumerate(ctxs):
            lo, hi = r * SH, (r + 1) * SH
            mine = torch.empty((864,), dtype=torch.uint8, device="cuda")
            dev.batch_partial(cx, d[0][lo:hi], d[1][lo:hi], d[2][lo:hi], codes[lo:hi], mine, stream=st)
            parts[r].copy_(mine)                                      # the all-gather
        for r, cx in enumerate(ctxs):
            lo, hi = r * SH, (r + 1) * SH
            dev.combine_partials_async(cx, parts, SH, codes[lo:hi], stream=st)
    for cx in ctxs:
        dev.batch_wait(cx)
    torch.cuda.synchronize()
    assert codes.cpu().numpy().tolist() == want.tolist()
    # the shards' partials alone: the combined check fails (invalid votes in shards 1 and 6)
    assert dev.combine_partials(ctxs[0], parts) is False
    ok = [r for r in range(SHARDS) if r not in (1, 6)]
    assert dev.combine_partials(ctxs[0], parts[ok]) is True
    for cx in ctxs:
        cx.close()


def _corrupt(base, golden_negs, batch):
    """Batch `batch` of the pipelined tests: the base votes with sigma + G2 and golden negatives
    at batch-dependent positions (both shards of a two-device split)."""
    sigs, hs, pks = (x.copy() for x in base)
    n = sigs.shape[0]
    pos = [(977 * batch + 131 * k) % n for k in range(3)] + [n // 2 + 7 * batch + 1]
    for i in pos[:2]:
        sigs[i] = np.frombuffer(sv.add_g2(bytes(sigs[i])), dtype=np.uint8)
    for c, i in zip(golden_negs[batch % len(golden_negs):], pos[2:]):
        sigs[i] = np.frombuffer(bytes.fromhex(c["sig"]), dtype=np.uint8)
        hs[i] = np.frombuffer(bytes.fromhex(c["hash"]), dtype=np.uint8)
        pks[i] = np.frombuffer(bytes.fromhex(c["pk"]), dtype=np.uint8)
    return (sigs, hs, pks), sorted(set(pos))


def _want(batch, base_want, pos):
    import orc
    sigs, hs, pks = batch
    w = base_want.copy()
    for i in pos:
        w[i] = orc.verify(bytes(sigs[i]), bytes(hs[i]), bytes(pks[i]))
    return w


@pytest.fixture(scope="module")
def golden_negs():
    with open(os.path.join(ROOT, "tests", "golden", "golden_v1.json")) as fh:
        g = json.load(fh)
    return [c for c in g["verify"] if len(c["sig"]) == 192 and len(c["hash"]) == 64 and len(c["pk"]) == 96
            and c["code"] != 0]


@pytest.mark.parametrize("devices,nb,n", [([0, 0], 4, 8192), (None, 8, 1024)])
def test_pipelined_host_batches(golden_negs, devices, nb, n):
    """ovh_verify_batch_async: four 8,192-vote batches over a two-device context ({0, 0}: two
    device pipelines, rotating final device) and eight 1,024-vote batches on one context (the ring
    of OVH_BATCH_SLOTS = 6 slots wraps), invalid votes in flight in every batch and half the voters in the
    validator table (table / other split per shard); every batch's codes equal the oracle's."""
    import consensus_overlord_amd as coa
    from consensus_overlord_amd.crypto import Context
    one = coa.ConsensusCrypto(bytes.fromhex("c5" * 32))
    base = sv.make(one.ctx, n, lo=200000)
    base_want = sv.oracle_codes(*base, threads=16)
    assert (base_want == 0).all()
    c = coa.ConsensusCrypto(bytes.fromhex("c5" * 32), ctx=Context(devices=devices) if devices else None)
    c.update_pubkeys([bytes(base[2][i]) for i in range(0, n, 2)])
    batches = [_corrupt(base, golden_negs, b) for b in range(nb)]
    outs = [np.full(n, -1, dtype=np.int32) for _ in range(nb)]
    for (bt, _), o in zip(batches, outs):
        c.verify_batch_async(list(map(bytes, bt[0])), list(map(bytes, bt[1])), list(map(bytes, bt[2])), o)
    c.wait()
    for b, ((bt, pos), o) in enumerate(zip(batches, outs)):
        assert o.tolist() == _want(bt, base_want, pos).tolist(), b
        assert (o[pos] != 0).all()
