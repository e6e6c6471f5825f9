"""The vote pool (ovhip.hip k_vm_pool; DESIGN.md section 3, "Vote pool") through the pipelined
C ABI (ovh_verify_batch_device_async + ovh_batch_wait), against the C oracle's per-vote verify.

The pool reads a batch on its own schedule, batches later; the library stages each batch's
signatures and keys into the batch slot's own buffer on ovh_stream (k_pool_stage) and consumes
the hashes there (hash_to_field), so the contract of include/ovhip.h holds: the inputs are read
in ovh_stream order, and work the caller enqueues on ovh_stream after the call may overwrite
them."""
import numpy as np
import pytest

import synth_votes as sv

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def votes():
    from consensus_overlord_amd.crypto import Context
    ctx = Context(0)
    s, h, p = sv.make(ctx, 2048, lo=86000)
    ctx.close()
    return s, h, p


def test_inputs_overwritten_on_ovh_stream_after_enqueue(votes):
    """Six pipelined 2,048-vote batches from ONE set of input buffers: after each enqueue the
    caller overwrites the buffers on ovh_stream -- the next batch's inputs, or junk after the last
    -- while the pool has not yet reached that batch. Every batch's codes equal the oracle's for
    the inputs it was enqueued with (batches 1, 3, 5 carry 1% sigma + G2 and a key that does not
    parse; 0, 2, 4 are valid)."""
    import torch
    from consensus_overlord_amd import device as dev
    from consensus_overlord_amd.crypto import Context
    s, h, p = votes
    n = len(s)
    bad_s, bad_p = s.copy(), p.copy()
    flagged = sv.seeded_positions(n, 0.01, 51)
    for i in flagged:
        bad_s[i] = np.frombuffer(sv.add_g2(bytes(bad_s[i])), dtype=np.uint8)
    bad_p[7] = np.frombuffer(bytes.fromhex("ff" * 48), dtype=np.uint8)
    jobs = [(s, p) if k % 2 == 0 else (bad_s, bad_p) for k in range(6)]
    want_bad = sv.oracle_codes(bad_s, h, bad_p)
    assert (want_bad != 0).sum() == len(flagged) + (0 if 7 in flagged else 1)

    ctx = Context(0)
    ovh = torch.cuda.ExternalStream(ctx.stream)
    d_s = torch.empty((n, 96), dtype=torch.uint8, device="cuda")
    d_h = torch.from_numpy(h).cuda()
    d_p = torch.empty((n, 48), dtype=torch.uint8, device="cuda")
    # the batches' inputs as device tensors made on torch's stream before the loop (device-to-device
    # copies on ovh_stream below: no pinned host block records an event on the library's stream)
    src = [(torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()) for a, b in jobs]
    codes = [torch.full((n,), -1, dtype=torch.int32, device="cuda") for _ in jobs]
    junk = torch.full((n, 96), 0xFF, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    with torch.cuda.stream(ovh):
        d_s.copy_(src[0][0])
        d_p.copy_(src[0][1])
    for k in range(len(jobs)):
        dev.verify_batch_async(ctx, d_s, d_h, d_p, codes[k])
        with torch.cuda.stream(ovh):   # stream-ordered after the call: the library has staged them
            if k + 1 < len(jobs):
                d_s.copy_(src[k + 1][0])
                d_p.copy_(src[k + 1][1])
            else:
                d_s.copy_(junk)
                d_p.copy_(junk[:, :48])
                d_h.zero_()
    dev.batch_wait(ctx)
    torch.cuda.synchronize()
    for k in range(len(jobs)):
        got = codes[k].cpu().numpy()
        if k % 2 == 0:
            assert (got == 0).all(), (k, np.nonzero(got)[0][:8])
        else:
            assert got.tolist() == want_bad.tolist(), k
    del src, d_s, d_h, d_p, junk, codes
    torch.cuda.synchronize()
    ctx.close()


def _bad_jobs(votes):
    s, h, p = votes
    n = len(s)
    bad_s, bad_p = s.copy(), p.copy()
    for i in sv.seeded_positions(n, 0.01, 53):
        bad_s[i] = np.frombuffer(sv.add_g2(bytes(bad_s[i])), dtype=np.uint8)
    bad_p[11] = np.frombuffer(bytes.fromhex("ff" * 48), dtype=np.uint8)
    return bad_s, bad_p, sv.oracle_codes(bad_s, h, bad_p)


def test_pinned_host_inputs_on_ovh_stream_then_close(votes):
    """The r05ab pattern: the inputs come from PINNED host tensors copied
    with non_blocking=True on torch.cuda.ExternalStream(ctx.stream), so torch's pinned-host
    allocator records its own events on the library's stream; the context is then closed while
    those blocks are still cached and their events not yet queried. ovh_destroy parks its streams
    instead of destroying them (include/ovhip.h), so the allocator's later event queries -- on
    freeing the tensors, on the next pinned allocation, and in a second context that takes the
    parked streams back -- touch live streams. Codes equal the oracle's."""
    import torch
    from consensus_overlord_amd import device as dev
    from consensus_overlord_amd.crypto import Context
    s, h, p = votes
    n = len(s)
    bad_s, bad_p, want_bad = _bad_jobs(votes)
    jobs = [(s, p), (bad_s, bad_p), (s, p), (bad_s, bad_p)]
    ctx = Context(0)
    ovh = torch.cuda.ExternalStream(ctx.stream)
    src = [(torch.from_numpy(a.copy()).pin_memory(), torch.from_numpy(b.copy()).pin_memory()) for a, b in jobs]
    d_h = torch.from_numpy(h).cuda()
    ins = [(torch.empty((n, 96), dtype=torch.uint8, device="cuda"),
            torch.empty((n, 48), dtype=torch.uint8, device="cuda")) for _ in jobs]
    codes = [torch.full((n,), -1, dtype=torch.int32, device="cuda") for _ in jobs]
    torch.cuda.synchronize()
    for k in range(len(jobs)):
        with torch.cuda.stream(ovh):
            ins[k][0].copy_(src[k][0], non_blocking=True)
            ins[k][1].copy_(src[k][1], non_blocking=True)
        dev.verify_batch_async(ctx, ins[k][0], d_h, ins[k][1], codes[k])
    dev.batch_wait(ctx)
    got = [c.cpu().numpy() for c in codes]
    ctx.close()                      # streams parked; torch still holds events recorded on them
    del src                          # the pinned blocks go back to torch's cache (event bookkeeping)
    more = torch.empty((n, 96), dtype=torch.uint8).pin_memory()   # the allocator processes its events
    ctx2 = Context(0)                # takes the parked streams back
    ovh2 = torch.cuda.ExternalStream(ctx2.stream)
    with torch.cuda.stream(ovh2):
        more.copy_(torch.from_numpy(s), non_blocking=False)
        ins[0][0].copy_(more, non_blocking=True)
    c2 = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    dev.verify_batch_async(ctx2, ins[0][0], d_h, ins[0][1], c2)
    dev.batch_wait(ctx2)
    assert (c2.cpu().numpy() == 0).all()
    ctx2.close()
    del more, ins, codes, c2
    torch.cuda.synchronize()
    for k in range(len(jobs)):
        if k % 2 == 0:
            assert (got[k] == 0).all(), (k, np.nonzero(got[k])[0][:8])
        else:
            assert got[k].tolist() == want_bad.tolist(), k


@pytest.mark.parametrize("reserve", [False, True])
def test_async_batch_then_shard_partial_without_wait(votes, reserve):
    """a pipelined batch (persistent pool grids) and, with no ovh_batch_wait
    between them, a shard batch (ovh_batch_partial_device on a stream: a grid of its own on the
    other pool stream) are in the pool together. Each pool stream has its own fixed spill-scratch
    region, so no two co-resident workgroups share one; both batches' codes equal the oracle's.
    reserve: the same on an OVH_FLAG_POOL_RESERVE context (CU-masked pool streams; the shard batch
    joins the persistent pool)."""
    import torch
    from consensus_overlord_amd import device as dev
    from consensus_overlord_amd.crypto import Context, FLAG_POOL_RESERVE
    s, h, p = votes
    n = len(s)
    bad_s, bad_p, want_bad = _bad_jobs(votes)
    ctx = Context(0, flags=FLAG_POOL_RESERVE if reserve else 0)
    d_h = torch.from_numpy(h).cuda()
    a_s, a_p = torch.from_numpy(bad_s).cuda(), torch.from_numpy(bad_p).cuda()
    b_s, b_p = torch.from_numpy(s).cuda(), torch.from_numpy(p).cuda()
    codes_a = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    codes_b = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    codes_c = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    part = torch.zeros((1, 864), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        dev.verify_batch_async(ctx, a_s, d_h, a_p, codes_a)
        dev.batch_partial(ctx, a_s, d_h, a_p, codes_b, part[0], stream=True)
        dev.combine_partials_async(ctx, part, n, codes_b, stream=True)
        dev.verify_batch_async(ctx, b_s, d_h, b_p, codes_c)
    dev.batch_wait(ctx)
    torch.cuda.synchronize()
    assert codes_a.cpu().numpy().tolist() == want_bad.tolist()
    assert codes_b.cpu().numpy().tolist() == want_bad.tolist()
    assert (codes_c.cpu().numpy() == 0).all()
    ctx.close()


def test_reserved_pool_shard_pipeline_with_gather_copies(votes):
    """OVH_FLAG_POOL_RESERVE (include/ovhip.h): eight shard batches -- more than the context's
    batch slots -- pipelined on one stream as bench.py's shard path runs them: partial, a
    device copy of the partial standing in for the RCCL all-gather (a kernel that needs CU places
    beside the persistent pool), combine. Batches 2 and 5 carry invalid votes; every batch's codes
    equal the oracle's. Then the masked streams are parked and taken back: an unreserved context
    in between runs a batch of its own on unmasked streams."""
    import torch
    from consensus_overlord_amd import device as dev
    from consensus_overlord_amd.crypto import Context, FLAG_POOL_RESERVE
    s, h, p = votes
    n = len(s)
    bad_s, bad_p, want_bad = _bad_jobs(votes)
    d_h = torch.from_numpy(h).cuda()
    good = (torch.from_numpy(s).cuda(), torch.from_numpy(p).cuda())
    bad = (torch.from_numpy(bad_s).cuda(), torch.from_numpy(bad_p).cuda())
    for rep in range(2):
        ctx = Context(0, flags=FLAG_POOL_RESERVE)
        nb = 8
        codes = torch.full((nb, n), -1, dtype=torch.int32, device="cuda")
        mine = torch.zeros((nb, 864), dtype=torch.uint8, device="cuda")
        gathered = torch.zeros((nb, 1, 864), dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):
            for b in range(nb):
                sg, pk = bad if b in (2, 5) else good
                dev.batch_partial(ctx, sg, d_h, pk, codes[b], mine[b], stream=True)
                gathered[b, 0].copy_(mine[b])
                dev.combine_partials_async(ctx, gathered[b], n, codes[b], stream=True)
        dev.batch_wait(ctx)
        torch.cuda.synchronize()
        got = codes.cpu().numpy()
        for b in range(nb):
            want = want_bad.tolist() if b in (2, 5) else [0] * n
            assert got[b].tolist() == want, (rep, b)
        ctx.close()
        if rep == 0:
            other = Context(0)
            c2 = torch.full((n,), -1, dtype=torch.int32, device="cuda")
            dev.verify_batch_async(other, bad[0], d_h, bad[1], c2)
            dev.batch_wait(other)
            torch.cuda.synchronize()
            assert c2.cpu().numpy().tolist() == want_bad.tolist()
            other.close()
