"""Multi-GPU orchestration (consensus_overlord_amd/shard.py) on CPU: world_size 2 over gloo,
each rank verifying its shard of the golden votes with the C oracle as the compute backend
(test infrastructure; the GPU backend is libovhip). Checks: per-rank codes equal the per-vote
verdicts, the pipelined double-buffered partials, the combined verdict equals the single-process
RLC batch (one global vote index across the ranks), and a batch with one swapped signature falls
back exactly on the owning shard."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import orc
from consensus_overlord_amd.shard import ShardVerifier, shard_bounds


class OracleBackend:
    """Test seeds (the device backend draws secret ones): batch s uses seed 0xC17A + s, vote i of
    the whole batch SplitMix64(seed, i) -- the rank's shard offset is the index base."""

    def __init__(self):
        self.last = None
        self.verdicts = []
        self.batch = 0

    def empty_partials(self, world):
        return torch.zeros((2, world, 864), dtype=torch.uint8)

    def partial(self, sigs, hashes, pks, codes, out_row, index_base):
        seed = 0xC17A + self.batch
        self.batch += 1
        c, part = orc.batch_partial(sigs.numpy(), hashes.numpy(), pks.numpy(), seed, base=index_base)
        codes.copy_(torch.from_numpy(c))
        out_row.copy_(torch.from_numpy(part))
        self.last = (sigs.numpy(), hashes.numpy(), pks.numpy())

    def combine_async(self, parts, n, codes):
        ok = orc.combine_partials(parts.numpy())
        self.verdicts.append(ok)
        if not ok:
            orc.batch_fallback(*self.last, codes.numpy())

    def wait(self):
        pass


def _batches(golden):
    v, k = golden["votes"], golden["keys"]
    sigs = np.stack([np.frombuffer(bytes.fromhex(x["sig"]), dtype=np.uint8) for x in v])
    hs = np.stack([np.frombuffer(bytes.fromhex(x["digest"]), dtype=np.uint8) for x in v])
    pks = np.stack([np.frombuffer(bytes.fromhex(x["pk"]), dtype=np.uint8) for x in k])
    bad = sigs.copy()
    bad[[1, 6]] = sigs[[6, 1]]          # votes 1 and 6 (different shards) swap signatures
    return [(sigs, hs, pks), (bad, hs, pks), (sigs, hs, pks)]


def _worker(rank, world, port, golden, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    be = OracleBackend()
    sv = ShardVerifier(be)
    out = []
    for s, (sg, hs, pk) in enumerate(_batches(golden)):
        lo, hi = shard_bounds(len(sg), world, rank)
        codes = torch.full((hi - lo,), -1, dtype=torch.int32)
        sv.submit(s, torch.from_numpy(sg[lo:hi].copy()), torch.from_numpy(hs[lo:hi].copy()),
                  torch.from_numpy(pk[lo:hi].copy()), codes, index_base=lo)
        out.append(codes)
    sv.wait()
    got = [None] * world
    dist.all_gather_object(got, ([c.tolist() for c in out], be.verdicts))
    if rank == 0:
        q.put(got)
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_gloo_shards(golden):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, golden, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for s, (sg, hs, pk) in enumerate(_batches(golden)):
        want = orc.verify_many(sg, hs, pk)
        codes = np.concatenate([np.array(got[r][0][s], dtype=np.int32) for r in range(world)])
        assert codes.tolist() == want.tolist(), s
        # every rank saw the same combined verdict, equal to the single-process RLC batch's
        ref_codes, ref_ok = orc.verify_batch_rlc(sg, hs, pk, seed=0xC17A + s)
        assert got[0][1][s] == got[1][1][s] == ref_ok == (s != 1)
        assert ref_codes.tolist() == want.tolist()



class AsyncOracleBackend(OracleBackend):
    """The oracle behind a host "stream": partial, gather and combine are queued tasks run in
    order by one worker thread, which starts only at wait() -- so submit() returns before any
    code is written, batches pile up in flight, and the partial rows (BATCH_SLOTS of them) are
    reused while earlier batches are still queued, as on the GPU's streams."""

    def __init__(self):
        super().__init__()
        import queue
        import threading
        self.q = queue.Queue()
        self.go = threading.Event()
        self.err = []
        self.t = threading.Thread(target=self._run, daemon=True)
        self.t.start()

    def _run(self):
        self.go.wait()
        while True:
            fn = self.q.get()
            if fn is None:
                return
            try:
                fn()
            except Exception as e:   # surfaced by wait()
                self.err.append(e)

    def empty_partials(self, world):
        from consensus_overlord_amd.shard import BATCH_SLOTS
        return torch.zeros((BATCH_SLOTS, world, 864), dtype=torch.uint8)

    def enqueue(self, fn):
        self.q.put(fn)

    def partial(self, sigs, hashes, pks, codes, out_row, index_base):
        self.enqueue(lambda: OracleBackend.partial(self, sigs, hashes, pks, codes, out_row, index_base))

    def combine_async(self, parts, n, codes):
        self.enqueue(lambda: OracleBackend.combine_async(self, parts, n, codes))

    def wait(self):
        self.go.set()
        self.q.put(None)
        self.t.join()
        assert not self.err, self.err


def _async_worker(rank, world, port, golden, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    be = AsyncOracleBackend()
    sv = ShardVerifier(be)
    out = []
    batches = _batches(golden) * 2          # six batches through three partial rows
    for s, (sg, hs, pk) in enumerate(batches):
        lo, hi = shard_bounds(len(sg), world, rank)
        codes = torch.full((hi - lo,), -1, dtype=torch.int32)
        sv.submit(s, torch.from_numpy(sg[lo:hi].copy()), torch.from_numpy(hs[lo:hi].copy()),
                  torch.from_numpy(pk[lo:hi].copy()), codes, index_base=lo)
        out.append(codes)
    deferred = all(int(c.min()) == -1 and int(c.max()) == -1 for c in out) and be.verdicts == []
    sv.wait()
    got = [None] * world
    dist.all_gather_object(got, ([c.tolist() for c in out], be.verdicts, deferred))
    if rank == 0:
        q.put(got)
    dist.destroy_process_group()


def test_two_rank_gloo_shards_async_pipeline(golden):
    """shard.py's pipelining at world 2: every batch is submitted before any work runs (codes
    deferred until wait()), the gathers run in stream order, and six batches reuse the three
    partial rows; codes and combined verdicts equal the single-process results."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_async_worker, args=(r, world, port, golden, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0][2] and got[1][2], "codes were written before wait()"
    for s, (sg, hs, pk) in enumerate(_batches(golden) * 2):
        want = orc.verify_many(sg, hs, pk)
        codes = np.concatenate([np.array(got[r][0][s], dtype=np.int32) for r in range(world)])
        assert codes.tolist() == want.tolist(), s
        _, ref_ok = orc.verify_batch_rlc(sg, hs, pk, seed=0xC17A + s)
        assert got[0][1][s] == got[1][1][s] == ref_ok == (s % 3 != 1)
