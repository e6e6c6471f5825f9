"""Multi-GPU batch verification: one process per GPU, each rank verifies its
own shard of votes -- weak scaling, the votes are independent units -- and the only data
exchange per batch is an all-gather of the 864-byte per-shard partials (Fp12 Miller product +
projective G2 sum, include/ovhip.h OVH_PARTIAL_BYTES): RCCL over xGMI between GPUs, gloo on
CPU. Every rank then runs the same combined check on the gathered partials and, only if it
fails, the per-vote fallback of its own shard, so each rank ends with the exact per-vote codes
of its votes (ConsensusCrypto::verify_signature, src/consensus.rs:397-416, vote by vote).

Batches are pipelined: batch s's combined check / bisection is enqueued on the backend's second
stream and overlaps batch s + 1's per-vote stages; `wait()` completes everything submitted.
The device backend is stream-ordered with torch's current stream (the stream the RCCL
all-gather is ordered on): the partial is written after the stream's earlier work (the previous
gather out of the same buffer) and the stream waits for it; the combined check starts after the
gather and the stream waits until the gathered partials were read (include/ovhip.h).

RLC coefficients: every rank's library context draws its own secret seed per batch (getrandom),
so the coefficients of different ranks are independent; a backend with explicit test seeds uses
one global vote index (index_base = the rank's shard offset), never a per-rank seed variant.

The backend supplies the compute (DeviceBackend = libovhip on this rank's GPU; the CPU tests
plug in the C oracle); this module is the orchestration both share.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

PARTIAL_BYTES = 864
BATCH_SLOTS = 6      # include/ovhip.h OVH_BATCH_SLOTS: batches in flight per context


class DeviceBackend:
    """libovhip on the current GPU (consensus_overlord_amd.device)."""

    def __init__(self, ctx):
        from . import device
        self.ctx = ctx
        self.dev = device
        # the gather's stream: a stream of its own, never torch's default (null) stream, whose
        # handle 0 would ask libovhip for the synchronous partial (include/ovhip.h) and put the
        # fold levels, the MSM and the packing back in line with the vote kernels
        self.stream = torch.cuda.Stream()

    def empty_partials(self, world: int) -> torch.Tensor:
        return torch.empty((BATCH_SLOTS, world, PARTIAL_BYTES), dtype=torch.uint8, device="cuda")

    def inputs_ready(self, producer) -> None:
        """The library reads a batch's inputs in its own stream's order (ovh_stream,
        include/ovhip.h): that stream waits for the producer stream's work so far -- not the
        gather stream, which also carries the previous batch's combine."""
        lib_stream = torch.cuda.ExternalStream(self.ctx.stream)
        lib_stream.wait_stream(producer)

    def partial(self, sigs, hashes, pks, codes, out_row, index_base: int) -> None:
        self.dev.batch_partial(self.ctx, sigs, hashes, pks, codes, out_row, stream=self.stream)

    def combine_async(self, parts, n: int, codes) -> None:
        self.dev.combine_partials_async(self.ctx, parts, n, codes, stream=self.stream)

    def wait(self) -> None:
        self.dev.batch_wait(self.ctx)


class ShardVerifier:
    """Per-rank driver: submit(s, ...) verifies this rank's shard of batch s."""

    def __init__(self, backend, group=None):
        self.backend = backend
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.nccl = dist.get_backend(group) == "nccl"
        self.partials = backend.empty_partials(self.world)   # one per batch in flight (pipelining)
        self._inflight = []

    def _all_gather(self, part: torch.Tensor) -> None:
        mine = part[self.rank].clone()
        if self.nccl:
            dist.all_gather_into_tensor(part, mine, group=self.group)
        else:
            dist.all_gather(list(part.unbind(0)), mine, group=self.group)

    def submit(self, s: int, sigs, hashes, pks, codes, index_base: int = 0) -> None:
        """Enqueue batch s: this rank's n votes (global indices index_base ..) -> partial ->
        all-gather -> combined check and (device-gated) bisection into `codes`, final after
        wait()."""
        part = self.partials[s % self.partials.shape[0]]
        st = getattr(self.backend, "stream", None)
        # the library's streams read the inputs and write `codes` after this call returns: the
        # tensors stay referenced until wait(), so the caching allocator cannot hand them out
        self._inflight.append((sigs, hashes, pks, codes))
        if st is not None:
            cur = torch.cuda.current_stream()
            self.backend.inputs_ready(cur)                 # the caller's inputs, for the library
            st.wait_stream(cur)                            # and for the gather
            with torch.cuda.stream(st):
                self._submit(part, sigs, hashes, pks, codes, index_base)
        else:
            self._submit(part, sigs, hashes, pks, codes, index_base)

    def _submit(self, part, sigs, hashes, pks, codes, index_base):
        self.backend.partial(sigs, hashes, pks, codes, part[self.rank], index_base)
        # the gather runs in the backend's stream order: on the GPU the RCCL collective is
        # enqueued on the current (gather) stream; a host backend that defers its work to a
        # stream of its own (the CPU tests' asynchronous oracle) takes the gather as a task
        enqueue = getattr(self.backend, "enqueue", None)
        if enqueue is not None:
            enqueue(lambda: self._all_gather(part))
        else:
            self._all_gather(part)
        self.backend.combine_async(part, sigs.shape[0], codes)

    def wait(self) -> None:
        self.backend.wait()
        self._inflight.clear()


def shard_bounds(n_total: int, world: int, rank: int):
    """Contiguous shard [lo, hi) of rank `rank` when n_total votes are split over `world` ranks."""
    base, extra = divmod(n_total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)
