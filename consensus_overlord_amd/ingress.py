"""Vote-batching ingress at `proc_network_msg` (src/consensus.rs:210-258).

The reference decodes each network message and hands it to overlord at once (consensus.rs:
212-256); overlord then calls `Crypto::verify_signature` once per `SignedVote` / `SignedChoke`,
serially (consensus.rs:397-416 -- one device check of one vote each on this backend). This
module sits between the two: it decodes the messages, holds the signed votes and chokes of a
(height, round, kind) group for a short while, verifies everything it holds as ONE device
batch (`ConsensusCrypto.prefetch` -> `ovh_prefetch`: RLC batch check + exact per-vote codes
into the library's verdict cache), and only then forwards the messages to overlord, in arrival
order. overlord's serial `verify_signature` calls on those messages are answered from the cache
with the exact per-vote code (hits are counted by `ovh_cache_stats`).

Flush policy: a group that reaches `batch_size` messages flushes everything pending. The
default is what one round can bring over the network: the validator count minus one when this
node is a validator (its own vote never crosses the network -- overlord hands it to itself,
consensus.rs:721-771), else the validator count. A deadline flushes the rest: every arrival
checks it, and `poll()` -- to be driven by a timer (the node's tokio interval) -- flushes a
group that stopped growing (offline validators) once its oldest message has waited
`max_delay_s`. `AggregatedVote` and `SignedProposal` are not batched (one aggregated check per
QC / one proposal per round); they first flush what is held, so overlord sees every message in
arrival order, as the reference's proc_network_msg forwards them. A message that does not
decode is dropped with a warning, as the reference does.

Wire layouts [dep: overlord 0.4 types + rlp 0.5, not vendored; named assumption 7 in DESIGN.md]:
  SignedVote   = rlp([signature bytes, Vote, voter bytes])
  Vote         = rlp([height u64, round u64, vote_type u8, block_hash bytes])  (vote.rlp_vote)
  SignedChoke  = rlp([signature bytes, Choke, address bytes])
  Choke        = rlp([height u64, round u64, UpdateFrom])
  UpdateFrom   = rlp([kind u8, qc])   (PrevoteQC 0 / PrecommitQC 1: AggregatedVote, ChokeQC 2)
The signed bytes: hash(rlp(Vote)) for a vote, hash(rlp([height, round])) (overlord HashChoke)
for a choke; `hash` is Crypto::hash (SM3, util.rs:83-87).
"""
from __future__ import annotations

import logging
import time
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Tuple

from . import vote as _v

log = logging.getLogger(__name__)

SIGNED_VOTE = "SignedVote"
AGGREGATED_VOTE = "AggregatedVote"
SIGNED_PROPOSAL = "SignedProposal"
SIGNED_CHOKE = "SignedChoke"
CHOKE_KIND = 2          # group key kind of a choke (vote kinds are PREVOTE 0 / PRECOMMIT 1)


@dataclass(frozen=True)
class SignedVote:
    signature: bytes
    height: int
    round: int
    vote_type: int
    block_hash: bytes
    voter: bytes

    def vote_rlp(self) -> bytes:
        return _v.rlp_vote(self.height, self.round, self.vote_type, self.block_hash)


@dataclass(frozen=True)
class SignedChoke:
    signature: bytes
    height: int
    round: int
    update_from: bytes      # the UpdateFrom item, re-encoded RLP (not needed for the signed hash)
    address: bytes

    def hash_rlp(self) -> bytes:
        """overlord HashChoke {height, round}: the bytes a choke signs (through hash)."""
        return _v._rlp_list([_v._rlp_uint(self.height), _v._rlp_uint(self.round)])


def _bytes(x) -> bytes:
    if isinstance(x, list):
        raise ValueError("expected an RLP string")
    return x


def _u8(x) -> int:
    v = _v._uint(_bytes(x))
    if v > 0xFF:
        raise ValueError("bad u8")
    return v


def _reencode(item) -> bytes:
    if isinstance(item, list):
        return _v._rlp_list([_reencode(x) for x in item])
    return _v._rlp_bytes(item)


def encode_signed_vote(sv: SignedVote) -> bytes:
    return _v._rlp_list([_v._rlp_bytes(sv.signature), sv.vote_rlp(), _v._rlp_bytes(sv.voter)])


def decode_signed_vote(b: bytes) -> SignedVote:
    """`SignedVote::decode` (consensus.rs:212); ValueError when it would fail."""
    it = _v.rlp_decode(b)
    if not isinstance(it, list) or len(it) != 3 or not isinstance(it[1], list) or len(it[1]) != 4:
        raise ValueError("not a SignedVote")
    sig, (h, r, t, bh), voter = it
    vt = _u8(t)
    if vt not in (_v.PREVOTE, _v.PRECOMMIT):
        raise ValueError("bad vote type")
    return SignedVote(_bytes(sig), _v._uint(_bytes(h)), _v._uint(_bytes(r)), vt, _bytes(bh), _bytes(voter))


def encode_signed_choke(sc: SignedChoke) -> bytes:
    choke = _v._rlp_list([_v._rlp_uint(sc.height), _v._rlp_uint(sc.round), sc.update_from])
    return _v._rlp_list([_v._rlp_bytes(sc.signature), choke, _v._rlp_bytes(sc.address)])


def decode_signed_choke(b: bytes) -> SignedChoke:
    """`SignedChoke::decode` (consensus.rs:247); ValueError when it would fail."""
    it = _v.rlp_decode(b)
    if not isinstance(it, list) or len(it) != 3 or not isinstance(it[1], list) or len(it[1]) != 3:
        raise ValueError("not a SignedChoke")
    sig, (h, r, frm), addr = it
    if not isinstance(frm, list) or len(frm) != 2 or _u8(frm[0]) > 2:
        raise ValueError("bad UpdateFrom")
    return SignedChoke(_bytes(sig), _v._uint(_bytes(h)), _v._uint(_bytes(r)), _reencode(frm), _bytes(addr))


@dataclass
class _Pending:
    kind: str
    msg: object
    signature: bytes
    voter: bytes
    t: float


class VoteIngress:
    """proc_network_msg with vote batching. `crypto`: a ConsensusCrypto (prefetch, hash,
    vote_digests, pubkeys); `forward(kind, msg)`: hands a decoded message to overlord
    (overlord_handler.send_msg, consensus.rs:214-253)."""

    def __init__(self, crypto, forward: Callable[[str, object], None], batch_size: Optional[int] = None,
                 max_delay_s: float = 0.002, clock: Callable[[], float] = time.monotonic):
        self.crypto = crypto
        self.forward = forward
        self.batch_size = batch_size
        self.max_delay_s = max_delay_s
        self.clock = clock
        self.pending: List[_Pending] = []
        self.groups: Dict[Tuple[int, int, int], int] = {}
        self.stats = {"batches": 0, "prefetched": 0, "forwarded": 0, "dropped": 0, "unbatched": 0}

    def _limit(self) -> int:
        if self.batch_size:
            return self.batch_size
        pks = list(getattr(self.crypto, "pubkeys", []) or [])
        if not pks:
            return 256
        own = getattr(self.crypto, "name", None)
        return max(1, len(pks) - (1 if own is not None and own in pks else 0))

    def proc_network_msg(self, kind: str, payload: bytes) -> None:
        """consensus.rs:210-258 (msg.r#type, msg.msg)."""
        self.poll()   # the deadline of what is already held
        try:
            if kind == SIGNED_VOTE:
                m = decode_signed_vote(payload)
                self._hold(kind, m, (m.height, m.round, m.vote_type), m.signature, m.voter)
                return
            if kind == SIGNED_CHOKE:
                m = decode_signed_choke(payload)
                self._hold(kind, m, (m.height, m.round, CHOKE_KIND), m.signature, m.address)
                return
            if kind == AGGREGATED_VOTE or kind == SIGNED_PROPOSAL:
                self.flush()                # what arrived before goes first (arrival order)
                self._send(kind, payload)   # decoded by overlord's own types in the node
                return
        except ValueError as e:
            log.warning("decode %s failed: %s", kind, e)
            self.stats["dropped"] += 1
            return
        log.warning("unexpected network msg %r", kind)
        self.stats["dropped"] += 1

    def _hold(self, kind, m, key, sig, voter) -> None:
        self.pending.append(_Pending(kind, m, sig, voter, self.clock()))
        self.groups[key] = self.groups.get(key, 0) + 1
        if self.groups[key] >= self._limit():
            self.flush()

    def poll(self) -> None:
        """Flush when the oldest pending message has waited max_delay_s (call from a timer)."""
        if self.pending and self.clock() - self.pending[0].t >= self.max_delay_s:
            self.flush()

    def _hashes(self, items: List[_Pending]) -> List[bytes]:
        out: List[Optional[bytes]] = [None] * len(items)
        votes = [(i, p.msg) for i, p in enumerate(items) if p.kind == SIGNED_VOTE and len(p.msg.block_hash) <= 64]
        if votes and hasattr(self.crypto, "vote_digests"):
            # rlp(Vote) + SM3 of the whole batch on the device (ovh_vote_digests)
            ds = self.crypto.vote_digests([(m.height, m.round, m.vote_type, m.block_hash) for _, m in votes])
            for (i, _), d in zip(votes, ds):
                out[i] = d
        for i, p in enumerate(items):
            if out[i] is None:
                out[i] = self.crypto.hash(p.msg.vote_rlp() if p.kind == SIGNED_VOTE else p.msg.hash_rlp())
        return out

    def flush(self) -> None:
        """Batch-verify every held message (one prefetch), then forward them in arrival order."""
        items, self.pending, self.groups = self.pending, [], {}
        if not items:
            return
        hs = self._hashes(items)
        fixed = [k for k, p in enumerate(items) if len(p.signature) == 96 and len(p.voter) == 48 and len(hs[k]) == 32]
        # other encodings go to overlord as they are: its verify_signature takes the exact
        # per-call path (a cache miss)
        self.stats["unbatched"] += len(items) - len(fixed)
        if fixed:
            self.crypto.prefetch([items[k].signature for k in fixed], [hs[k] for k in fixed],
                                 [items[k].voter for k in fixed])
            self.stats["batches"] += 1
            self.stats["prefetched"] += len(fixed)
        for p in items:
            self._send(p.kind, p.msg)

    def _send(self, kind, msg) -> None:
        self.stats["forwarded"] += 1
        self.forward(kind, msg)


def overlord_verify(crypto, kind: str, msg) -> None:
    """What overlord does with a forwarded SignedVote / SignedChoke: one Crypto::verify_signature
    on hash(rlp(...)) (the call the verdict cache answers). Raises the ConsensusError."""
    if kind == SIGNED_VOTE:
        crypto.verify_signature(msg.signature, crypto.hash(msg.vote_rlp()), msg.voter)
    elif kind == SIGNED_CHOKE:
        crypto.verify_signature(msg.signature, crypto.hash(msg.hash_rlp()), msg.address)
