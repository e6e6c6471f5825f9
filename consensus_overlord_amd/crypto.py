"""Host-side mirror of the reference's `ConsensusCrypto` (src/consensus.rs:334-463) over the
libovhip C ABI: same method names, argument meaning and error behaviour. Every method runs
its arithmetic in HIP kernels on the context's MI355X (hash/SM3 runs on the host, as in the
reference, util.rs:83-87).

Errors mirror `ConsensusError` (src/error.rs:20-44): `Other(String)` for the hash-length,
length-mismatch and "lose public key" cases, `CryptoErr(code)` for blst errors.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence

import numpy as np

from . import _lib

OK = 0
ERR_HASH_LEN = 100
ERR_LEN_MISMATCH = 101
ERR_PUBKEY = 102
ERR_ARG = 103
ERR_DEVICE = 200
ERR_RNG = 201

# include/ovhip.h context flags
FLAG_AGG_NO_GROUPCHECK = 0x1
FLAG_PROFILE = 0x2
FLAG_VM_TRACE = 0x4
FLAG_TEST_RLC = 0x8     # tests only: predictable batch coefficients (Context.set_test_rlc)
FLAG_SK_RAW = 0x10      # private key = raw scalar 0 < sk < r instead of IETF KeyGen
FLAG_VM_CLOCK = 0x20    # diagnostics: clock stamps around every vote workgroup (pool log)
FLAG_POOL_RESERVE = 0x40  # the vote pool leaves 8 CUs to the caller's collective (shard contexts)

BLST_ERRORS = {
    1: "BLST_BAD_ENCODING",
    2: "BLST_POINT_NOT_ON_CURVE",
    3: "BLST_POINT_NOT_IN_GROUP",
    4: "BLST_AGGR_TYPE_MISMATCH",
    5: "BLST_VERIFY_FAIL",
    6: "BLST_PK_IS_INFINITY",
    7: "BLST_BAD_SCALAR",
}


class ConsensusError(Exception):
    """src/error.rs:20 ConsensusError."""


class Other(ConsensusError):
    """ConsensusError::Other(String)."""


class CryptoErr(ConsensusError):
    """ConsensusError::CryptoErr(Box<ophelia::Error>)."""

    def __init__(self, code: int):
        super().__init__("Crypto error %s" % BLST_ERRORS.get(code, code))
        self.code = code


class DeviceError(ConsensusError):
    pass


def raise_for(code: int) -> None:
    if code == OK:
        return
    if code == ERR_HASH_LEN:
        raise Other("failed to convert hash value")
    if code == ERR_LEN_MISMATCH:
        raise Other("signatures length does not match voters length")
    if code == ERR_PUBKEY:
        raise Other("lose public key")
    if 1 <= code <= 7:
        raise CryptoErr(code)
    if code == ERR_ARG:
        raise ValueError("invalid argument")
    raise DeviceError("libovhip device error (code %d)" % code)


def _concat(items: Sequence[bytes]):
    items = [bytes(x) for x in items]
    lens = (ctypes.c_size_t * max(1, len(items)))(*[len(x) for x in items])
    return b"".join(items), lens


class Context:
    """One libovhip context (device memory, streams, DST) on HIP device `device`, or over
    several devices of this process (`devices=[...]`, ovh_create_multi)."""

    def __init__(self, device: int = 0, dst: Optional[bytes] = None, flags: int = 0,
                 devices: Optional[Sequence[int]] = None):
        self.lib = _lib.load()
        d = None if dst is None else bytes(dst)
        if devices:
            arr = (ctypes.c_int * len(devices))(*devices)
            self.ptr = self.lib.ovh_create_multi(arr, len(devices), d, 0 if d is None else len(d), flags)
            device = devices[0]
        else:
            self.ptr = self.lib.ovh_create(device, d, 0 if d is None else len(d), flags)
        if not self.ptr:
            raise DeviceError("ovh_create failed on device %d (no usable MI355X?)" % device)
        self.device = device
        self.flags = flags

    @property
    def device_count(self) -> int:
        return self.lib.ovh_device_count(self.ptr)

    def peer_matrix(self):
        """ovh_multi_peer_matrix: n x n rows, [a][b] True when device a reaches b's memory
        directly (xGMI peer access) or a and b are one device."""
        buf = ctypes.create_string_buffer(64)
        n = self.lib.ovh_multi_peer_matrix(self.ptr, buf, 64)
        raise_for(n if n < 0 else 0)
        return [[bool(buf.raw[a * n + b]) for b in range(n)] for a in range(n)]

    def set_test_rlc(self, seed: int, index_base: int = 0) -> None:
        """Tests only (context made with FLAG_TEST_RLC): reproducible batch coefficients."""
        raise_for(self.lib.ovh_set_test_rlc(self.ptr, seed & 0xFFFFFFFFFFFFFFFF, index_base))

    def close(self):
        if getattr(self, "ptr", None):
            self.lib.ovh_destroy(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self) -> int:
        return self.lib.ovh_stream(self.ptr)


class ConsensusCrypto:
    """Mirror of `ConsensusCrypto` / overlord's `Crypto` trait (consensus.rs:339-463)."""

    def __init__(self, private_key: bytes, device: int = 0, dst: Optional[bytes] = None, ctx: Optional[Context] = None):
        """consensus.rs:347-359 `new`: the private key file's bytes (hex text or raw bytes),
        parsed as ophelia-blst's BlsPrivateKey::try_from (IETF KeyGen by default, see
        ovh_sk_parse); name = the 48-byte compressed public key; common_ref = ''."""
        if isinstance(private_key, str):
            private_key = bytes.fromhex(private_key.strip())
        self.ctx = ctx if ctx is not None else Context(device, dst)
        self.lib = self.ctx.lib
        self.private_key = bytes(private_key)
        self.common_ref = ""
        out = ctypes.create_string_buffer(48)
        raise_for(self.lib.ovh_sk_to_pk(self.ctx.ptr, self.private_key, len(self.private_key), out))
        self.name = out.raw
        self.pubkeys: List[bytes] = []

    @classmethod
    def from_key_file(cls, path: str, **kw) -> "ConsensusCrypto":
        with open(path) as fh:
            return cls(bytes.fromhex(fh.read().strip()), **kw)

    def update_pubkeys(self, new_pubkeys: Sequence[bytes]) -> None:
        """consensus.rs:361-363 (callers :131-136, :622-629): the validator keys, 48-byte
        compressed, in config order -> the device validator table (ovh_set_validators)."""
        keys = [bytes(p) for p in new_pubkeys]
        if any(len(k) != 48 for k in keys):
            raise Other("lose public key")
        self.pubkeys = keys
        raise_for(self.lib.ovh_set_validators(self.ctx.ptr, b"".join(keys), len(keys)))

    def scalar(self) -> bytes:
        """The 32-byte scalar the private key parses to (ovh_sk_parse)."""
        out = ctypes.create_string_buffer(32)
        raise_for(self.lib.ovh_sk_parse(self.ctx.ptr, self.private_key, len(self.private_key), out))
        return out.raw

    # ---- overlord::Crypto ----
    def hash(self, msg: bytes) -> bytes:
        """consensus.rs:386-388 -> util.rs:83-87 (SM3)."""
        msg = bytes(msg)
        out = ctypes.create_string_buffer(32)
        raise_for(self.lib.ovh_sm3(msg, len(msg), out))
        return out.raw

    def sign(self, hash_: bytes) -> bytes:
        """consensus.rs:390-395."""
        hash_ = bytes(hash_)
        out = ctypes.create_string_buffer(96)
        raise_for(self.lib.ovh_sign(self.ctx.ptr, self.private_key, len(self.private_key), hash_, len(hash_), out))
        return out.raw

    def verify_signature(self, signature: bytes, hash_: bytes, voter: bytes) -> None:
        """consensus.rs:397-416."""
        s, h, v = bytes(signature), bytes(hash_), bytes(voter)
        raise_for(self.lib.ovh_verify(self.ctx.ptr, s, len(s), h, len(h), v, len(v)))

    def aggregate_signatures(self, signatures: Sequence[bytes], voters: Sequence[bytes]) -> bytes:
        """consensus.rs:418-444."""
        sd, sl = _concat(signatures)
        vd, vl = _concat(voters)
        out = ctypes.create_string_buffer(96)
        raise_for(self.lib.ovh_aggregate_sigs(self.ctx.ptr, sd, sl, len(signatures), vd, vl, len(voters), out))
        return out.raw

    def verify_aggregated_signature(self, aggregated_signature: bytes, hash_: bytes, voters: Sequence[bytes]) -> None:
        """consensus.rs:446-462."""
        a, h = bytes(aggregated_signature), bytes(hash_)
        vd, vl = _concat(voters)
        raise_for(self.lib.ovh_verify_aggregated(self.ctx.ptr, a, len(a), h, len(h), vd, vl, len(voters)))

    # ---- extensions ----
    def vote_digests(self, votes) -> List[bytes]:
        """hash(rlp(Vote)) of many votes on the device (ovh_vote_digests: overlord Vote RLP +
        SM3, consensus.rs:169-175, util.rs:83-87). votes: (height, round, vote_type,
        block_hash) tuples, block_hash <= 64 bytes (empty for a nil vote)."""
        n = len(votes)
        if n == 0:
            return []
        h = np.array([v[0] for v in votes], dtype=np.uint64)
        r = np.array([v[1] for v in votes], dtype=np.uint64)
        t = np.array([v[2] for v in votes], dtype=np.uint8)
        lens = np.array([len(v[3]) for v in votes], dtype=np.uint8)
        if any(len(v[3]) > 64 for v in votes):
            raise ValueError("block hashes of up to 64 bytes")
        bh = np.zeros((n, 64), dtype=np.uint8)
        for i, v in enumerate(votes):
            bh[i, :len(v[3])] = np.frombuffer(bytes(v[3]), dtype=np.uint8)
        out = np.zeros((n, 32), dtype=np.uint8)
        ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)   # noqa: E731
        raise_for(self.lib.ovh_vote_digests(self.ctx.ptr, n, ptr(h), ptr(r), ptr(t), ptr(bh), ptr(lens), ptr(out)))
        return [out[i].tobytes() for i in range(n)]

    def aggregate_public_keys(self, voters: Sequence[bytes]) -> bytes:
        """BlsPublicKey::aggregate (consensus.rs:371) -> 48-byte compressed."""
        vd, vl = _concat(voters)
        out = ctypes.create_string_buffer(48)
        raise_for(self.lib.ovh_aggregate_pks(self.ctx.ptr, vd, vl, len(voters), out))
        return out.raw

    @staticmethod
    def _fixed(signatures, hashes, voters):
        n = len(signatures)
        if not (len(hashes) == len(voters) == n):
            raise ValueError("batch lists must have equal length")
        sig = b"".join(bytes(s) for s in signatures)
        hs = b"".join(bytes(h) for h in hashes)
        pk = b"".join(bytes(v) for v in voters)
        if len(sig) != 96 * n or len(hs) != 32 * n or len(pk) != 48 * n:
            raise ValueError("batches take 96-byte signatures, 32-byte hashes, 48-byte voters")
        return n, sig, hs, pk

    def verify_batch(self, signatures, hashes, voters) -> np.ndarray:
        """Batched verify_signature: returns int32 codes[n], codes[i] == the ovh_verify result
        for vote i (0 = Ok). Fixed-size inputs: 96-byte sigs, 32-byte hashes, 48-byte pks."""
        n, sig, hs, pk = self._fixed(signatures, hashes, voters)
        codes = np.zeros(max(n, 1), dtype=np.int32)
        raise_for(self.lib.ovh_verify_batch(self.ctx.ptr, n, sig, hs, pk, codes.ctypes.data_as(ctypes.c_void_p)))
        return codes[:n]

    def verify_batch_async(self, signatures, hashes, voters, codes: np.ndarray) -> None:
        """Pipelined verify_batch (ovh_verify_batch_async, any context kind): returns at once;
        `codes` (int32[n], kept alive by this object until wait) is final after wait()."""
        n, sig, hs, pk = self._fixed(signatures, hashes, voters)
        if codes.dtype != np.int32 or codes.shape != (n,) or not codes.flags.c_contiguous:
            raise ValueError("codes must be a contiguous int32[n] array")
        self._inflight = getattr(self, "_inflight", [])
        self._inflight.append(codes)
        raise_for(self.lib.ovh_verify_batch_async(self.ctx.ptr, n, sig, hs, pk, codes.ctypes.data_as(ctypes.c_void_p)))

    def wait(self) -> None:
        """ovh_batch_wait: every batch in flight is complete, its codes written."""
        raise_for(self.lib.ovh_batch_wait(self.ctx.ptr))
        self._inflight = []

    def prefetch(self, signatures, hashes, voters) -> None:
        """Vote-batching ingress (ovh_prefetch): batch-verify the votes now; later
        verify_signature calls on the same bytes are answered from the context's cache."""
        n, sig, hs, pk = self._fixed(signatures, hashes, voters)
        raise_for(self.lib.ovh_prefetch(self.ctx.ptr, n, sig, hs, pk))

    def cache_stats(self):
        """(hits, misses, entries) of the verdict cache."""
        st = (ctypes.c_uint64 * 3)()
        raise_for(self.lib.ovh_cache_stats(self.ctx.ptr, st))
        return tuple(int(x) for x in st)

    def samemsg_stats(self):
        """(batches, votes, distinct hashes) checked by the same-message path (ovh_samemsg_stats)."""
        st = (ctypes.c_uint64 * 3)()
        raise_for(self.lib.ovh_samemsg_stats(self.ctx.ptr, st))
        return tuple(int(x) for x in st)

    def verify_qc_batch(self, signatures, hashes, bitmaps) -> np.ndarray:
        """Batched QC check (ovh_verify_qc_batch): QC j signed by the validators (update_pubkeys)
        selected by bitmaps[j] over the key-sorted validator list; codes[j] equals
        verify_aggregated_signature(signatures[j], hashes[j], those voters)."""
        n = len(signatures)
        if not (len(hashes) == len(bitmaps) == n):
            raise ValueError("QC lists must have equal length")
        bl = len(bitmaps[0]) if n else 0
        if any(len(b) != bl for b in bitmaps):
            raise ValueError("bitmaps must have equal length")
        sig = b"".join(bytes(s) for s in signatures)
        hs = b"".join(bytes(h) for h in hashes)
        if len(sig) != 96 * n or len(hs) != 32 * n:
            raise ValueError("QC batches take 96-byte signatures and 32-byte hashes")
        codes = np.zeros(max(n, 1), dtype=np.int32)
        raise_for(self.lib.ovh_verify_qc_batch(self.ctx.ptr, n, sig, hs, b"".join(bytes(b) for b in bitmaps), bl,
                                               codes.ctypes.data_as(ctypes.c_void_p)))
        return codes[:n]

    # ---- Consensus::check_block (consensus.rs:143-207) over the Crypto surface ----
    def check_block(self, proposal_height: int, proposal_data: bytes, proof: bytes,
                    authority_list: Optional[Sequence[bytes]] = None) -> bool:
        """consensus.rs:143-207: sm3(proposal data) (:148); decode the overlord Proof (:158,
        layout in vote.py); proof.block_hash == that hash and proof.height == proposal height
        (:165); voters = extract_voters(authority list, bitmap) (:166-167); vote hash =
        hash(rlp(Vote{height, round, Precommit, block_hash})) (:169-175);
        verify_aggregated_signature(...).is_ok() (:176-183). authority_list: the brain's node
        addresses, i.e. the validator keys (util.rs validators_to_nodes); default = the keys
        given to update_pubkeys. Every failure returns False, as the reference does."""
        from . import vote as _vote
        auth = self.pubkeys if authority_list is None else [bytes(a) for a in authority_list]
        block_hash = self.hash(proposal_data)
        try:
            height, round_, bh, sig, bitmap = _vote.decode_proof(proof)
        except ValueError:
            return False
        if bytes(bh) != block_hash or height != proposal_height:
            return False
        voters = _vote.extract_voters(auth, bitmap)
        vh = self.hash(_vote.rlp_vote(height, round_, _vote.PRECOMMIT, bh))
        try:
            self.verify_aggregated_signature(sig, vh, voters)
        except ConsensusError:
            return False
        return True

    def check_blocks(self, blocks) -> np.ndarray:
        """Many check_block calls against the validator table (update_pubkeys) in one pass:
        blocks = (proposal_height, proposal_data, proof) tuples -> bool[n], element j ==
        check_block(*blocks[j]). Vote hashes come from ovh_vote_digests and the aggregated
        signatures are checked by ovh_verify_qc_batch (bitmaps over the key-sorted table, the
        extract_voters order), one batch per bitmap length."""
        from . import vote as _vote
        n = len(blocks)
        ok = np.zeros(n, dtype=bool)
        live = []
        for j, (ph, data, proof) in enumerate(blocks):
            try:
                height, round_, bh, sig, bitmap = _vote.decode_proof(proof)
            except ValueError:
                continue
            if bytes(bh) != self.hash(data) or height != ph:
                continue
            if len(sig) != 96 or len(bh) > 64:
                # the QC batch takes compressed signatures only; anything else goes the scalar way
                ok[j] = self.check_block(ph, data, proof)
                continue
            live.append((j, height, round_, bytes(bh), bytes(sig), bytes(bitmap)))
        if not live:
            return ok
        if not self.pubkeys:
            # no validator table (update_pubkeys never called, or given []): check_block answers
            # every block itself (empty authority list -> no voters -> False, consensus.rs:167-183)
            for j, *_ in live:
                ok[j] = self.check_block(*blocks[j])
            return ok
        digests = self.vote_digests([(h, r, _vote.PRECOMMIT, bh) for _, h, r, bh, _, _ in live])
        groups = {}
        for (j, _, _, _, sig, bm), d in zip(live, digests):
            groups.setdefault(len(bm), []).append((j, sig, d, bm))
        for items in groups.values():
            codes = self.verify_qc_batch([s for _, s, _, _ in items], [d for _, _, d, _ in items],
                                         [b for _, _, _, b in items])
            for (j, _, _, _), c in zip(items, codes):
                ok[j] = c == 0
        return ok
