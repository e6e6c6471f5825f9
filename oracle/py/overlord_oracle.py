"""CPU ORACLE (test infrastructure only) — the overlord `Crypto` trait semantics.

Restates `ConsensusCrypto` (src/consensus.rs:334-463) on top of `bls12_381.py`, with the
reference's error precedence, mapped to the C-ABI return codes of `include/ovhip.h`:

    0    OK
    1..7 BLST_ERROR from a signature parse / aggregate / verify -> ConsensusError::CryptoErr
    100  hash is not 32 bytes        -> Other("failed to convert hash value")  (consensus.rs:403-404, 375-376, 391-392)
    101  len(signatures) != len(voters) -> Other("signatures length does not match voters length") (:423-427)
    102  public key does not parse   -> Other("lose public key")              (:406-407, 435-436, 455-456)

Also: SM3 (`util.rs:83-87`, libsm 0.6 -> restated with OpenSSL's `hashlib.new("sm3")`), and the
overlord 0.4 `Vote` RLP encoding that `Consensus::check_block` hashes (consensus.rs:169-175).
Only tests/ and the golden-fixture script import this module.
"""
from __future__ import annotations

import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import bls12_381 as bls  # noqa: E402

OK = 0
ERR_HASH_LEN = 100
ERR_LEN_MISMATCH = 101
ERR_PUBKEY = 102

PREVOTE = 0
PRECOMMIT = 1


def sm3(data: bytes) -> bytes:
    """util.rs:83-87 sm3_hash."""
    return hashlib.new("sm3", bytes(data)).digest()


# --------------------------------------------------------------------------------------
# RLP (rlp 0.5) for overlord::types::Vote{height, round, vote_type, block_hash}
# --------------------------------------------------------------------------------------

def _rlp_bytes(b: bytes) -> bytes:
    if len(b) == 1 and b[0] < 0x80:
        return b
    if len(b) < 56:
        return bytes([0x80 + len(b)]) + b
    ln = len(b).to_bytes((len(b).bit_length() + 7) // 8, "big")
    return bytes([0xB7 + len(ln)]) + ln + b


def _rlp_uint(v: int) -> bytes:
    if v == 0:
        return b"\x80"
    return _rlp_bytes(v.to_bytes((v.bit_length() + 7) // 8, "big"))


def _rlp_list(items) -> bytes:
    payload = b"".join(items)
    if len(payload) < 56:
        return bytes([0xC0 + len(payload)]) + payload
    ln = len(payload).to_bytes((len(payload).bit_length() + 7) // 8, "big")
    return bytes([0xF7 + len(ln)]) + ln + payload


def rlp_vote(height: int, round_: int, vote_type: int, block_hash: bytes) -> bytes:
    return _rlp_list([_rlp_uint(height), _rlp_uint(round_), _rlp_uint(vote_type), _rlp_bytes(block_hash)])


def vote_hash(height: int, round_: int, vote_type: int, block_hash: bytes) -> bytes:
    """consensus.rs:169-175: Crypto::hash(rlp(Vote))."""
    return sm3(rlp_vote(height, round_, vote_type, block_hash))


# --------------------------------------------------------------------------------------
# Synthetic workload: seed 0xC17A
# --------------------------------------------------------------------------------------
SEED = 0xC17A


def synth_sk(i: int, seed: int = SEED) -> int:
    v = int.from_bytes(hashlib.sha256(seed.to_bytes(8, "big") + i.to_bytes(8, "big")).digest(), "big") % bls.R
    return v if v != 0 else 1


def synth_block_hash(i: int, seed: int = SEED) -> bytes:
    return sm3(seed.to_bytes(8, "big") + i.to_bytes(8, "big"))


def synth_vote_digest(i: int, seed: int = SEED) -> bytes:
    return vote_hash(1 + i // 64, i % 3, PRECOMMIT, synth_block_hash(i, seed))


# --------------------------------------------------------------------------------------
# ConsensusCrypto semantics
# --------------------------------------------------------------------------------------

def _parse_pk(b):
    try:
        return bls.g1_from_bytes(b), 0
    except bls.BlstError as e:
        return None, e.code


def _parse_sig(b):
    try:
        return bls.g2_from_bytes(b), 0
    except bls.BlstError as e:
        return None, e.code


def verify_signature(signature: bytes, hash_: bytes, voter: bytes, dst: bytes = bls.DST_NUL) -> int:
    """consensus.rs:397-416."""
    if len(hash_) != 32:
        return ERR_HASH_LEN
    pk, e = _parse_pk(voter)
    if e:
        return ERR_PUBKEY
    sig, e = _parse_sig(signature)
    if e:
        return e
    return bls.core_verify(pk, sig, bytes(hash_), dst)


def aggregate_signatures(signatures, voters):
    """consensus.rs:418-444 -> (code, 96-byte compressed aggregate or None)."""
    if len(signatures) != len(voters):
        return ERR_LEN_MISMATCH, None
    sigs = []
    for s, v in zip(signatures, voters):
        sig, e = _parse_sig(s)
        if e:
            return e, None
        _, e = _parse_pk(v)
        if e:
            return ERR_PUBKEY, None
        sigs.append(sig)
    try:
        agg = bls.aggregate_g2(sigs, groupcheck=True)
    except bls.BlstError as e:
        return e.code, None
    return OK, bls.g2_compress(agg)


def aggregate_public_keys(voters):
    """BlsPublicKey::aggregate as used at consensus.rs:371 -> (code, 48-byte compressed)."""
    pks = []
    for v in voters:
        pk, e = _parse_pk(v)
        if e:
            return ERR_PUBKEY, None
        pks.append(pk)
    try:
        agg = bls.aggregate_g1(pks)
    except bls.BlstError as e:
        return e.code, None
    return OK, bls.g1_compress(agg)


def verify_aggregated_signature(aggregated_signature: bytes, hash_: bytes, voters, dst: bytes = bls.DST_NUL) -> int:
    """consensus.rs:446-462 + inner_verify_aggregated_signature :365-382 (note the order:
    pk parse, aggregate (empty -> 4), sig parse, then the hash length)."""
    pks = []
    for v in voters:
        pk, e = _parse_pk(v)
        if e:
            return ERR_PUBKEY
        pks.append(pk)
    try:
        agg_pk = bls.aggregate_g1(pks)
    except bls.BlstError as e:
        return e.code
    sig, e = _parse_sig(aggregated_signature)
    if e:
        return e
    if len(hash_) != 32:
        return ERR_HASH_LEN
    return bls.core_verify(agg_pk, sig, bytes(hash_), dst)


def sign(sk: int, hash_: bytes, dst: bytes = bls.DST_NUL):
    """consensus.rs:390-395 -> (code, 96-byte compressed signature)."""
    if len(hash_) != 32:
        return ERR_HASH_LEN, None
    return OK, bls.g2_compress(bls.sign(sk, bytes(hash_), dst))
