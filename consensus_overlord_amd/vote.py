"""overlord 0.4 `Vote` RLP encoding (the bytes `Consensus::check_block` hashes,
src/consensus.rs:169-175) and the bitmap -> voters expansion of `extract_voters`
(consensus.rs:167). Host logic; no crypto."""
from __future__ import annotations

from typing import List, Sequence

PREVOTE = 0
PRECOMMIT = 1


def _rlp_bytes(b: bytes) -> bytes:
    if len(b) == 1 and b[0] < 0x80:
        return b
    if len(b) < 56:
        return bytes([0x80 + len(b)]) + b
    ln = len(b).to_bytes((len(b).bit_length() + 7) // 8, "big")
    return bytes([0xB7 + len(ln)]) + ln + b


def _rlp_uint(v: int) -> bytes:
    return b"\x80" if v == 0 else _rlp_bytes(v.to_bytes((v.bit_length() + 7) // 8, "big"))


def rlp_vote(height: int, round_: int, vote_type: int, block_hash: bytes) -> bytes:
    items = [_rlp_uint(height), _rlp_uint(round_), _rlp_uint(vote_type), _rlp_bytes(bytes(block_hash))]
    payload = b"".join(items)
    if len(payload) < 56:
        return bytes([0xC0 + len(payload)]) + payload
    ln = len(payload).to_bytes((len(payload).bit_length() + 7) // 8, "big")
    return bytes([0xF7 + len(ln)]) + ln + payload


def vote_hash(crypto, height: int, round_: int, vote_type: int, block_hash: bytes) -> bytes:
    """Crypto::hash(rlp(Vote)) through a ConsensusCrypto-like object."""
    return crypto.hash(rlp_vote(height, round_, vote_type, block_hash))


def extract_voters(authority_addresses: Sequence[bytes], bitmap: bytes) -> List[bytes]:
    """overlord::extract_voters: authority list sorted by address, zipped with the
    MSB-first bit vector (overlord 0.4 [dep])."""
    auth = sorted(bytes(a) for a in authority_addresses)
    out = []
    for i, a in enumerate(auth):
        byte, bit = divmod(i, 8)
        if byte < len(bitmap) and (bitmap[byte] >> (7 - bit)) & 1:
            out.append(a)
    return out
