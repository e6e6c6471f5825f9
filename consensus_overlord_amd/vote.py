"""overlord 0.4 `Vote` RLP encoding (the bytes `Consensus::check_block` hashes,
src/consensus.rs:169-175), the `Proof` RLP it decodes (consensus.rs:158) and the bitmap ->
voters expansion of `extract_voters` (consensus.rs:167). Host logic; no crypto.

Proof layout [dep: overlord 0.4, not vendored]: rlp([height u64, round u64, block_hash bytes,
rlp([signature bytes, address_bitmap bytes])]) -- AggregatedSignature nested as a two-item
list. Named assumption 6 in DESIGN.md."""
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


def rlp_decode(b: bytes):
    """RLP bytes -> nested lists of bytes (whole input must be one item)."""
    item, rest = _rlp_item(bytes(b))
    if rest:
        raise ValueError("trailing bytes after the RLP item")
    return item


def _rlp_len(b: bytes, n: int) -> int:
    if n == 0 or len(b) < n or b[0] == 0:
        raise ValueError("bad RLP length")
    return int.from_bytes(b[:n], "big")


def _rlp_item(b: bytes):
    if not b:
        raise ValueError("empty RLP")
    h = b[0]
    if h < 0x80:
        return b[:1], b[1:]
    if h < 0xB8:
        n = h - 0x80
        if len(b) < 1 + n or (n == 1 and b[1] < 0x80):
            raise ValueError("bad RLP string")
        return b[1:1 + n], b[1 + n:]
    if h < 0xC0:
        ln = h - 0xB7
        n = _rlp_len(b[1:], ln)
        if n < 56 or len(b) < 1 + ln + n:
            raise ValueError("bad RLP long string")
        return b[1 + ln:1 + ln + n], b[1 + ln + n:]
    if h < 0xF8:
        n, off = h - 0xC0, 1
    else:
        ln = h - 0xF7
        n, off = _rlp_len(b[1:], ln), 1 + ln
        if n < 56:
            raise ValueError("bad RLP long list")
    if len(b) < off + n:
        raise ValueError("truncated RLP list")
    body, out = b[off:off + n], []
    while body:
        it, body = _rlp_item(body)
        out.append(it)
    return out, b[off + n:]


def _rlp_list(items) -> bytes:
    payload = b"".join(items)
    if len(payload) < 56:
        return bytes([0xC0 + len(payload)]) + payload
    ln = len(payload).to_bytes((len(payload).bit_length() + 7) // 8, "big")
    return bytes([0xF7 + len(ln)]) + ln + payload


def _uint(b: bytes) -> int:
    if isinstance(b, list) or len(b) > 8 or (b[:1] == b"\x00"):
        raise ValueError("bad RLP u64")
    return int.from_bytes(b, "big")


def encode_proof(height: int, round_: int, block_hash: bytes, signature: bytes, bitmap: bytes) -> bytes:
    """overlord Proof -> RLP bytes (layout: module docstring)."""
    agg = _rlp_list([_rlp_bytes(bytes(signature)), _rlp_bytes(bytes(bitmap))])
    return _rlp_list([_rlp_uint(height), _rlp_uint(round_), _rlp_bytes(bytes(block_hash)), agg])


def decode_proof(b: bytes):
    """RLP bytes -> (height, round, block_hash, signature, address_bitmap); ValueError if the
    bytes are not a Proof (`Proof::decode` failing, consensus.rs:158)."""
    it = rlp_decode(b)
    if not isinstance(it, list) or len(it) != 4 or not isinstance(it[3], list) or len(it[3]) != 2:
        raise ValueError("not a Proof")
    h, r, bh, (sig, bm) = it
    if any(isinstance(x, list) for x in (bh, sig, bm)):
        raise ValueError("not a Proof")
    return _uint(h), _uint(r), bh, sig, bm
