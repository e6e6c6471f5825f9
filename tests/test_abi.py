"""CPU checks of the boundary: libovhip.so loads and exports every entry point that
include/ovhip.h declares (no compute calls: there is no GPU here); SM3 (host code in the
product, ovh_sm3) against the GB/T 32905 vectors; host-side vote helpers."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "ovhip.h")).read()
    return sorted(set(re.findall(r"\b(ovh_[a-z0-9_]+)\s*\(", src)))


def test_header_symbols_exported():
    from consensus_overlord_amd import _lib
    lib = _lib.load()
    names = _declared()
    assert len(names) >= 17
    for n in names:
        assert hasattr(lib, n), n
    assert sorted(n for n, _, _ in _lib.SIGNATURES) == names


def test_ovh_sm3_kat():
    from consensus_overlord_amd import _lib
    lib = _lib.load()
    out = ctypes.create_string_buffer(32)
    for msg, want in ((b"abc", "66c7f0f462eeedd9d1f2d46bdc10e4e24167c4875cf2f7a2297da02b8f4ba8e0"),
                      (b"abcd" * 16, "debe9ff92275b8a138604889c18e5a4d6fdb70e5387e5765293dcba39c0c5732"),
                      (b"", "1ab21d8355cfa17f8e61194831e81a8f22bec8c728fefb747ed035eb5082aa2b"),
                      (bytes(range(200)), None)):
        assert lib.ovh_sm3(msg, len(msg), out) == 0
        if want:
            assert out.raw.hex() == want
        else:
            import hashlib
            assert out.raw == hashlib.new("sm3", msg).digest()


def test_vote_rlp_and_extract_voters():
    from consensus_overlord_amd import vote
    assert vote.rlp_vote(1, 0, vote.PRECOMMIT, bytes.fromhex(
        "1ab21d8355cfa17f8e61194831e81a8f22bec8c728fefb747ed035eb5082aa2b")).hex() == (
        "e4018001a01ab21d8355cfa17f8e61194831e81a8f22bec8c728fefb747ed035eb5082aa2b")
    auth = [bytes([i]) * 48 for i in (5, 1, 3, 2)]
    assert vote.extract_voters(auth, bytes([0b10100000])) == [bytes([1]) * 48, bytes([3]) * 48]


def test_no_cpu_fallback_when_library_missing(monkeypatch, tmp_path):
    from consensus_overlord_amd import _lib
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(RuntimeError):
        _lib.load()


def test_batch_slots_mirrored_in_shard():
    """shard.py's partial rows (one per batch in flight) follow include/ovhip.h OVH_BATCH_SLOTS."""
    from consensus_overlord_amd.shard import BATCH_SLOTS
    src = open(os.path.join(ROOT, "include", "ovhip.h")).read()
    assert int(re.search(r"#define OVH_BATCH_SLOTS (\d+)", src).group(1)) == BATCH_SLOTS
