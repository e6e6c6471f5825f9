"""Vote digests, SURVEY.md 8(f) row 4: SM3(rlp(Vote{height, round, vote_type, block_hash})),
the hash overlord signs and Consensus::check_block rebuilds (consensus.rs:169-175 ->
util.rs:83-87). The device code (csrc/rlp.hpp + sm3.hpp, kernel k_vote_digest) against the host
RLP of consensus_overlord_amd/vote.py and hashlib's SM3, on edge cases of the RLP rules (zero,
single bytes < 0x80, u64 max, empty / one-byte / 55- / 56- / 64-byte block hashes) and seeded
random votes; the SURVEY Appendix B example is the pinned fixture (illustrative, [dep] overlord
0.4 field order)."""
import ctypes
import hashlib
import random

import pytest

from consensus_overlord_amd import vote
from test_host_harness import hx  # noqa: F401  (module fixture: builds libhx.so)

APPX_B = (1, 0, vote.PRECOMMIT, bytes.fromhex("1ab21d8355cfa17f8e61194831e81a8f22bec8c728fefb747ed035eb5082aa2b"))
APPX_B_RLP = "e4018001a01ab21d8355cfa17f8e61194831e81a8f22bec8c728fefb747ed035eb5082aa2b"
APPX_B_SM3 = "b879a90276edf81f09f6f5577740dd6e9d4a6ce799f7cedd2a7c46bd1e231325"


def edge_votes():
    rng = random.Random(0x5E3)
    out = [APPX_B]
    for h in (0, 1, 0x7F, 0x80, 0xFF, 0x100, 2 ** 32, 2 ** 64 - 1):
        for r in (0, 1, 0x80):
            out.append((h, r, vote.PREVOTE if (h + r) % 2 else vote.PRECOMMIT, bytes(32)))
    for ln in (0, 1, 2, 31, 32, 33, 54, 55, 56, 63, 64):
        out.append((7, 3, vote.PRECOMMIT, bytes(rng.randrange(256) for _ in range(ln))))
    # vote types >= 0x80 encode as two bytes (0x81 xx): the longest RLP, 88 bytes
    for t in (0x7F, 0x80, 0xFF):
        out.append((2 ** 64 - 1, 2 ** 64 - 1, t, bytes(rng.randrange(256) for _ in range(64))))
    out.append((9, 2, vote.PREVOTE, b"\x00"))
    out.append((9, 2, vote.PREVOTE, b"\x7f"))
    out.append((9, 2, vote.PREVOTE, b"\x80"))
    for _ in range(40):
        out.append((rng.getrandbits(rng.choice((8, 16, 40, 64))), rng.randrange(0, 300), rng.randrange(2),
                    bytes(rng.randrange(256) for _ in range(rng.choice((0, 1, 32, 64))))))
    return out


def want(v):
    return hashlib.new("sm3", vote.rlp_vote(*v)).digest()


def test_appendix_b_fixture():
    assert vote.rlp_vote(*APPX_B).hex() == APPX_B_RLP
    assert want(APPX_B).hex() == APPX_B_SM3


def test_host_build_of_device_rlp_and_sm3(hx):  # noqa: F811
    hx.hx_vote_rlp.restype = ctypes.c_int
    hx.hx_vote_rlp.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint8, ctypes.c_char_p,
                               ctypes.c_uint32]
    hx.hx_vote_digest.argtypes = hx.hx_vote_rlp.argtypes
    for v in edge_votes():
        buf = ctypes.create_string_buffer(96)
        n = hx.hx_vote_rlp(buf, v[0], v[1], v[2], v[3], len(v[3]))
        assert buf.raw[:n] == vote.rlp_vote(*v), v
        d = ctypes.create_string_buffer(32)
        hx.hx_vote_digest(d, v[0], v[1], v[2], v[3], len(v[3]))
        assert d.raw == want(v), v


@pytest.mark.gpu
def test_device_vote_digests():
    import consensus_overlord_amd as coa
    cc = coa.ConsensusCrypto(bytes(31) + b"\x07")
    votes = edge_votes()
    assert cc.vote_digests(votes) == [want(v) for v in votes]
    assert cc.vote_digests([APPX_B])[0].hex() == APPX_B_SM3


@pytest.mark.gpu
def test_device_vote_digest_rejects_overlong_hash():
    """ovh_vote_digests_device reads the lengths from device memory: a length above 64 gets the
    all-zero digest instead of overrunning the kernel's 64-byte hash buffer."""
    import torch
    import consensus_overlord_amd as coa
    from consensus_overlord_amd.crypto import Context
    ctx = Context(0)
    votes = [(5, 1, vote.PRECOMMIT, bytes(range(64))), (5, 1, vote.PRECOMMIT, bytes(range(64))), APPX_B]
    lens = [64, 200, len(APPX_B[3])]
    n = len(votes)
    h = torch.tensor([v[0] for v in votes], dtype=torch.int64).cuda()
    r = torch.tensor([v[1] for v in votes], dtype=torch.int64).cuda()
    t = torch.tensor([v[2] for v in votes], dtype=torch.uint8).cuda()
    bh = torch.zeros((n, 64), dtype=torch.uint8)
    for i, v in enumerate(votes):
        bh[i, :len(v[3])] = torch.tensor(list(v[3]), dtype=torch.uint8)
    bh = bh.cuda()
    ln = torch.tensor(lens, dtype=torch.uint8).cuda()
    out = torch.full((n, 32), 0xAA, dtype=torch.uint8).cuda()
    p = lambda x: ctypes.c_void_p(x.data_ptr())   # noqa: E731
    coa.crypto.raise_for(ctx.lib.ovh_vote_digests_device(ctx.ptr, n, p(h), p(r), p(t), p(bh), p(ln), p(out)))
    torch.cuda.synchronize()
    got = [bytes(out[i].cpu().numpy()) for i in range(n)]
    assert got[0] == want(votes[0])
    assert got[1] == bytes(32)
    assert got[2].hex() == APPX_B_SM3
    ctx.close()
