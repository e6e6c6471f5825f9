"""Vote-batching ingress (consensus_overlord_amd/ingress.py) at proc_network_msg
(consensus.rs:210-258): overlord message codecs, the hold / flush / forward logic over an
oracle-backed Crypto (CPU), and the whole shim on the GPU: a 100-validator prevote + precommit
stream (1% sigma + G2, three voters outside the validator table, a few chokes) after which every
serial verify_signature overlord makes is a cache hit with the oracle's exact code."""
import hashlib
import random

import numpy as np
import pytest

from consensus_overlord_amd import ingress as ig
from consensus_overlord_amd import vote
from consensus_overlord_amd.crypto import ConsensusError, CryptoErr, Other


def sm3(b):
    return hashlib.new("sm3", b).digest()


def test_signed_vote_and_choke_round_trip():
    sv = ig.SignedVote(b"\x01" * 96, 2 ** 40 + 3, 7, vote.PRECOMMIT, bytes(range(32)), b"\x02" * 48)
    b = ig.encode_signed_vote(sv)
    assert ig.decode_signed_vote(b) == sv
    assert ig.decode_signed_vote(b).vote_rlp() == vote.rlp_vote(2 ** 40 + 3, 7, 1, bytes(range(32)))
    qc = vote._rlp_list([vote._rlp_uint(0), vote._rlp_list([vote._rlp_bytes(b"\x05" * 96), vote._rlp_bytes(b"\xf0")])])
    sc = ig.SignedChoke(b"\x03" * 96, 9, 0, qc, b"\x04" * 48)
    assert ig.decode_signed_choke(ig.encode_signed_choke(sc)) == sc
    assert sc.hash_rlp() == bytes([0xC2, 0x09, 0x80])


@pytest.mark.parametrize("bad", [
    b"",
    b"\xc0",
    vote.rlp_vote(1, 0, 1, bytes(32)),                              # a Vote, not a SignedVote
    ig.encode_signed_vote(ig.SignedVote(b"s", 1, 0, 1, b"h", b"v")) + b"\x00",   # trailing byte
    vote._rlp_list([vote._rlp_bytes(b"s"), vote.rlp_vote(1, 0, 5, b"h"), vote._rlp_bytes(b"v")]),  # vote type 5
    vote._rlp_list([vote._rlp_bytes(b"s"), vote._rlp_list([b"\x00\x01", b"\x80", b"\x01", b"\x80"]),
                    vote._rlp_bytes(b"v")]),                         # non-canonical height
])
def test_decode_signed_vote_rejects(bad):
    with pytest.raises(ValueError):
        ig.decode_signed_vote(bad)


class OracleCrypto:
    """The Crypto surface the shim uses, answered by the C oracle, with a verdict cache like
    ovh_prefetch's (test infrastructure)."""

    def __init__(self, pubkeys):
        self.pubkeys = list(pubkeys)
        self.cache = {}
        self.hits = self.misses = 0
        self.prefetch_calls = []

    def hash(self, m):
        return sm3(m)

    def prefetch(self, sigs, hashes, voters):
        import orc
        self.prefetch_calls.append(len(sigs))
        for s, h, v in zip(sigs, hashes, voters):
            self.cache[(bytes(s), bytes(h), bytes(v))] = orc.verify(bytes(s), bytes(h), bytes(v))

    def verify_signature(self, s, h, v):
        import orc
        k = (bytes(s), bytes(h), bytes(v))
        if k in self.cache:
            self.hits += 1
            code = self.cache[k]
        else:
            self.misses += 1
            code = orc.verify(*k)
        if code == 102:
            raise Other("lose public key")
        if code:
            raise CryptoErr(code)


def _stream(nval, height, round_, block_hash, sign, pks, bad=(), chokes=0):
    msgs = []
    for t in (vote.PREVOTE, vote.PRECOMMIT):
        d = sm3(vote.rlp_vote(height, round_, t, block_hash))
        for i in range(nval):
            msgs.append(("SignedVote", ig.SignedVote(sign(i, d), height, round_, t, block_hash, pks[i])))
    for i in range(chokes):
        frm = vote._rlp_list([vote._rlp_uint(2), vote._rlp_list([vote._rlp_bytes(b"\x00"), vote._rlp_bytes(b"")])])
        c = ig.SignedChoke(b"", height, round_, frm, pks[i])
        msgs.append(("SignedChoke", ig.SignedChoke(sign(i, sm3(c.hash_rlp())), height, round_, frm, pks[i])))
    return msgs


def test_ingress_batches_then_forwards_in_order():
    import orc
    nval = 6
    sks = [(int.from_bytes(sm3(b"ingress %d" % i), "big") >> 3).to_bytes(32, "big") for i in range(nval)]
    pks = [orc.sk_to_pk(k)[1] for k in sks]
    msgs = _stream(nval, 3, 1, sm3(b"block 3"), lambda i, d: orc.sign(sks[i], d)[1], pks, chokes=2)
    oc = OracleCrypto(pks)
    fwd = []
    now = [0.0]
    sh = ig.VoteIngress(oc, lambda k, m: fwd.append((k, m)), max_delay_s=0.01, clock=lambda: now[0])
    payloads = [(k, ig.encode_signed_vote(m) if k == "SignedVote" else ig.encode_signed_choke(m)) for k, m in msgs]
    for k, p in payloads[:nval - 1]:
        sh.proc_network_msg(k, p)
    assert fwd == [] and oc.prefetch_calls == []          # held: the prevote group is not full
    sh.proc_network_msg(*payloads[nval - 1])               # the group reaches the validator count
    assert oc.prefetch_calls == [nval] and [m for _, m in fwd] == [m for _, m in msgs[:nval]]
    for k, p in payloads[nval:]:
        sh.proc_network_msg(k, p)
    assert len(oc.prefetch_calls) == 2
    sh.proc_network_msg("SignedVote", b"\xc0")            # undecodable: dropped, as the reference
    sh.proc_network_msg("Unknown", b"")
    assert sh.stats["dropped"] == 2
    sh.poll()
    assert len(fwd) == 2 * nval                             # the two chokes wait for the deadline
    now[0] += 0.02
    sh.poll()
    assert [m for _, m in fwd] == [m for _, m in msgs]
    for k, m in fwd:
        ig.overlord_verify(oc, k, m)
    assert oc.hits == len(msgs) and oc.misses == 0


@pytest.mark.gpu
def test_ingress_stream_on_device_every_verify_is_a_cache_hit():
    import torch
    import orc
    import consensus_overlord_amd as coa
    from consensus_overlord_amd import device as dev
    import synth_votes as sv
    nval = 100
    cc = coa.ConsensusCrypto(bytes.fromhex("5a" * 32))
    sks = torch.from_numpy(sv.scalars(50000, nval)).cuda()
    pks = dev.sk_to_pk_batch(cc.ctx, sks).cpu().numpy()
    pk_list = [bytes(pks[i]) for i in range(nval)]
    cc.update_pubkeys(pk_list[3:])                          # three voters outside the table
    bh = sm3(b"block 12")
    digs = {}

    def sign(i, d):
        digs.setdefault(d, []).append(i)
        return None
    plan = _stream(nval, 12, 0, bh, sign, pk_list, chokes=4)
    # device signatures per digest
    sigs = {}
    for d, idx in digs.items():
        out = dev.sign_batch(cc.ctx, sks[idx], torch.from_numpy(np.tile(np.frombuffer(d, dtype=np.uint8),
                                                                        (len(idx), 1))).cuda())
        for k, i in enumerate(idx):
            sigs[(d, i)] = bytes(out[k].cpu().numpy())
    rng = random.Random(12)
    bad = set(rng.sample(range(len(plan)), 2))             # 1% of the 200 votes: sigma + G2
    msgs = []
    for k, (kind, m) in enumerate(plan):
        d = sm3(m.vote_rlp() if kind == "SignedVote" else m.hash_rlp())
        i = pk_list.index(m.voter if kind == "SignedVote" else m.address)
        s = sigs[(d, i)]
        if k in bad:
            s = sv.add_g2(s)
        msgs.append((kind, type(m)(s, *[getattr(m, f) for f in m.__dataclass_fields__][1:])))
    rng.shuffle(msgs)
    fwd = []
    sh = ig.VoteIngress(cc, lambda k, m: fwd.append((k, m)))
    for kind, m in msgs:
        sh.proc_network_msg(kind, ig.encode_signed_vote(m) if kind == "SignedVote" else ig.encode_signed_choke(m))
    sh.flush()
    assert sorted(map(repr, (m for _, m in fwd))) == sorted(map(repr, (m for _, m in msgs)))
    h0, m0, _ = cc.cache_stats()
    nbad = 0
    for kind, m in fwd:
        voter = m.voter if kind == "SignedVote" else m.address
        h = cc.hash(m.vote_rlp() if kind == "SignedVote" else m.hash_rlp())
        want = orc.verify(m.signature, h, voter)
        try:
            ig.overlord_verify(cc, kind, m)
            got = 0
        except CryptoErr as e:
            got = e.code
        except ConsensusError:
            got = 102
        assert got == want, (kind, m.height, m.round)
        nbad += want != 0
    h1, m1, _ = cc.cache_stats()
    assert h1 - h0 == len(fwd) and m1 == m0
    assert nbad == 2 and sh.stats["batches"] >= 1


def test_relayer_flushes_at_n_minus_one_without_the_deadline():
    """A validator never receives its own vote over the network (consensus.rs:721-771): with its
    name among the validators, a group flushes at N - 1 votes, with no deadline and no poll()."""
    import orc
    nval = 5
    sks = [(int.from_bytes(sm3(b"relayer %d" % i), "big") >> 3).to_bytes(32, "big") for i in range(nval)]
    pks = [orc.sk_to_pk(k)[1] for k in sks]
    oc = OracleCrypto(pks)
    oc.name = pks[0]                                        # this node is validator 0
    msgs = _stream(nval, 4, 0, sm3(b"block 4"), lambda i, d: orc.sign(sks[i], d)[1], pks)
    fwd = []
    sh = ig.VoteIngress(oc, lambda k, m: fwd.append((k, m)), max_delay_s=1e9, clock=lambda: 0.0)
    others = [(k, m) for k, m in msgs if m.voter != pks[0]]
    prevotes = [x for x in others if x[1].vote_type == vote.PREVOTE]
    assert len(prevotes) == nval - 1
    for k, m in prevotes[:-1]:
        sh.proc_network_msg(k, ig.encode_signed_vote(m))
    assert fwd == []
    sh.proc_network_msg(prevotes[-1][0], ig.encode_signed_vote(prevotes[-1][1]))
    assert oc.prefetch_calls == [nval - 1] and [m for _, m in fwd] == [m for _, m in prevotes]


def test_aggregated_vote_and_proposal_keep_arrival_order():
    """Held votes are forwarded before an AggregatedVote / SignedProposal that arrives after them."""
    import orc
    nval = 4
    sks = [(int.from_bytes(sm3(b"order %d" % i), "big") >> 3).to_bytes(32, "big") for i in range(nval)]
    pks = [orc.sk_to_pk(k)[1] for k in sks]
    oc = OracleCrypto(pks)
    msgs = _stream(nval, 5, 2, sm3(b"block 5"), lambda i, d: orc.sign(sks[i], d)[1], pks)
    fwd = []
    sh = ig.VoteIngress(oc, lambda k, m: fwd.append((k, m)), max_delay_s=1e9, clock=lambda: 0.0)
    for k, m in msgs[:2]:
        sh.proc_network_msg(k, ig.encode_signed_vote(m))
    assert fwd == []
    sh.proc_network_msg("AggregatedVote", b"qc bytes")
    assert [k for k, _ in fwd] == ["SignedVote", "SignedVote", "AggregatedVote"]
    assert oc.prefetch_calls == [2]
    sh.proc_network_msg(*("SignedVote", ig.encode_signed_vote(msgs[2][1])))
    sh.proc_network_msg("SignedProposal", b"proposal bytes")
    assert [k for k, _ in fwd][3:] == ["SignedVote", "SignedProposal"]


def test_deadline_checked_on_arrival():
    """A held group whose oldest message has waited max_delay_s is flushed by the next arrival."""
    import orc
    nval = 6
    sks = [(int.from_bytes(sm3(b"deadline %d" % i), "big") >> 3).to_bytes(32, "big") for i in range(nval)]
    pks = [orc.sk_to_pk(k)[1] for k in sks]
    oc = OracleCrypto(pks)
    msgs = _stream(nval, 6, 0, sm3(b"block 6"), lambda i, d: orc.sign(sks[i], d)[1], pks)
    fwd = []
    now = [0.0]
    sh = ig.VoteIngress(oc, lambda k, m: fwd.append((k, m)), max_delay_s=0.01, clock=lambda: now[0])
    sh.proc_network_msg("SignedVote", ig.encode_signed_vote(msgs[0][1]))
    now[0] = 0.05
    sh.proc_network_msg("SignedVote", ig.encode_signed_vote(msgs[1][1]))
    assert [m for _, m in fwd] == [msgs[0][1]] and oc.prefetch_calls == [1]
