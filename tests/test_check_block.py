"""Consensus::check_block (consensus.rs:143-207) composed over the Crypto surface: the overlord
Proof RLP (vote.py, layout [dep] overlord 0.4), the height / block-hash check (:165), the voters
from the bitmap (:166-167), the Precommit vote hash (:169-175) and the aggregated-signature check
(:176-183). The CPU tests run the host logic with the C oracle in place of the device (test
infrastructure); the GPU test runs ConsensusCrypto.check_block / check_blocks through the C ABI
and compares every verdict with that oracle-backed mirror."""
import hashlib
import random

import pytest

from consensus_overlord_amd import vote
from consensus_overlord_amd.crypto import ConsensusCrypto, CryptoErr

N_VAL = 100


def sm3(b):
    return hashlib.new("sm3", bytes(b)).digest()


# ---- RLP / Proof codec ----

def test_rlp_decode_round_trips_votes_and_proofs():
    rng = random.Random(0xB10C)
    for _ in range(200):
        h, r = rng.getrandbits(rng.choice((0, 8, 32, 64))), rng.getrandbits(rng.choice((0, 7, 16)))
        bh = bytes(rng.randrange(256) for _ in range(rng.choice((0, 1, 32, 55, 56, 64))))
        sig = bytes(rng.randrange(256) for _ in range(rng.choice((0, 1, 96, 300))))
        bm = bytes(rng.randrange(256) for _ in range(rng.choice((0, 1, 13, 60))))
        p = vote.encode_proof(h, r, bh, sig, bm)
        assert vote.decode_proof(p) == (h, r, bh, sig, bm)
        t = rng.randrange(2)
        assert vote.rlp_decode(vote.rlp_vote(h, r, t, bh)) == [
            h.to_bytes((h.bit_length() + 7) // 8, "big"), r.to_bytes((r.bit_length() + 7) // 8, "big"),
            bytes([t]) if t else b"", bh]


@pytest.mark.parametrize("bad", [
    b"", b"\xc0", b"\x80", b"\xc4\x01\x02\x03\x04",                           # not a 4-item proof
    bytes.fromhex("c701020380c2c0c0"),                                        # nested list as bytes
    bytes.fromhex("c8820001028080c28080"),                                    # u64 with a leading zero
    bytes.fromhex("cc890102030405060708090280c28080"),                        # u64 wider than 8 bytes
    bytes.fromhex("c6010280c28080") + b"\x00",                                # trailing byte
    bytes.fromhex("c7010280c28080"),                                          # truncated list
    bytes.fromhex("c6010280c2817f"),                                          # non-canonical single byte
])
def test_decode_proof_rejects_malformed(bad):
    with pytest.raises(ValueError):
        vote.decode_proof(bad)


# ---- fixtures: 100 validators, QCs signed with the C oracle ----

@pytest.fixture(scope="module")
def net():
    import orc
    sks = [(int.from_bytes(hashlib.sha256(b"check_block validator %d" % i).digest(), "big") >> 2).to_bytes(32, "big")
           for i in range(N_VAL)]
    pks = [orc.sk_to_pk(sk)[1] for sk in sks]
    skeys = sorted(pks)
    order = {pk: i for i, pk in enumerate(skeys)}

    def qc(height, round_, data, signers, nbytes=(N_VAL + 7) // 8, extra_bits=()):
        bh = sm3(data)
        vh = sm3(vote.rlp_vote(height, round_, vote.PRECOMMIT, bh))
        sigs = [orc.sign(sks[i], vh)[1] for i in signers]
        agg = orc.aggregate_sigs(sigs, [pks[i] for i in signers])[1]
        bm = bytearray(nbytes)
        for i in list(signers):
            k = order[pks[i]]
            bm[k // 8] |= 0x80 >> (k % 8)
        for k in extra_bits:
            bm[k // 8] |= 0x80 >> (k % 8)
        return agg, bh, bytes(bm)
    return pks, qc


def cases(net):
    pks, qc = net
    d1, d2 = b"block at height 10" * 7, b"block at height 11"
    agg, bh, bm = qc(10, 1, d1, range(67))
    agg_all, bh2, bm_all = qc(11, 0, d2, range(N_VAL), extra_bits=(100, 101, 103))
    agg_r3, _, bm_r3 = qc(10, 3, d1, range(33, 100))
    bm_less = bytearray(bm)
    first = next(i for i in range(N_VAL) if bm[i // 8] & (0x80 >> (i % 8)))
    bm_less[first // 8] &= ~(0x80 >> (first % 8)) & 0xFF
    P = vote.encode_proof
    return [
        ("valid 67/100", (10, d1, P(10, 1, bh, agg, bm)), True),
        ("valid 100/100, bits past the list", (11, d2, P(11, 0, bh2, agg_all, bm_all)), True),
        ("valid, round 3, other signers", (10, d1, P(10, 3, bh, agg_r3, bm_r3)), True),
        ("proposal height differs", (11, d1, P(10, 1, bh, agg, bm)), False),
        ("proposal data differs", (10, d2, P(10, 1, bh, agg, bm)), False),
        ("proof height differs", (9, d1, P(9, 1, bh, agg, bm)), False),
        ("round not the signed one", (10, d1, P(10, 2, bh, agg, bm)), False),
        ("signer missing from bitmap", (10, d1, P(10, 1, bh, agg, bytes(bm_less))), False),
        ("other QC's signature", (10, d1, P(10, 1, bh, agg_r3, bm)), False),
        ("empty bitmap", (10, d1, P(10, 1, bh, agg, b"")), False),
        ("short signature", (10, d1, P(10, 1, bh, agg[:95], bm)), False),
        ("signature not a point", (10, d1, P(10, 1, bh, b"\xff" * 96, bm)), False),
        ("undecodable proof", (10, d1, P(10, 1, bh, agg, bm)[:-1]), False),
        ("not a proof", (10, d1, vote.rlp_vote(10, 1, 1, bh)), False),
    ]


class OracleCrypto:
    """The Crypto surface check_block uses, answered by the C oracle (test infrastructure)."""

    def __init__(self, pks):
        self.pubkeys = list(pks)

    def hash(self, msg):
        return sm3(msg)

    def verify_aggregated_signature(self, agg, h, voters):
        import orc
        code = orc.verify_aggregated(bytes(agg), bytes(h), list(voters))
        if code:
            raise CryptoErr(code)


def test_check_block_host_logic_with_oracle_crypto(net):
    oc = OracleCrypto(net[0])
    for name, args, want in cases(net):
        assert ConsensusCrypto.check_block(oc, *args) is want, name
    # a caller-given authority list that lacks the signers
    name, args, _ = cases(net)[0]
    assert ConsensusCrypto.check_block(oc, *args, authority_list=net[0][67:]) is False


@pytest.mark.gpu
def test_check_block_on_device(net):
    import consensus_overlord_amd as coa
    cc = coa.ConsensusCrypto(bytes.fromhex("99" * 32))
    cc.update_pubkeys(net[0])
    cs = cases(net)
    got = [cc.check_block(*args) for _, args, _ in cs]
    assert got == [w for _, _, w in cs], [(n, g) for (n, _, _), g in zip(cs, got)]
    assert cc.check_blocks([args for _, args, _ in cs]).tolist() == got
    assert cc.check_block(*cs[0][1], authority_list=net[0][67:]) is False


@pytest.mark.gpu
def test_check_blocks_without_validator_table(net):
    """No update_pubkeys (or an empty list): check_blocks answers like check_block -- every
    block False (no authority list, no voters) -- instead of raising."""
    import consensus_overlord_amd as coa
    cc = coa.ConsensusCrypto(bytes.fromhex("98" * 32))
    cs = cases(net)[:3]
    assert cc.check_blocks([args for _, args, _ in cs]).tolist() == [False] * 3
    cc.update_pubkeys([])
    assert cc.check_blocks([args for _, args, _ in cs]).tolist() == [False] * 3
