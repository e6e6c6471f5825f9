"""GPU parity: the HIP path (through the C ABI) against the oracle's golden fixtures and
against the Python oracle on seeded inputs. Bit-exact: verdicts, error codes and
aggregated signature / public key bytes."""
import hashlib
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cc():
    import consensus_overlord_amd as coa
    return coa.ConsensusCrypto(bytes.fromhex("11" * 32))


def _b(h):
    return bytes.fromhex(h)


def _code(fn):
    from consensus_overlord_amd.crypto import ConsensusError, CryptoErr, Other
    try:
        fn()
        return 0
    except CryptoErr as e:
        return e.code
    except Other as e:
        return {"failed to convert hash value": 100,
                "signatures length does not match voters length": 101,
                "lose public key": 102}[str(e)]


def test_verify_golden_exact_codes(cc, golden):
    for c in golden["verify"]:
        got = cc.lib.ovh_verify(cc.ctx.ptr, _b(c["sig"]), len(_b(c["sig"])), _b(c["hash"]), len(_b(c["hash"])),
                                _b(c["pk"]), len(_b(c["pk"])))
        assert got == c["code"], c["name"]


def test_trait_error_mapping(cc, golden):
    by = {c["name"]: c for c in golden["verify"]}
    for name, code in (("valid_0", 0), ("hash_31", 100), ("pk_47", 102), ("sig_95", 1), ("wrong_msg", 5)):
        c = by[name]
        assert _code(lambda: cc.verify_signature(_b(c["sig"]), _b(c["hash"]), _b(c["pk"]))) == code


def test_sign_and_pubkey_golden(golden):
    """Golden keys are raw scalars: a context with OVH_FLAG_SK_RAW (blst SecretKey::from_bytes)."""
    import consensus_overlord_amd as coa
    from consensus_overlord_amd.crypto import FLAG_SK_RAW, Context
    ctx = Context(flags=FLAG_SK_RAW)
    for k, v in zip(golden["keys"][:4], golden["votes"][:4]):
        c = coa.ConsensusCrypto(_b(k["sk"]), ctx=ctx)
        assert c.name.hex() == k["pk"]
        assert c.sign(_b(v["digest"])).hex() == v["sig"]
        assert c.hash(_b(v["rlp"])).hex() == v["digest"]


def test_reference_example_private_key():
    """ConsensusCrypto::new on the reference's own example/private_key (>= r): KeyGen parse,
    name and signatures equal the oracle's fixture (tests/golden/example_key.json); the strict
    scalar parse (OVH_FLAG_SK_RAW) rejects it with BLST_BAD_ENCODING."""
    import json
    import os
    import consensus_overlord_amd as coa
    from consensus_overlord_amd.crypto import FLAG_SK_RAW, Context, CryptoErr
    with open(os.path.join(os.path.dirname(__file__), "golden", "example_key.json")) as fh:
        ex = json.load(fh)
    c = coa.ConsensusCrypto(ex["key_hex"] + "\n")      # the key file's text, as read from disk
    assert c.scalar().hex() == ex["scalar"]
    assert c.name.hex() == ex["name"]
    for s in ex["signatures"]:
        assert c.sign(_b(s["digest"])).hex() == s["sig"]
        c.verify_signature(_b(s["sig"]), _b(s["digest"]), c.name)
    try:
        coa.ConsensusCrypto(ex["key_hex"], ctx=Context(flags=FLAG_SK_RAW))
        raise AssertionError("strict parse accepted a key >= r")
    except CryptoErr as e:
        assert e.code == ex["raw_parse_code"]


def test_aggregate_golden(cc, golden):
    for c in golden["aggregate"]:
        sigs = [_b(s) for s in c["sigs"]]
        pks = [_b(p) for p in c["pks"]]
        out = {}

        def run():
            out["v"] = cc.aggregate_signatures(sigs, pks)
        code = _code(run)
        assert code == c["code"], c["name"]
        if code == 0:
            assert out["v"].hex() == c["out"], c["name"]
    for c in golden["aggregate_pks"]:
        pks = [_b(p) for p in c["pks"]]
        out = {}

        def run():
            out["v"] = cc.aggregate_public_keys(pks)
        code = _code(run)
        assert code == c["code"], c["name"]
        if code == 0:
            assert out["v"].hex() == c["out"], c["name"]


def test_qc_config2(cc, golden):
    q = golden["qc"]
    pks = [_b(p) for p in q["pks"]]
    sigs = [_b(s) for s in q["sigs"]]
    h = _b(q["hash"])
    assert cc.aggregate_signatures(sigs, pks[:67]).hex() == q["agg_sig"]
    assert cc.aggregate_public_keys(pks[:67]).hex() == q["agg_pk"]
    agg = _b(q["agg_sig"])
    assert _code(lambda: cc.verify_aggregated_signature(agg, h, pks[:67])) == q["verify_ok"]
    assert _code(lambda: cc.verify_aggregated_signature(agg, h, pks[:66])) == q["verify_missing_one"]
    assert _code(lambda: cc.verify_aggregated_signature(agg, _b("00" * 32), pks[:67])) == 5
    assert _code(lambda: cc.verify_aggregated_signature(agg, h, [])) == q["verify_empty"]
    assert _code(lambda: cc.verify_aggregated_signature(agg, h[:31], pks[:67])) == q["verify_hash_31"]
    assert _code(lambda: cc.verify_aggregated_signature(agg, h, pks[:66] + [pks[0][:40]])) == q["verify_bad_pk"]


def test_batch_matches_per_vote_golden(cc, golden):
    # every fixed-size golden case (96/32/48 bytes) through the batch path == per-vote code
    cases = [c for c in golden["verify"] if len(_b(c["sig"])) == 96 and len(_b(c["hash"])) == 32
             and len(_b(c["pk"])) == 48]
    codes = cc.verify_batch([_b(c["sig"]) for c in cases], [_b(c["hash"]) for c in cases],
                            [_b(c["pk"]) for c in cases])
    for c, got in zip(cases, codes):
        assert got == c["code"], c["name"]


def test_batch_all_valid_uses_rlc(cc, golden):
    v = golden["votes"]
    k = golden["keys"]
    codes = cc.verify_batch([_b(x["sig"]) for x in v], [_b(x["digest"]) for x in v], [_b(x["pk"]) for x in k])
    assert list(codes) == [0] * len(v)


def _synth(n, seed=0xC17A):
    import torch
    import overlord_oracle as ov
    sks = np.zeros((n, 32), dtype=np.uint8)
    hs = np.zeros((n, 32), dtype=np.uint8)
    for i in range(n):
        sks[i] = np.frombuffer(ov.synth_sk(i, seed).to_bytes(32, "big"), dtype=np.uint8)
        hs[i] = np.frombuffer(hashlib.sha256(b"vote%d" % i).digest(), dtype=np.uint8)
    return torch.from_numpy(sks).cuda(), torch.from_numpy(hs).cuda()


def test_device_batch_config5_invalid_positions(cc):
    """Config 5 shape at n = 256: 1% invalid (sigma replaced by sigma + G2) at seeded random
    positions; every invalid position flagged (code 5), every other vote Ok."""
    import torch
    import bls12_381 as bls
    from consensus_overlord_amd import device as dev
    n = 256
    sks, hs = _synth(n)
    pks = dev.sk_to_pk_batch(cc.ctx, sks)
    sigs = dev.sign_batch(cc.ctx, sks, hs)
    # oracle spot-check of device signing/pk derivation
    rng = random.Random(3)
    for i in rng.sample(range(n), 3):
        sk = int.from_bytes(sks[i].cpu().numpy().tobytes(), "big")
        assert bytes(pks[i].cpu().numpy()) == bls.g1_compress(bls.sk_to_pk(sk))
        assert bytes(sigs[i].cpu().numpy()) == bls.g2_compress(bls.sign(sk, bytes(hs[i].cpu().numpy())))
    bad = sorted(rng.sample(range(n), max(1, n // 100)))
    s_host = sigs.cpu().numpy().copy()
    for i in bad:
        pt = bls.g2_from_bytes(bytes(s_host[i]))
        s_host[i] = np.frombuffer(bls.g2_compress(bls.pt_add(bls.Fp2Ops, pt, bls.G2_GEN)), dtype=np.uint8)
    sigs2 = torch.from_numpy(s_host).cuda()
    torch.cuda.synchronize()
    codes = dev.verify_batch(cc.ctx, sigs2, hs, pks).cpu().numpy()
    assert [i for i in range(n) if codes[i] != 0] == bad
    assert all(codes[i] == 5 for i in bad)
    codes = dev.verify_batch(cc.ctx, sigs, hs, pks).cpu().numpy()
    assert (codes == 0).all()


def test_partials_combine_two_shards(cc):
    import torch
    from consensus_overlord_amd import device as dev
    n = 128
    sks, hs = _synth(n, seed=5)
    pks = dev.sk_to_pk_batch(cc.ctx, sks)
    sigs = dev.sign_batch(cc.ctx, sks, hs)
    parts = torch.empty((2, 864), dtype=torch.uint8, device="cuda")
    codes = torch.empty((n,), dtype=torch.int32, device="cuda")
    h = n // 2
    dev.batch_partial(cc.ctx, sigs[:h], hs[:h], pks[:h], codes[:h], parts[0])
    dev.batch_partial(cc.ctx, sigs[h:], hs[h:], pks[h:], codes[h:], parts[1])
    assert dev.combine_partials(cc.ctx, parts)
    # swap two hashes across shards: the combined check must fail
    hs2 = hs.clone()
    hs2[[0, h]] = hs[[h, 0]]
    torch.cuda.synchronize()
    dev.batch_partial(cc.ctx, sigs[:h], hs2[:h], pks[:h], codes[:h], parts[0])
    dev.batch_partial(cc.ctx, sigs[h:], hs2[h:], pks[h:], codes[h:], parts[1])
    assert not dev.combine_partials(cc.ctx, parts)
    # the synchronous bisection of the last shard flags exactly its swapped vote
    dev.batch_fallback(cc.ctx, n - h, codes[h:])
    c = codes[h:].cpu().numpy()
    assert [i for i in range(n - h) if c[i] != 0] == [0] and c[0] == 5


def test_pipelined_batches_with_invalid(cc):
    """Four batches in flight through ovh_verify_batch_device_async (two state slots): batch 1
    holds invalid votes, so its device-gated fallback runs on the final stream while batch 2's
    per-vote stages run; every batch's codes equal the per-vote verdicts after batch_wait."""
    import torch
    import bls12_381 as bls
    from consensus_overlord_amd import device as dev
    n = 192
    sks, hs = _synth(n, seed=21)
    pks = dev.sk_to_pk_batch(cc.ctx, sks)
    sigs = dev.sign_batch(cc.ctx, sks, hs)
    s_host = sigs.cpu().numpy().copy()
    bad = [3, 77, 150]
    for i in bad:
        pt = bls.g2_from_bytes(bytes(s_host[i]))
        s_host[i] = np.frombuffer(bls.g2_compress(bls.pt_add(bls.Fp2Ops, pt, bls.G2_GEN)), dtype=np.uint8)
    sigs_bad = torch.from_numpy(s_host).cuda()
    codes = torch.full((4, n), -1, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    for b, sg in enumerate((sigs, sigs_bad, sigs, sigs_bad)):
        dev.verify_batch_async(cc.ctx, sg, hs, pks, codes[b])
    dev.batch_wait(cc.ctx)
    c = codes.cpu().numpy()
    assert (c[0] == 0).all() and (c[2] == 0).all()
    for b in (1, 3):
        assert [i for i in range(n) if c[b, i] != 0] == bad
        assert all(c[b, i] == 5 for i in bad)


def test_pipelined_combine_async(cc):
    """Multi-GPU form on one device: partial -> combine_partials_async (final stream, fallback
    gated on the verdict) for a valid and an invalid shard pair."""
    import torch
    from consensus_overlord_amd import device as dev
    n = 96
    sks, hs = _synth(n, seed=33)
    pks = dev.sk_to_pk_batch(cc.ctx, sks)
    sigs = dev.sign_batch(cc.ctx, sks, hs)
    h = n // 2
    hs2 = hs.clone()
    hs2[[1, 2]] = hs[[2, 1]]       # two votes of shard 0 sign the other's digest
    torch.cuda.synchronize()
    out = []
    for hh in (hs, hs2):
        parts = torch.empty((2, 864), dtype=torch.uint8, device="cuda")
        c1 = torch.full((h,), -1, dtype=torch.int32, device="cuda")
        c0 = torch.full((h,), -1, dtype=torch.int32, device="cuda")
        dev.batch_partial(cc.ctx, sigs[h:], hh[h:], pks[h:], c1, parts[1], stream=True)
        dev.batch_partial(cc.ctx, sigs[:h], hh[:h], pks[:h], c0, parts[0], stream=True)
        dev.combine_partials_async(cc.ctx, parts, h, c0, stream=True)   # bisection of the last shard
        dev.batch_wait(cc.ctx)
        out.append(c0.cpu().numpy())
    assert (out[0] == 0).all()
    assert [i for i in range(h) if out[1][i] != 0] == [1, 2] and all(out[1][i] == 5 for i in (1, 2))


def test_partials_interoperate_with_oracle(cc):
    """A GPU shard partial and a C-oracle shard partial (same 864-byte format) combine on the GPU
    and in the oracle to the same verdict: valid batch -> pass, cross-shard digest swap -> fail."""
    import torch
    import orc
    from consensus_overlord_amd import device as dev
    n = 64
    sks, hs = _synth(n, seed=44)
    pks = dev.sk_to_pk_batch(cc.ctx, sks)
    sigs = dev.sign_batch(cc.ctx, sks, hs)
    h = n // 2
    for swap, want in ((False, True), (True, False)):
        hh = hs.clone()
        if swap:
            hh[[0, h]] = hs[[h, 0]]
        torch.cuda.synchronize()
        parts = torch.empty((2, 864), dtype=torch.uint8, device="cuda")
        codes = torch.empty((h,), dtype=torch.int32, device="cuda")
        dev.batch_partial(cc.ctx, sigs[:h], hh[:h], pks[:h], codes, parts[0])
        c1, p1 = orc.batch_partial(sigs[h:].cpu().numpy(), hh[h:].cpu().numpy(), pks[h:].cpu().numpy(), 72)
        assert (c1 == 0).all()
        parts[1] = torch.from_numpy(p1).cuda()
        assert dev.combine_partials(cc.ctx, parts) == want
        assert orc.combine_partials(parts.cpu().numpy()) == want


def test_shard_verifier_rccl_single_rank(cc):
    """The multi-GPU driver (consensus_overlord_amd/shard.py) on the GPU with libovhip as the
    backend, over a one-rank RCCL group: pipelined shard batches (one with invalid votes) give
    the per-vote codes, with the test's context and with an OVH_FLAG_POOL_RESERVE one."""
    import os
    import socket
    import torch
    import torch.distributed as dist
    import bls12_381 as bls
    from consensus_overlord_amd import device as dev
    from consensus_overlord_amd.crypto import Context, FLAG_POOL_RESERVE
    from consensus_overlord_amd.shard import DeviceBackend, ShardVerifier
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        n = 64
        sks, hs = _synth(n, seed=55)
        pks = dev.sk_to_pk_batch(cc.ctx, sks)
        sigs = dev.sign_batch(cc.ctx, sks, hs)
        s_host = sigs.cpu().numpy().copy()
        pt = bls.g2_from_bytes(bytes(s_host[9]))
        s_host[9] = np.frombuffer(bls.g2_compress(bls.pt_add(bls.Fp2Ops, pt, bls.G2_GEN)), dtype=np.uint8)
        bad = torch.from_numpy(s_host).cuda()
        # the test's context, then one whose pool leaves CUs to the collective (OVH_FLAG_POOL_RESERVE:
        # shard batches in the persistent pool, bench.py's shard path)
        rsv = Context(0, flags=FLAG_POOL_RESERVE)
        for ctx in (cc.ctx, rsv):
            sv = ShardVerifier(DeviceBackend(ctx))
            codes = torch.full((3, n), -1, dtype=torch.int32, device="cuda")
            torch.cuda.synchronize()
            for b, sg in enumerate((sigs, bad, sigs)):
                sv.submit(b, sg, hs, pks, codes[b])
            sv.wait()
            c = codes.cpu().numpy()
            assert (c[0] == 0).all() and (c[2] == 0).all()
            assert [i for i in range(n) if c[1, i] != 0] == [9] and c[1, 9] == 5
        rsv.close()
    finally:
        dist.destroy_process_group()


def test_aggregate_vm_tree_matches_oracle(cc, golden):
    """aggregate_signatures' VM path (k_vm_sigchk + the padd tree) at sizes 1 .. 300, with
    repeated signatures (the tree doubles), a sigma / -sigma pair, the infinity encoding, and
    every 96-byte golden signature alone (exact codes and bytes against the C oracle)."""
    import orc
    import synth_votes as sv
    sigs, _, pks = sv.make(cc.ctx, 300, lo=70000)
    sigs, pks = [bytes(s) for s in sigs], [bytes(p) for p in pks]
    neg = sv.bls.g2_compress(sv.bls.pt_neg(sv.bls.Fp2Ops, sv.bls.g2_from_bytes(sigs[5])))
    inf = bytes([0xC0]) + bytes(95)
    lists = [(sigs[:n], pks[:n]) for n in (1, 2, 3, 67, 128, 129, 300)]
    lists.append((sigs[:40] + sigs[:40] + [sigs[7]], pks[:40] + pks[:40] + [pks[7]]))
    lists.append((sigs[:9] + [neg, inf], pks[:11]))
    for c in golden["verify"]:
        if len(c["sig"]) == 192:
            lists.append(([_b(c["sig"])], [pks[0]]))
            lists.append((sigs[:5] + [_b(c["sig"])], pks[:6]))
    for ss, ps in lists:
        want = orc.aggregate_sigs(ss, ps)
        out = {}

        def run():
            out["v"] = cc.aggregate_signatures(ss, ps)
        code = _code(run)
        assert code == want[0], (len(ss), want)
        if code == 0:
            assert out["v"] == want[1], len(ss)


def test_vm_pkgen_edge_scalars(cc):
    """Public keys on the VM (program pkgen, four 64-bit chunks) through the device batch entry:
    scalars 1, 2, 3, empty 64-bit chunks, 2^64 +- 1, r - 1 and seeded random ones == the oracle's
    compressed [k] G1."""
    import torch
    import bls12_381 as bls
    from consensus_overlord_amd import device as dev
    r = bls.R
    rng = random.Random(17)
    ks = [1, 2, 3, 2 ** 64 - 1, 2 ** 64, 2 ** 64 + 1, 2 ** 192, r - 1, r - 2] + [rng.randrange(1, r) for _ in range(23)]
    sks = torch.from_numpy(np.stack([np.frombuffer(k.to_bytes(32, "big"), dtype=np.uint8) for k in ks])).cuda()
    got = dev.sk_to_pk_batch(cc.ctx, sks).cpu().numpy()
    for k, g in zip(ks, got):
        assert bytes(g) == bls.g1_compress(bls.sk_to_pk(k)), hex(k)


def test_vm_sign_edge_scalars(cc):
    """Crypto::sign on the VM (signg0 + 3 x signg1: the GLS digits of k mod r as selb bits):
    scalars with empty 64-bit chunks, single bits, r - 1, powers of |x| and their neighbours
    (digit carries and all-maximal digits), scalars >= r (reduced on the device) and random ones,
    batch and per-call, against the C oracle."""
    import torch
    import orc
    from consensus_overlord_amd import device as dev
    r = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
    rng = random.Random(0x516)
    ks = [1, 2, 3, 2 ** 64 - 1, 2 ** 64, 2 ** 128 + 1, 2 ** 192, 2 ** 254, r - 1, r - 2 ** 64]
    x = 0xD201000000010000
    ks += [x - 1, x, x + 1, x ** 2 - 1, x ** 2, x ** 3 - 1, x ** 3, x ** 3 + x - 1,
           (x - 1) * (1 + x + x ** 2), (r // x ** 3 - 1) * x ** 3 + (x - 1) * (1 + x + x ** 2),
           r, r + 1, 2 * r + 5, 2 ** 256 - 1]
    ks += [rng.randrange(1, r) for _ in range(41)]
    sks = [k.to_bytes(32, "big") for k in ks]
    hs = [hashlib.sha256(b"sign %d" % i).digest() for i in range(len(ks))]
    # H has order r: [k] H = [k mod r] H (the oracle's key parse takes only 0 < k < r; [r] H is
    # the point at infinity)
    want = [orc.sign((k % r).to_bytes(32, "big"), h) if k % r else (0, bytes([0xC0]) + bytes(95))
            for k, h in zip(ks, hs)]
    assert all(w[0] == 0 for w in want)
    d_sk = torch.from_numpy(np.frombuffer(b"".join(sks), dtype=np.uint8).reshape(-1, 32).copy()).cuda()
    d_h = torch.from_numpy(np.frombuffer(b"".join(hs), dtype=np.uint8).reshape(-1, 32).copy()).cuda()
    got = dev.sign_batch(cc.ctx, d_sk, d_h).cpu().numpy()
    for i, w in enumerate(want):
        assert bytes(got[i]) == w[1], ks[i]
    from consensus_overlord_amd.crypto import FLAG_SK_RAW, Context
    import consensus_overlord_amd as coa
    ctx = Context(flags=FLAG_SK_RAW)
    for i in (0, 4, 8, 9, 11, 19):
        assert coa.ConsensusCrypto(sks[i], ctx=ctx).sign(hs[i]) == want[i][1], ks[i]
