"""SURVEY.md 8(d) synthetic votes for the GPU parity tests (test infrastructure).

Seed 0xC17A; sk_i = SHA-256(seed || i) mod r; vote i = rlp(Vote{height 1 + i/64, round i%3,
Precommit, block_hash SM3(seed || i)}), digest = SM3(rlp) (the bytes check_block hashes,
consensus.rs:169-175); pk_i = sk_i G1 and sigma_i = sk_i H(digest) are made on the device
(ovh_sk_to_pk_batch_device / ovh_sign_batch_device) and spot-checked against the C oracle."""
import hashlib

import numpy as np

import bls12_381 as bls
import orc
import overlord_oracle as ov

SEED = 0xC17A


def digests(lo: int, n: int, seed: int = SEED) -> np.ndarray:
    out = np.zeros((n, 32), dtype=np.uint8)
    for k in range(n):
        out[k] = np.frombuffer(ov.synth_vote_digest(lo + k, seed), dtype=np.uint8)
    return out


def scalars(lo: int, n: int, seed: int = SEED) -> np.ndarray:
    out = np.zeros((n, 32), dtype=np.uint8)
    for k in range(n):
        out[k] = np.frombuffer(ov.synth_sk(lo + k, seed).to_bytes(32, "big"), dtype=np.uint8)
    return out


def make(ctx, n: int, lo: int = 0, seed: int = SEED, check: int = 2):
    """-> (sigs (n, 96), hashes (n, 32), pks (n, 48)) numpy uint8, device-signed."""
    import torch
    from consensus_overlord_amd import device as dev
    sks = torch.from_numpy(scalars(lo, n, seed)).cuda()
    hs = torch.from_numpy(digests(lo, n, seed)).cuda()
    pks = dev.sk_to_pk_batch(ctx, sks)
    sigs = dev.sign_batch(ctx, sks, hs)
    out = sigs.cpu().numpy(), hs.cpu().numpy(), pks.cpu().numpy()
    sk_np = sks.cpu().numpy()
    for i in np.linspace(0, n - 1, num=min(check, n), dtype=int):
        assert orc.sk_to_pk(bytes(sk_np[i])) == (0, bytes(out[2][i])), "device pk differs from the oracle"
        assert orc.sign(bytes(sk_np[i]), bytes(out[1][i])) == (0, bytes(out[0][i])), "device signature differs"
    return out


def add_g2(sig: bytes) -> bytes:
    """sigma + G2 (still in G2, no longer a signature of the vote): the config-5 corruption."""
    return bls.g2_compress(bls.pt_add(bls.Fp2Ops, bls.g2_from_bytes(sig), bls.G2_GEN))


def oracle_codes(sigs, hs, pks, threads: int = 16) -> np.ndarray:
    return orc.verify_many(sigs, hs, pks, threads=threads)


def seeded_positions(n: int, frac: float, seed: int):
    import random
    return sorted(random.Random(seed).sample(range(n), max(1, int(round(n * frac)))))


def sha(b: bytes) -> bytes:
    return hashlib.sha256(b).digest()
