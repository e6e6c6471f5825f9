"""Soundness of the random-linear-combination batch (VERDICT r1 "What's weak" 4, ADVICE high):
with predictable coefficients two invalid signatures can cancel inside the combined check. The C
oracle (test infrastructure) shows the attack succeeds under the known seed and fails under any
other; tests/test_gpu_parity.py shows libovhip's default (getrandom) seeds flag both votes."""
import numpy as np

import orc
import overlord_oracle as ov
from rlc_attack import cancel_pair, coefficient, splitmix


def _votes(golden, n=4):
    v, k = golden["votes"][:n], golden["keys"][:n]
    sigs = [bytes.fromhex(x["sig"]) for x in v]
    hs = [bytes.fromhex(x["digest"]) for x in v]
    pks = [bytes.fromhex(x["pk"]) for x in k]
    return sigs, hs, pks


def _arr(items, w):
    return np.frombuffer(b"".join(items), dtype=np.uint8).reshape(-1, w)


def test_known_seed_lets_cancelling_signatures_pass(golden):
    sigs, hs, pks = _votes(golden)
    seed = 0x1234
    sigs[0], sigs[2] = cancel_pair(sigs[0], sigs[2], seed, 0, 2)
    per_vote = [ov.verify_signature(s, h, p) for s, h, p in zip(sigs, hs, pks)]
    assert per_vote == [5, 0, 5, 0]                       # both forged votes are invalid
    codes, ok = orc.verify_batch_rlc(_arr(sigs, 96), _arr(hs, 32), _arr(pks, 48), seed)
    assert ok and codes.tolist() == [0, 0, 0, 0]         # ...but the known-seed batch accepts them
    codes, ok = orc.verify_batch_rlc(_arr(sigs, 96), _arr(hs, 32), _arr(pks, 48), seed + 1)
    assert not ok and codes.tolist() == per_vote          # any other seed catches both


def test_per_rank_seed_variant_collides_global_index_does_not():
    """rank r used seed ^ r*phi with phi the SplitMix64 stride, so for
    seed & phi == 0 (seed 0) rank 1's vote i had rank 0's vote i + 1 coefficient. One seed with a
    global vote index gives distinct coefficients across the shards."""
    phi = 0x9E3779B97F4A7C15
    old = lambda rank, i, seed=0: splitmix(seed ^ (rank * phi), i)  # noqa: E731
    assert old(1, 0) == old(0, 1)
    n, world = 64, 4
    new = {coefficient(7, lo + i) for lo in range(0, n, n // world) for i in range(n // world)}
    assert len(new) == n
