"""Shared construction of the cancellation attack on a random-linear-combination batch whose
coefficients are predictable (test helper; oracle-side arithmetic only).

With the coefficients r_a, r_b of votes a and b known, an adversary submits
  sigma_a' = sigma_a + [r_b] T,   sigma_b' = sigma_b - [r_a] T   (T any point of G2):
both stay in G2, sum_i r_i sigma_i' = sum_i r_i sigma_i, so the combined check still passes and
the per-vote bisection never runs -- two invalid votes would be accepted. libovhip therefore
draws the batch seed from getrandom(2) (include/ovhip.h, OVH_FLAG_TEST_RLC is for tests only)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools", "fpvm"))

import bls12_381 as bls  # noqa: E402
from alg import rlc_scalar  # noqa: E402  (r = a + b lambda from the 64-bit SplitMix64 value)

M64 = (1 << 64) - 1


def splitmix(seed: int, i: int) -> int:
    """The 64-bit coefficient source of vote i (ovhip.hip rlc_scalar, bls_oracle.c splitmix)."""
    z = (seed + 0x9E3779B97F4A7C15 * (i + 1)) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    z ^= z >> 31
    return z or 1


def coefficient(seed: int, i: int) -> int:
    return rlc_scalar(splitmix(seed, i))


def cancel_pair(sig_a: bytes, sig_b: bytes, seed: int, a: int, b: int):
    """-> (sigma_a', sigma_b') compressed, cancelling under the coefficients of (seed, a, b)."""
    ra, rb = coefficient(seed, a), coefficient(seed, b)
    T = bls.G2_GEN
    pa = bls.pt_add(bls.Fp2Ops, bls.g2_from_bytes(sig_a), bls.pt_mul(bls.Fp2Ops, T, rb))
    pb = bls.pt_add(bls.Fp2Ops, bls.g2_from_bytes(sig_b), bls.pt_neg(bls.Fp2Ops, bls.pt_mul(bls.Fp2Ops, T, ra)))
    return bls.g2_compress(pa), bls.g2_compress(pb)
