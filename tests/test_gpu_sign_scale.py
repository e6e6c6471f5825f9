"""Signing and key generation at the benchmark's batch size (4096, BASELINE configs[2]) on the VM
(k_vm_signg: GLS digits of the scalar as selb bits, 32-lane slices; k_vm_pkgen): a seeded sample
of 512 signatures and keys byte-equal to the C oracle's (orc.sign / orc.sk_to_pk, consensus.rs
:352,390-395), and every one of the 4096 (sig, hash, key) triples verifies in one batch."""
import hashlib
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


def test_sign_and_keys_4096_match_oracle():
    import torch
    import orc
    import consensus_overlord_amd as coa
    from consensus_overlord_amd import device as dev
    cc = coa.ConsensusCrypto(bytes.fromhex("13" * 32))
    n = 4096
    rng = random.Random(0x5161)
    ks = [rng.randrange(1, R) for _ in range(n)]
    sks = np.stack([np.frombuffer(k.to_bytes(32, "big"), dtype=np.uint8) for k in ks])
    hs = np.stack([np.frombuffer(hashlib.sha256(b"scale %d" % i).digest(), dtype=np.uint8) for i in range(n)])
    d_sk, d_h = torch.from_numpy(sks).cuda(), torch.from_numpy(hs).cuda()
    sigs = dev.sign_batch(cc.ctx, d_sk, d_h)
    pks = dev.sk_to_pk_batch(cc.ctx, d_sk)
    s_host, p_host = sigs.cpu().numpy(), pks.cpu().numpy()
    for i in sorted(rng.sample(range(n), 512)):
        sk, h = bytes(sks[i]), bytes(hs[i])
        assert bytes(s_host[i]) == orc.sign(sk, h)[1], i
        assert bytes(p_host[i]) == orc.sk_to_pk(sk)[1], i
    codes = dev.verify_batch(cc.ctx, sigs, d_h, pks).cpu().numpy()
    assert (codes == 0).all(), np.nonzero(codes)[0][:10]
