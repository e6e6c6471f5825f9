#!/usr/bin/env python
"""Generate tests/golden/example_key.json from the Python oracle (test infrastructure).

The reference's one crypto fixture is its example private key file,
/root/reference/example/private_key (the README runs the node with it, README.md:66). Its 32
bytes are >= r, and ConsensusCrypto::new unwraps the parse (src/consensus.rs:349-350), so
ophelia-blst's BlsPrivateKey::try_from must accept them: blst SecretKey::key_gen (IETF KeyGen),
pinned here by the EIP-2333 master-key and RFC 5869 vectors (tests/test_oracle_kat.py).

The key's 64 hex characters are copied below (a data fixture, not reference code), so the GPU
tests do not need /root/reference. Records: the KeyGen scalar, name = the compressed public key
(consensus.rs:352,357), and signatures over the Appendix B vote digest and over SM3("").

    python tests/golden/make_example_key.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle", "py"))

import bls12_381 as bls  # noqa: E402
import overlord_oracle as ov  # noqa: E402

EXAMPLE_KEY_HEX = "ed391472f4ecd53a398b5bac8044afbe27dca9ad356823a723609488b1f31690"


def main():
    key = bytes.fromhex(EXAMPLE_KEY_HEX)
    assert int.from_bytes(key, "big") >= bls.R, "the example key is expected to be >= r"
    sk = bls.sk_keygen(key)
    pk = bls.g1_compress(bls.sk_to_pk(sk))
    vote_digest = ov.vote_hash(1, 0, ov.PRECOMMIT, ov.sm3(b""))
    sigs = []
    for d in (vote_digest, ov.sm3(b"")):
        code, sig = ov.sign(sk, d)
        assert code == 0
        assert ov.verify_signature(sig, d, pk) == 0
        sigs.append({"digest": d.hex(), "sig": sig.hex()})
    out = {
        "key_hex": EXAMPLE_KEY_HEX,
        "source": "/root/reference/example/private_key (hex text, as read by consensus.rs:349)",
        "parse": "IETF KeyGen (blst SecretKey::key_gen(key, \"\"))",
        "scalar": "%064x" % sk,
        "name": pk.hex(),
        "signatures": sigs,
        "raw_parse_code": 1,   # OVH_FLAG_SK_RAW: the key is >= r -> BLST_BAD_ENCODING
    }
    with open(os.path.join(HERE, "example_key.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote example_key.json", out["name"])


if __name__ == "__main__":
    main()
