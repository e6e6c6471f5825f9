"""The device arithmetic headers (consensus_overlord_amd/csrc/bls/*.hpp) compiled for the
host with g++ (tests/host/harness.cpp) against the golden fixtures. Test-only build: it is
never linked into the product."""
import ctypes
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def hx():
    out = os.path.join(ROOT, "tests", "host", "_build", "libhx.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    # built under a per-process name and renamed into place: parallel workers (pytest -n) never
    # load a half-written library
    tmp = "%s.%d" % (out, os.getpid())
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", tmp,
                           os.path.join(ROOT, "tests", "host", "harness.cpp")])
    os.replace(tmp, out)
    return ctypes.CDLL(out)


def test_gt_value(hx, golden):
    out = ctypes.create_string_buffer(576)
    hx.hx_gt_g1g2(out)
    assert ["%096x" % int.from_bytes(out.raw[48 * i:48 * i + 48], "big") for i in range(12)] == golden["gt_e_g1_g2_cubed"]


def test_hash_to_g2(hx, golden):
    dst = golden["dst"].encode()
    for h in golden["hash_to_g2"]:
        o = ctypes.create_string_buffer(192)
        assert hx.hx_hash_to_g2(bytes.fromhex(h["msg"]), dst, len(dst), o) == 0
        assert o.raw.hex() == h["point"]


def test_verify_codes(hx, golden):
    for c in golden["verify"]:
        s, h, p = (bytes.fromhex(c[k]) for k in ("sig", "hash", "pk"))
        assert hx.hx_verify(s, len(s), h, len(h), p, len(p)) == c["code"], c["name"]
