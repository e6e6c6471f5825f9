"""CPU ORACLE (test infrastructure + CPU baseline only) -- ctypes binding of the C restatement
oracle/c/bls_oracle.c (built by `make -C oracle` into oracle/_build/liborc.so). Imported only by
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_ORACLE = os.path.dirname(_HERE)
LIB = os.path.join(_ORACLE, "_build", "liborc.so")
_lib = None
_u8 = ctypes.c_char_p
_sz = ctypes.c_size_t
_szp = ctypes.POINTER(ctypes.c_size_t)
_vp = ctypes.c_void_p


def load(build_if_missing: bool = True):
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB) and build_if_missing:
        subprocess.check_call(["make", "-C", _ORACLE], stdout=subprocess.DEVNULL)
    lib = ctypes.CDLL(LIB)
    sig = {
        "orc_set_dst": (None, [_u8, _sz]),
        "orc_hash_to_g2": (ctypes.c_int, [_u8, _sz, _u8]),
        "orc_sk_to_pk": (ctypes.c_int, [_u8, _sz, _u8]),
        "orc_sign": (ctypes.c_int, [_u8, _sz, _u8, _sz, _u8]),
        "orc_verify": (ctypes.c_int, [_u8, _sz, _u8, _sz, _u8, _sz]),
        "orc_aggregate_sigs": (ctypes.c_int, [_u8, _szp, _sz, _u8, _szp, _sz, _u8]),
        "orc_aggregate_pks": (ctypes.c_int, [_u8, _szp, _sz, _u8]),
        "orc_verify_aggregated": (ctypes.c_int, [_u8, _sz, _u8, _sz, _u8, _szp, _sz]),
        "orc_verify_many": (ctypes.c_int, [_sz, _vp, _vp, _vp, _vp, ctypes.c_int]),
        "orc_verify_batch_rlc": (ctypes.c_int, [_sz, _vp, _vp, _vp, ctypes.c_uint64, _vp, ctypes.c_int,
                                                ctypes.POINTER(ctypes.c_int)]),
        "orc_gt_g1g2": (None, [_u8]),
        "orc_batch_partial": (ctypes.c_int, [_sz, _vp, _vp, _vp, ctypes.c_uint64, ctypes.c_uint64, _vp, ctypes.c_int,
                                             _vp]),
        "orc_sk_keygen": (ctypes.c_int, [_u8, _sz, _u8]),
        "orc_combine_partials": (ctypes.c_int, [_sz, _vp, ctypes.POINTER(ctypes.c_int)]),
        "orc_mulx_active": (ctypes.c_int, []),
        "orc_mulx_selftest": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_int]),
        "orc_batch_fallback": (ctypes.c_int, [_sz, _vp, _vp, _vp, _vp, ctypes.c_int]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _lens(items):
    items = [bytes(x) for x in items]
    return b"".join(items), (ctypes.c_size_t * max(1, len(items)))(*[len(x) for x in items])


def sk_to_pk(sk: bytes):
    out = ctypes.create_string_buffer(48)
    c = load().orc_sk_to_pk(sk, len(sk), out)
    return c, (out.raw if c == 0 else None)


def sign(sk: bytes, h: bytes):
    out = ctypes.create_string_buffer(96)
    c = load().orc_sign(sk, len(sk), h, len(h), out)
    return c, (out.raw if c == 0 else None)


def verify(sig: bytes, h: bytes, pk: bytes) -> int:
    return load().orc_verify(sig, len(sig), h, len(h), pk, len(pk))


def aggregate_sigs(sigs, pks):
    sd, sl = _lens(sigs)
    pd, pl = _lens(pks)
    out = ctypes.create_string_buffer(96)
    c = load().orc_aggregate_sigs(sd, sl, len(sigs), pd, pl, len(pks), out)
    return c, (out.raw if c == 0 else None)


def aggregate_pks(pks):
    pd, pl = _lens(pks)
    out = ctypes.create_string_buffer(48)
    c = load().orc_aggregate_pks(pd, pl, len(pks), out)
    return c, (out.raw if c == 0 else None)


def verify_aggregated(agg: bytes, h: bytes, pks) -> int:
    pd, pl = _lens(pks)
    return load().orc_verify_aggregated(agg, len(agg), h, len(h), pd, pl, len(pks))


def hash_to_g2(msg: bytes, dst: bytes = None) -> bytes:
    lib = load()
    if dst is not None:
        lib.orc_set_dst(dst, len(dst))
    out = ctypes.create_string_buffer(192)
    try:
        assert lib.orc_hash_to_g2(msg, len(msg), out) == 0
    finally:
        if dst is not None:
            lib.orc_set_dst(None, 0)
    return out.raw


def _arr(a, width):
    a = np.ascontiguousarray(np.asarray(a, dtype=np.uint8).reshape(-1, width))
    return a, a.ctypes.data_as(ctypes.c_void_p)


def verify_many(sigs, hashes, pks, threads: int = 1) -> np.ndarray:
    s, sp = _arr(sigs, 96)
    h, hp = _arr(hashes, 32)
    p, pp = _arr(pks, 48)
    n = s.shape[0]
    codes = np.zeros(max(n, 1), dtype=np.int32)
    assert load().orc_verify_many(n, sp, hp, pp, codes.ctypes.data_as(ctypes.c_void_p), threads) == 0
    return codes[:n]


def verify_batch_rlc(sigs, hashes, pks, seed: int, threads: int = 1):
    s, sp = _arr(sigs, 96)
    h, hp = _arr(hashes, 32)
    p, pp = _arr(pks, 48)
    n = s.shape[0]
    codes = np.zeros(max(n, 1), dtype=np.int32)
    ok = ctypes.c_int(0)
    assert load().orc_verify_batch_rlc(n, sp, hp, pp, seed & 0xFFFFFFFFFFFFFFFF,
                                       codes.ctypes.data_as(ctypes.c_void_p), threads, ctypes.byref(ok)) == 0
    return codes[:n], bool(ok.value)


def gt_g1g2() -> list:
    out = ctypes.create_string_buffer(576)
    load().orc_gt_g1g2(out)
    return ["%096x" % int.from_bytes(out.raw[48 * i:48 * i + 48], "big") for i in range(12)]


def sk_keygen(ikm: bytes):
    """orc_sk_keygen (IETF KeyGen, BlsPrivateKey::try_from): -> (code, 32-byte scalar)."""
    out = ctypes.create_string_buffer(32)
    c = load().orc_sk_keygen(ikm, len(ikm), out)
    return c, (out.raw if c == 0 else None)


def batch_partial(sigs, hashes, pks, seed: int, threads: int = 1, base: int = 0):
    """orc_batch_partial: -> (codes, 864-byte partial in libovhip's format); vote i's
    coefficient is SplitMix64(seed, base + i)."""
    s, sp = _arr(sigs, 96)
    h, hp = _arr(hashes, 32)
    p, pp = _arr(pks, 48)
    n = s.shape[0]
    codes = np.zeros(max(n, 1), dtype=np.int32)
    out = np.zeros(864, dtype=np.uint8)
    assert load().orc_batch_partial(n, sp, hp, pp, seed & 0xFFFFFFFFFFFFFFFF, base,
                                    codes.ctypes.data_as(ctypes.c_void_p), threads,
                                    out.ctypes.data_as(ctypes.c_void_p)) == 0
    return codes[:n], out


def combine_partials(parts) -> bool:
    """orc_combine_partials over a (k, 864) uint8 array."""
    a = np.ascontiguousarray(parts, dtype=np.uint8).reshape(-1, 864)
    ok = ctypes.c_int(0)
    assert load().orc_combine_partials(a.shape[0], a.ctypes.data_as(ctypes.c_void_p), ctypes.byref(ok)) == 0
    return bool(ok.value)


def batch_fallback(sigs, hashes, pks, codes: np.ndarray, threads: int = 1) -> None:
    """orc_batch_fallback: codes (int32, in place) still 0 -> the per-vote verify code."""
    s, sp = _arr(sigs, 96)
    h, hp = _arr(hashes, 32)
    p, pp = _arr(pks, 48)
    assert codes.dtype == np.int32 and codes.flags.c_contiguous
    assert load().orc_batch_fallback(s.shape[0], sp, hp, pp, codes.ctypes.data_as(ctypes.c_void_p), threads) == 0
