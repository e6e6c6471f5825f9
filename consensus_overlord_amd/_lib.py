"""ctypes binding of libovhip.so (include/ovhip.h). No fallback: if the HIP library is
missing or cannot be loaded, importing the product raises."""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# OVH_LIBPATH: an alternative build of the same library (diagnostic A/B runs only)
LIB_PATH = os.environ.get("OVH_LIBPATH") or os.path.join(_HERE, "libovhip.so")

_u8p = ctypes.c_char_p
_sz = ctypes.c_size_t
_szp = ctypes.POINTER(ctypes.c_size_t)
_vp = ctypes.c_void_p

# (name, restype, argtypes) -- mirrors include/ovhip.h
SIGNATURES = [
    ("ovh_create", _vp, [ctypes.c_int, _u8p, _sz, ctypes.c_uint32]),
    ("ovh_create_multi", _vp, [ctypes.POINTER(ctypes.c_int), ctypes.c_int, _u8p, _sz, ctypes.c_uint32]),
    ("ovh_multi_peer_matrix", ctypes.c_int, [_vp, _u8p, _sz]),
    ("ovh_destroy", None, [_vp]),
    ("ovh_device_count", ctypes.c_int, [_vp]),
    ("ovh_stream", _vp, [_vp]),
    ("ovh_sm3", ctypes.c_int, [_u8p, _sz, _u8p]),
    ("ovh_vote_digests_device", ctypes.c_int, [_vp, _sz, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("ovh_vote_digests", ctypes.c_int, [_vp, _sz, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("ovh_sk_parse", ctypes.c_int, [_vp, _u8p, _sz, _u8p]),
    ("ovh_sign", ctypes.c_int, [_vp, _u8p, _sz, _u8p, _sz, _u8p]),
    ("ovh_sk_to_pk", ctypes.c_int, [_vp, _u8p, _sz, _u8p]),
    ("ovh_verify", ctypes.c_int, [_vp, _u8p, _sz, _u8p, _sz, _u8p, _sz]),
    ("ovh_aggregate_sigs", ctypes.c_int, [_vp, _u8p, _szp, _sz, _u8p, _szp, _sz, _u8p]),
    ("ovh_aggregate_pks", ctypes.c_int, [_vp, _u8p, _szp, _sz, _u8p]),
    ("ovh_verify_aggregated", ctypes.c_int, [_vp, _u8p, _sz, _u8p, _sz, _u8p, _szp, _sz]),
    ("ovh_set_validators", ctypes.c_int, [_vp, _u8p, _sz]),
    ("ovh_verify_batch", ctypes.c_int, [_vp, _sz, _u8p, _u8p, _u8p, _vp]),
    ("ovh_prefetch", ctypes.c_int, [_vp, _sz, _u8p, _u8p, _u8p]),
    ("ovh_cache_config", ctypes.c_int, [_vp, _sz]),
    ("ovh_cache_stats", ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_uint64)]),
    ("ovh_msg_cache_stats", ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_uint64)]),
    ("ovh_samemsg_stats", ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_uint64)]),
    ("ovh_verify_qc_batch", ctypes.c_int, [_vp, _sz, _u8p, _u8p, _u8p, _sz, _vp]),
    ("ovh_set_test_rlc", ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.c_uint64]),
    ("ovh_verify_batch_device", ctypes.c_int, [_vp, _sz, _vp, _vp, _vp, _vp]),
    ("ovh_batch_partial_device", ctypes.c_int, [_vp, _sz, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("ovh_combine_partials_device", ctypes.c_int, [_vp, _sz, _vp, ctypes.POINTER(ctypes.c_int32)]),
    ("ovh_batch_fallback_device", ctypes.c_int, [_vp, _sz, _vp]),
    ("ovh_verify_batch_device_async", ctypes.c_int, [_vp, _sz, _vp, _vp, _vp, _vp]),
    ("ovh_verify_samemsg_device_async", ctypes.c_int, [_vp, _sz, _vp, _vp, _vp, _vp]),
    ("ovh_vote_spans", ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_float), _sz]),
    ("ovh_verify_batch_async", ctypes.c_int, [_vp, _sz, _vp, _vp, _vp, _vp]),
    ("ovh_batch_wait", ctypes.c_int, [_vp]),
    ("ovh_combine_partials_device_async", ctypes.c_int, [_vp, _sz, _vp, _sz, _vp, _vp]),
    ("ovh_stage_times", ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_float), _sz]),
    ("ovh_stage_name", ctypes.c_char_p, [ctypes.c_int]),
    ("ovh_vm_trace", ctypes.c_int, [_vp, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64), _sz]),
    ("ovh_vm_clock", ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_uint64), _sz]),
    ("ovh_pool_log", ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_uint64), _sz]),
    ("ovh_diag_vm_occupancy", ctypes.c_int, [_vp, ctypes.c_int, _sz, ctypes.c_int, ctypes.c_int,
                                             ctypes.POINTER(ctypes.c_float)]),
    ("ovh_sign_batch_device", ctypes.c_int, [_vp, _sz, _vp, _vp, _vp]),
    ("ovh_sk_to_pk_batch_device", ctypes.c_int, [_vp, _sz, _vp, _vp]),
]

_lib = None


def load():
    """Load libovhip.so (raises OSError/RuntimeError if it is missing: no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            "libovhip.so not built (%s): run `make -C consensus_overlord_amd` or __graft_entry__.build()" % LIB_PATH)
    # One HIP runtime per process: torch (ROCm wheel) bundles its own libamdhip64.so.7. If it
    # is importable, load it first so libovhip's NEEDED libamdhip64.so.7 binds to that copy
    # and torch tensors / RCCL and libovhip share device contexts. Without torch, libovhip
    # binds to the system ROCm runtime (RUNPATH).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(LIB_PATH)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib
