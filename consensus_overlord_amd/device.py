"""Device-resident batch entry points (HBM in, HBM out). torch provides the device memory
only; every kernel is libovhip's. The library runs on its own HIP streams; the synchronous
calls return after their work completed, so callers synchronise torch's stream before handing
buffers over. The multi-GPU pair (batch_partial / combine_partials_async) is stream-ordered
with torch's current stream instead (include/ovhip.h)."""
from __future__ import annotations

import ctypes

import torch

from .crypto import Context, raise_for


def _ptr(t: torch.Tensor) -> ctypes.c_void_p:
    assert t.is_cuda and t.is_contiguous()
    return ctypes.c_void_p(t.data_ptr())


def sk_to_pk_batch(ctx: Context, sks: torch.Tensor) -> torch.Tensor:
    """sks: (n, 32) uint8 on device -> (n, 48) compressed pks."""
    n = sks.shape[0]
    out = torch.empty((n, 48), dtype=torch.uint8, device=sks.device)
    torch.cuda.synchronize(sks.device)
    raise_for(ctx.lib.ovh_sk_to_pk_batch_device(ctx.ptr, n, _ptr(sks), _ptr(out)))
    return out


def sign_batch(ctx: Context, sks: torch.Tensor, hashes: torch.Tensor) -> torch.Tensor:
    n = sks.shape[0]
    out = torch.empty((n, 96), dtype=torch.uint8, device=sks.device)
    torch.cuda.synchronize(sks.device)
    raise_for(ctx.lib.ovh_sign_batch_device(ctx.ptr, n, _ptr(sks), _ptr(hashes), _ptr(out)))
    return out


def verify_batch(ctx: Context, sigs: torch.Tensor, hashes: torch.Tensor, pks: torch.Tensor,
                 codes: torch.Tensor = None) -> torch.Tensor:
    n = sigs.shape[0]
    if codes is None:
        codes = torch.empty((n,), dtype=torch.int32, device=sigs.device)
    raise_for(ctx.lib.ovh_verify_batch_device(ctx.ptr, n, _ptr(sigs), _ptr(hashes), _ptr(pks), _ptr(codes)))
    return codes


def _stream(stream):
    if stream is None:
        return None
    if stream is True:
        stream = torch.cuda.current_stream()
    return ctypes.c_void_p(stream.cuda_stream)


def batch_partial(ctx: Context, sigs, hashes, pks, codes: torch.Tensor, partial: torch.Tensor, stream=None) -> None:
    """Per-shard partial (864 bytes: Fp12 Miller product + projective G2 sum) into `partial`.
    stream: None -> synchronous; True / a torch stream -> ordered on that stream."""
    n = sigs.shape[0]
    raise_for(ctx.lib.ovh_batch_partial_device(ctx.ptr, n, _ptr(sigs), _ptr(hashes), _ptr(pks), _ptr(codes),
                                               _ptr(partial), _stream(stream)))


def combine_partials(ctx: Context, partials: torch.Tensor) -> bool:
    """partials: (k, 864) uint8 on device -> combined check passed?"""
    k = partials.shape[0]
    v = ctypes.c_int32(-1)
    raise_for(ctx.lib.ovh_combine_partials_device(ctx.ptr, k, _ptr(partials), ctypes.byref(v)))
    return v.value == 1


def batch_fallback(ctx: Context, n: int, codes: torch.Tensor) -> None:
    raise_for(ctx.lib.ovh_batch_fallback_device(ctx.ptr, n, _ptr(codes)))


def verify_batch_async(ctx: Context, sigs: torch.Tensor, hashes: torch.Tensor, pks: torch.Tensor,
                       codes: torch.Tensor) -> None:
    """Enqueue one batch (ovh_verify_batch_device_async); `codes` is final after batch_wait."""
    n = sigs.shape[0]
    raise_for(ctx.lib.ovh_verify_batch_device_async(ctx.ptr, n, _ptr(sigs), _ptr(hashes), _ptr(pks), _ptr(codes)))


def verify_samemsg_async(ctx: Context, sigs: torch.Tensor, digest: bytes, pks: torch.Tensor,
                         codes: torch.Tensor) -> None:
    """Enqueue one batch of votes that all sign `digest` (ovh_verify_samemsg_device_async);
    `codes` is final after batch_wait."""
    if len(digest) != 32:
        raise ValueError("digest must be 32 bytes")
    n = sigs.shape[0]
    raise_for(ctx.lib.ovh_verify_samemsg_device_async(ctx.ptr, n, _ptr(sigs), digest, _ptr(pks), _ptr(codes)))


def combine_partials_async(ctx: Context, partials: torch.Tensor, n: int, codes: torch.Tensor, stream=None) -> None:
    """Enqueue the combined check of the gathered partials (stream-ordered after the gather on
    `stream`) and, device-gated on its verdict, the bisection of this rank's last partial's n
    votes into `codes` (final after batch_wait)."""
    raise_for(ctx.lib.ovh_combine_partials_device_async(ctx.ptr, partials.shape[0], _ptr(partials), n,
                                                        _ptr(codes), _stream(stream)))


def batch_wait(ctx: Context) -> None:
    raise_for(ctx.lib.ovh_batch_wait(ctx.ptr))
