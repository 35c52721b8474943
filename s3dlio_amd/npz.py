"""generate_npz_bytes (src/python_api/python_datagen_api.rs:395-414 ->
src/data_formats/npz.rs:322-434) on the GPU.

The archive is byte-identical to the reference's: x.npy carries the K2
keystream (2 MiB chunks, chunk k = Xoshiro256++ seed_from_u64(k)), its CRC-32
is computed by the device CRC kernel, the ZIP/NPY framing on the host.
"""
from __future__ import annotations

import ctypes
import numpy as np

from . import hostbuf
from ._lib import c_u32, c_u64, call, lib
from .device import Context, _ptr, _stream, host_context

def default_context() -> Context:
    """The next host slot's context, round-robin (include/s3dlio_gpu.h host
    slots: every visible GPU unless S3DLIO_GPU_DEVICE / S3DLIO_GPU_DEVICES
    say otherwise); borrowed from the pool."""
    return host_context(-1)


def _shape_arr(shape):
    dims = [int(d) for d in shape]
    if any(d < 0 for d in dims):
        raise ValueError("shape dimensions must be >= 0")
    return (c_u64 * max(1, len(dims)))(*dims), len(dims)


def npz_size(shape, dtype: str = "<f4", num_samples: int = 1) -> int:
    arr, nd = _shape_arr(shape)
    out = c_u64()
    call("s3dg_npz_size", arr, nd, dtype.encode(), int(num_samples), ctypes.byref(out))
    return out.value


def generate_npz_bytes(shape, dtype: str = "<f4", num_samples: int = 1):
    """Return the NPZ archive as a read-only zero-copy buffer (BytesView)."""
    arr, nd = _shape_arr(shape)
    total = npz_size(shape, dtype, num_samples)
    out = hostbuf.empty(total)               # every byte is written by the builder
    try:
        call("s3dg_npz_build", default_context()._h, arr, nd, dtype.encode(), int(num_samples),
             int(out.ctypes.data), total)
    except Exception as e:   # the reference maps errors to RuntimeError (:409)
        raise RuntimeError(str(e)) from e
    return hostbuf.readonly(out)


def crc32_device(ctx: Context, dst, nbytes: int | None = None, stream=None) -> int:
    """CRC-32 (IEEE) of a device buffer, computed on the GPU."""
    n = int(dst.numel() * dst.element_size()) if nbytes is None else nbytes
    out = c_u32()
    call("s3dg_crc32", ctx._h, _ptr(dst), n, _stream(stream), ctypes.byref(out))
    return out.value


def crc32_combine(crc1: int, crc2: int, len2: int) -> int:
    return int(lib.s3dg_crc32_combine(crc1, crc2, len2))
