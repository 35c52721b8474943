"""ctypes binding of libs3dlio_amd.so (the C ABI in include/s3dlio_gpu.h).

The library is built in-tree by s3dlio_amd/build.py.  There is no fallback:
if the .so is missing or cannot be loaded, importing this module raises.

HIP runtime: PyTorch-ROCm ships its own libamdhip64.so.7 (same SONAME as
/opt/rocm's).  When torch is importable we import it first so the dynamic
loader binds our library to torch's already-loaded runtime and the process
holds exactly one HIP runtime — then torch streams/events/tensors and this
library share devices, streams and pointers.
"""
from __future__ import annotations

import ctypes
import os

try:  # one HIP runtime per process (see module docstring)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the product
    torch = None

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("S3DLIO_AMD_LIB") or os.path.join(HERE, "libs3dlio_amd.so")   # override: A/B diagnostics
if os.environ.get("S3DLIO_AMD_LIB"):   # never silently: the override is named on stderr
    import sys as _sys
    print(f"s3dlio_amd: S3DLIO_AMD_LIB override: loading {LIB_PATH}", file=_sys.stderr)

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"{LIB_PATH} is missing: build it with `python -m s3dlio_amd.build` "
        "(hipcc --offload-arch=gfx950). There is no CPU fallback.")

_L = ctypes.CDLL(LIB_PATH)

c_u64, c_u32, c_int, c_vp = ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p
c_u8p = ctypes.POINTER(ctypes.c_uint8)


class ObjDesc(ctypes.Structure):
    """s3dg_obj_desc"""
    _fields_ = [("dst_off", c_u64), ("size", c_u64), ("entropy", c_u64), ("dedup", c_u64),
                ("f_num", c_u32), ("f_den", c_u32)]


class PutStats(ctypes.Structure):
    """s3dg_put_stats"""
    _fields_ = [("objects", c_u64), ("bytes", c_u64), ("seconds", ctypes.c_double),
                ("gpu_seconds", ctypes.c_double)]


# name -> (restype, argtypes); the exact export list of include/s3dlio_gpu.h
SIGNATURES = {
    "s3dg_ctx_create": (c_int, [c_int, ctypes.POINTER(c_vp)]),
    "s3dg_ctx_destroy": (c_int, [c_vp]),
    "s3dg_ctx_device": (c_int, [c_vp, ctypes.POINTER(c_int)]),
    "s3dg_set_base_block": (c_int, [c_vp, c_u8p]),
    "s3dg_set_base_block_seed": (c_int, [c_vp, c_u64]),
    "s3dg_get_base_block": (c_int, [c_vp, c_u8p]),
    "s3dg_set_waves_per_block": (c_int, [c_vp, c_int]),
    "s3dg_set_nontemporal": (c_int, [c_vp, c_int]),
    "s3dg_set_store_policy": (c_int, [c_vp, c_int, c_int]),
    "s3dg_set_occupancy": (c_int, [c_vp, c_int, c_int]),
    "s3dg_set_batch_prefetch": (c_int, [c_vp, c_u32]),
    "s3dg_set_batch_pace": (c_int, [c_vp, c_int]),
    "s3dg_set_batch_tile": (c_int, [c_vp, c_u32]),
    "s3dg_set_batch_split": (c_int, [c_vp, c_int]),
    "s3dg_set_stream_tiles": (c_int, [c_vp, c_int]),
    "s3dg_query_occupancy": (c_int, [c_vp, c_int, ctypes.POINTER(c_int)]),
    "s3dg_set_keystream_shape": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_u64, c_int]),
    "s3dg_set_keystream_xcd_group": (c_int, [c_vp, c_int, c_u32]),
    "s3dg_set_keystream_persist": (c_int, [c_vp, c_int]),
    "s3dg_set_keystream_tail": (c_int, [c_vp, c_int]),
    "s3dg_set_dgen_zero_split": (c_int, [c_vp, c_int, c_int, c_int, c_int, c_int]),
    "s3dg_query_keystream_occupancy": (c_int, [c_vp, c_int, ctypes.POINTER(c_int)]),
    "s3dg_unique_blocks": (c_u64, [c_u64, c_u64]),
    "s3dg_zero_class": (c_int, [c_u32, c_u32]),
    "s3dg_query_zero_tune": (c_int, [c_vp, c_int, ctypes.POINTER(c_int), ctypes.POINTER(ctypes.c_double),
                                     ctypes.POINTER(ctypes.c_double), ctypes.POINTER(c_u64)]),
    "s3dg_compress_ratio": (c_int, [c_u64, ctypes.POINTER(c_u32), ctypes.POINTER(c_u32)]),
    "s3dg_object_entropy": (c_u64, [c_u64, c_u64]),
    "s3dg_random_data": (c_int, [c_vp, c_vp, c_u64, c_u64, c_vp]),
    "s3dg_fill_controlled": (c_int, [c_vp, c_vp, c_u64, c_u64, c_u32, c_u32, c_u64, c_vp]),
    "s3dg_fill_controlled_range": (c_int, [c_vp, c_vp, c_u64, c_u64, c_u64, c_u64, c_u32, c_u32,
                                           c_u64, c_vp]),
    "s3dg_fill_controlled_stream": (c_int, [c_vp, c_vp, c_u64, c_u64, c_u64, c_u64, c_u32, c_u32,
                                            c_u64, c_u64, c_vp]),
    "s3dg_fill_controlled_batch": (c_int, [c_vp, c_vp, ctypes.POINTER(ObjDesc), c_u64, c_vp]),
    "s3dg_write_ceiling": (c_int, [c_vp, c_vp, c_u64, c_u32, c_vp]),
    "s3dg_write_ceiling_tiled": (c_int, [c_vp, c_vp, c_u64, c_u32, c_vp]),
    "s3dg_write_ceiling_fill": (c_int, [c_vp, c_vp, c_u64, c_u32, c_vp]),
    "s3dg_xoshiro_fill": (c_int, [c_vp, c_vp, c_u64, c_u64, c_u64, c_vp]),
    "s3dg_xoshiro_jump": (c_int, [ctypes.POINTER(c_u64), c_u64]),
    "s3dg_dgen_fill": (c_int, [c_vp, c_vp, c_u64, c_u64, c_u64, c_u64, c_u32, c_u32, c_u64, c_vp]),
    "s3dg_dgen_fill_stream": (c_int, [c_vp, c_vp, c_u64, c_u64, c_u64, c_u64, c_u32, c_u32, c_u64, c_u64, c_vp]),
    "s3dg_gen_create": (c_int, [c_u64, c_u64, c_u64, c_int, c_u64, ctypes.POINTER(c_vp)]),
    "s3dg_gen_create_ratio": (c_int, [c_u64, c_u64, c_u32, c_u32, c_int, c_u64,
                                      ctypes.POINTER(c_vp)]),
    "s3dg_gen_destroy": (c_int, [c_vp]),
    "s3dg_gen_fill_chunk": (c_int, [c_vp, c_vp, c_u64, ctypes.POINTER(c_u64)]),
    "s3dg_gen_fill_at": (c_int, [c_vp, c_vp, c_u64, c_u64]),
    "s3dg_gen_is_complete": (c_int, [c_vp]),
    "s3dg_gen_position": (c_u64, [c_vp]),
    "s3dg_gen_total_size": (c_u64, [c_vp]),
    "s3dg_gen_seed": (c_u64, [c_vp]),
    "s3dg_gen_reset": (c_int, [c_vp]),
    "s3dg_gen_slot": (c_int, [c_vp]),
    "s3dg_host_parse_devices": (c_int, [ctypes.c_char_p, ctypes.c_char_p, c_int, ctypes.POINTER(c_int), c_int,
                                        ctypes.POINTER(c_int)]),
    "s3dg_host_parse_devices_env": (c_int, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, c_int,
                                            ctypes.POINTER(c_int), c_int, ctypes.POINTER(c_int)]),
    "s3dg_host_slot_count": (c_int, [ctypes.POINTER(c_int)]),
    "s3dg_stream_release": (c_int, [c_vp, c_vp]),
    "s3dg_stream_state_count": (c_int, [c_vp, ctypes.POINTER(c_u64)]),
    "s3dg_host_slot_device": (c_int, [c_int, ctypes.POINTER(c_int)]),
    "s3dg_host_slot_context": (c_int, [c_int, ctypes.POINTER(c_vp)]),
    "s3dg_generate_data": (c_int, [c_vp, c_u64, c_u64, c_u64, c_int, c_u64]),
    "s3dg_crc32": (c_int, [c_vp, c_vp, c_u64, c_vp, ctypes.POINTER(c_u32)]),
    "s3dg_crc32_combine": (c_u32, [c_u32, c_u32, c_u64]),
    "s3dg_crc32_host": (c_u32, [c_u32, c_vp, c_u64]),
    "s3dg_npz_size": (c_int, [ctypes.POINTER(c_u64), c_int, ctypes.c_char_p, c_u64,
                              ctypes.POINTER(c_u64)]),
    "s3dg_npz_build": (c_int, [c_vp, ctypes.POINTER(c_u64), c_int, ctypes.c_char_p, c_u64, c_vp,
                               c_u64]),
    "s3dg_device_alloc": (c_int, [c_vp, c_u64, ctypes.POINTER(c_vp)]),
    "s3dg_device_free": (c_int, [c_vp, c_vp]),
    "s3dg_host_alloc_pinned": (c_int, [c_u64, ctypes.POINTER(c_vp)]),
    "s3dg_host_free_pinned": (c_int, [c_vp]),
    "s3dg_host_register": (c_int, [c_vp, c_u64]),
    "s3dg_host_unregister": (c_int, [c_vp]),
    "s3dg_host_alloc_pinned_local": (c_int, [c_int, c_u64, ctypes.POINTER(c_vp)]),
    "s3dg_device_numa_node": (c_int, [c_int, ctypes.POINTER(c_int)]),
    "s3dg_d2h_async": (c_int, [c_vp, c_vp, c_vp, c_u64, c_vp]),
    "s3dg_h2d_async": (c_int, [c_vp, c_vp, c_vp, c_u64, c_vp]),
    "s3dg_stream_create": (c_int, [c_vp, ctypes.POINTER(c_vp)]),
    "s3dg_stream_destroy": (c_int, [c_vp, c_vp]),
    "s3dg_sync": (c_int, [c_vp, c_vp]),
    "s3dg_device_count": (c_int, [ctypes.POINTER(c_int)]),
    "s3dlio_fill_controlled_data": (c_int, [c_vp, ctypes.c_size_t, ctypes.c_size_t,
                                            ctypes.c_size_t]),
    "s3dlio_fill_controlled_data_seeded": (c_int, [c_vp, ctypes.c_size_t, ctypes.c_size_t,
                                                   ctypes.c_size_t, c_u64, c_u8p]),
    "s3dg_object_size": (c_int, [c_int, c_u64, c_u64, ctypes.POINTER(c_u64)]),
    "s3dg_generate_object": (c_int, [c_int, c_u64, c_u64, c_int, c_u64, c_u64, c_int, c_int, c_u64,
                                     c_vp, c_u64, ctypes.POINTER(c_u64)]),
    "s3dg_build_tfrecord": (c_int, [c_u64, c_u64, c_vp, c_vp, c_vp]),
    "s3dg_npz_legacy_size": (c_int, [c_u64, c_u64, ctypes.POINTER(c_u64)]),
    "s3dg_build_npz": (c_int, [c_u64, c_vp, c_u64, c_vp, c_u64]),
    "s3dlio_generate_random_data": (c_int, [c_vp, ctypes.c_size_t]),
    "s3dg_put_objects": (c_int, [c_vp, ctypes.POINTER(ctypes.c_char_p), c_u64, c_u64, c_int, c_int,
                                 c_u64, c_u32, c_u32, c_u64, c_u32, c_vp, ctypes.POINTER(PutStats)]),
    "s3dg_put_objects_multi": (c_int, [ctypes.POINTER(c_vp), c_u32, ctypes.POINTER(ctypes.c_char_p), c_u64,
                                       c_u64, c_int, c_int, c_u64, c_u32, c_u32, c_u64, c_u32, c_vp,
                                       ctypes.POINTER(PutStats)]),
    "s3dg_last_error": (ctypes.c_char_p, []),
    "s3dg_version": (ctypes.c_char_p, []),
    "s3dg_build_digest": (ctypes.c_char_p, []),
}

for _name, (_res, _args) in SIGNATURES.items():
    _f = getattr(_L, _name)   # AttributeError here = the .so does not export the ABI
    _f.restype, _f.argtypes = _res, _args

lib = _L


class S3dgError(RuntimeError):
    """A failed C-ABI call (negative status); message from s3dg_last_error()."""

    def __init__(self, fn: str, code: int):
        msg = (_L.s3dg_last_error() or b"").decode(errors="replace")
        super().__init__(f"{fn} failed ({code}): {msg}")
        self.code = code


def check(fn: str, code: int) -> None:
    if code != 0:
        if code == -1:
            raise ValueError((_L.s3dg_last_error() or b"").decode(errors="replace"))
        if code == -4:   # S3DG_EIO
            raise OSError((_L.s3dg_last_error() or b"").decode(errors="replace"))
        raise S3dgError(fn, code)


def call(fn: str, *args) -> None:
    check(fn, getattr(_L, fn)(*args))
