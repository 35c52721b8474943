"""Object assembly: generate_object (src/data_gen.rs:29-94) and format builders.

    ObjectType / DataGenMode / Config      src/config.rs:10-152
    generate_object(cfg, seed=None)        src/data_gen.rs:29-94
    generate_random_data(size)             src/data_gen.rs:102-132 (seeded analogue layout)
    build_raw / build_tfrecord(_with_index) / build_npz
                                           src/data_formats/{raw,tfrecord,npz}.rs

Payloads come from the gfx950 kernels via the C ABI; framing is assembled by
the C++ layer (libs3dlio_amd.so).
"""
from __future__ import annotations

import ctypes
import enum
from dataclasses import dataclass

import numpy as np

from . import hostbuf
from ._lib import c_u64, call


class ObjectType(enum.IntEnum):
    """src/config.rs:10-17 (values are the C ABI's S3DG_OBJ_*)."""
    NPZ = 0
    TFRECORD = 1
    HDF5 = 2
    RAW = 3

    @classmethod
    def from_str(cls, s: str) -> "ObjectType":
        """src/s3_utils.rs:362-371: unknown names (e.g. "zeros") map to RAW."""
        return {"NPZ": cls.NPZ, "TFRECORD": cls.TFRECORD, "HDF5": cls.HDF5}.get(s.upper(), cls.RAW)


class DataGenMode(enum.IntEnum):
    """src/config.rs:35-41."""
    STREAMING = 0
    SINGLE_PASS = 1


@dataclass
class Config:
    """src/config.rs:97-111."""
    object_type: ObjectType
    elements: int
    element_size: int
    use_controlled: bool
    dedup_factor: int
    compress_factor: int
    data_gen_mode: DataGenMode = DataGenMode.STREAMING
    chunk_size: int = 256 * 1024

    @classmethod
    def new_with_defaults(cls, object_type, elements: int, element_size: int,
                          dedup_factor: int, compress_factor: int) -> "Config":
        """src/config.rs:115-133: use_controlled = dedup != 1 or compress != 1."""
        if isinstance(object_type, str):
            object_type = ObjectType.from_str(object_type)
        return cls(ObjectType(object_type), int(elements), int(element_size),
                   dedup_factor != 1 or compress_factor != 1, int(dedup_factor),
                   int(compress_factor))

    def with_data_gen_mode(self, mode: DataGenMode) -> "Config":
        self.data_gen_mode = DataGenMode(mode)
        return self

    def with_chunk_size(self, chunk_size: int) -> "Config":
        self.chunk_size = int(chunk_size)
        return self


def object_size(object_type, elements: int, element_size: int) -> int:
    out = c_u64()
    call("s3dg_object_size", int(ObjectType(object_type)), int(elements), int(element_size),
         ctypes.byref(out))
    return out.value


def generate_object(cfg: Config, seed: int | None = None):
    """Build one object payload (read-only buffer).  seed=None reproduces the
    reference's non-deterministic entropy; an int makes it reproducible."""
    n = object_size(cfg.object_type, cfg.elements, cfg.element_size)
    out = hostbuf.empty(n)
    w = c_u64()
    call("s3dg_generate_object", int(cfg.object_type), cfg.elements, cfg.element_size,
         1 if cfg.use_controlled else 0, max(0, cfg.dedup_factor), max(0, cfg.compress_factor),
         int(cfg.data_gen_mode), 0 if seed is None else 1,
         0 if seed is None else int(seed) & (2**64 - 1), int(out.ctypes.data) if n else 0, n,
         ctypes.byref(w))
    return hostbuf.readonly(out)


def generate_random_data(size: int) -> bytes:
    """src/data_gen.rs:102: time entropy, per-process random BASE_BLOCK."""
    out = np.empty(max(size, 1), np.uint8)
    if size:
        call("s3dlio_generate_random_data", int(out.ctypes.data), int(size))
    return out[:size].tobytes()


def build_raw(data) -> bytes:
    """src/data_formats/raw.rs:7-9 (a copy)."""
    return bytes(data)


def build_tfrecord_with_index(records: int, record_size: int, data) -> tuple[bytes, bytes]:
    """src/data_formats/tfrecord.rs:47-75."""
    src = np.frombuffer(memoryview(data).cast("B"), np.uint8)
    if src.size < records * record_size:
        raise ValueError("data shorter than records * record_size")
    out = np.empty(max(1, records * (16 + record_size)), np.uint8)
    idx = np.empty(max(1, 16 * records), np.uint8)
    call("s3dg_build_tfrecord", int(records), int(record_size), int(src.ctypes.data),
         int(out.ctypes.data), int(idx.ctypes.data))
    return out[:records * (16 + record_size)].tobytes(), idx[:16 * records].tobytes()


def build_tfrecord(records: int, record_size: int, data) -> bytes:
    """src/data_formats/tfrecord.rs:36-38."""
    return build_tfrecord_with_index(records, record_size, data)[0]


def build_npz(elements: int, element_size: int, data) -> bytes:
    """src/data_formats/npz.rs:114-132 ("data.npy", '|u1', shape (elements,))."""
    src = np.frombuffer(memoryview(data).cast("B"), np.uint8)
    n = c_u64()
    call("s3dg_npz_legacy_size", int(elements), int(src.size), ctypes.byref(n))
    out = np.empty(n.value, np.uint8)
    call("s3dg_build_npz", int(elements), int(src.ctypes.data) if src.size else 0, int(src.size),
         int(out.ctypes.data), n.value)
    return out.tobytes()
