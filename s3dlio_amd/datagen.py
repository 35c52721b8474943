"""Mirror of s3dlio's datagen surface over the C ABI (dgen-contract "DG1" layout).

PyO3 surface (src/python_api/python_datagen_api.rs:49-435), same names,
defaults and errors:
    generate_data(size, dedup=1, compress=1) -> BytesView (read-only buffer)
    generate_data_with_threads(size, dedup=1, compress=1, threads=None)
    generate_into_buffer(buffer, dedup=1, compress=1, threads=None) -> int
    Generator(size, dedup=1, compress=1, threads=None, chunk_size=None, seed=None)
        .fill_chunk(buffer) -> int, .is_complete(), .reset(), .chunk_size
    py_default_data_gen_threads(), py_total_cpus()
Rust streaming API (src/data_gen.rs:232-371, src/data_gen_alt.rs:42-149):
    DataGenerator(seed=None).begin_object(size, dedup, compress) -> ObjectGen
    ObjectGen.fill_chunk(chunk_size) -> bytes | None, is_complete, reset,
        position, total_size, fill_remaining
    generate_controlled_data_streaming(size, dedup, compress, chunk_size)
    generate_controlled_data_alt(size, dedup, compress, seed=None)
    optimal_chunk_size(total_size)

The bytes come from the gfx950 keystream kernel (s3dg_dgen_fill) on the
default GPU; the reference's engine (dgen-data 0.2.4) is absent, so the layout
is build-defined and meets the statistical contract its tests pin (SURVEY.md
Appendix B): exact sizes, unique 1 MiB blocks ~ n/dedup, zero fraction
~ (c-1)/c, incompressible at c=1, seeded determinism, chunk-size invariance.
`threads` is accepted for signature compatibility and ignored (no CPU pool).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import hostbuf
from ._lib import c_u64, c_vp, call, lib
from .device import compress_ratio

DGEN_BLOCK_SIZE = 1 << 20                       # src/constants.rs:348
DEFAULT_CHUNK_SIZE = 32 << 20                   # Generator default chunk (python_datagen_api.rs:279)


def _writable(buffer) -> tuple[int, int]:
    mv = memoryview(buffer)
    if mv.readonly:
        raise ValueError("Buffer must be writable")
    if not mv.c_contiguous:
        raise ValueError("Buffer must be C-contiguous for zero-copy operation")
    n = mv.nbytes
    if n == 0:
        return 0, 0
    return int(np.frombuffer(mv.cast("B"), np.uint8).ctypes.data), n


class _Gen:
    """Owner of one s3dg_gen handle."""

    def __init__(self, size: int, dedup: int, compress, seed: int | None):
        if size < 0:
            raise ValueError("size must be >= 0")
        h = c_vp()
        if isinstance(compress, (int, np.integer)) and not isinstance(compress, bool):
            call("s3dg_gen_create", int(size), max(0, int(dedup)), max(0, int(compress)),
                 0 if seed is None else 1, 0 if seed is None else int(seed) & (2**64 - 1),
                 ctypes.byref(h))
        else:
            fn, fd = compress_ratio(compress)
            call("s3dg_gen_create_ratio", int(size), max(0, int(dedup)), fn, fd,
                 0 if seed is None else 1, 0 if seed is None else int(seed) & (2**64 - 1),
                 ctypes.byref(h))
        self.h = h

    def fill(self, ptr: int, n: int) -> int:
        w = c_u64()
        call("s3dg_gen_fill_chunk", self.h, ptr, n, ctypes.byref(w))
        return w.value

    def close(self):
        if getattr(self, "h", None):
            lib.s3dg_gen_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _new_bytes(size: int, dedup: int, compress, seed: int | None):
    out = hostbuf.empty(size)                # every byte is written by the generator
    if size:
        g = _Gen(size, dedup, compress, seed)
        try:
            g.fill(int(out.ctypes.data), size)
        finally:
            g.close()
    return hostbuf.readonly(out)             # BytesView: read-only, zero-copy buffer


# ---- PyO3 surface --------------------------------------------------------------

def generate_data(size: int, dedup: int = 1, compress: int = 1):
    """python_datagen_api.rs:49-74; returns a read-only zero-copy buffer view."""
    return _new_bytes(size, dedup, compress, None)


def generate_data_with_threads(size: int, dedup: int = 1, compress: int = 1, threads=None):
    """python_datagen_api.rs:95-123 (`threads` ignored: generation runs on the GPU)."""
    return _new_bytes(size, dedup, compress, None)


def generate_into_buffer(buffer, dedup: int = 1, compress: int = 1, threads=None) -> int:
    """python_datagen_api.rs:150-200: fill `buffer` in place, return its size."""
    ptr, n = _writable(buffer)
    if n:
        g = _Gen(n, dedup, compress, None)
        try:
            g.fill(ptr, n)
        finally:
            g.close()
    return n


def py_total_cpus() -> int:
    """src/hardware.rs:155 total_cpus (logical CPUs)."""
    return os.cpu_count() or 1


def py_default_data_gen_threads() -> int:
    """src/hardware.rs:279-304 recommended_data_gen_threads: all affinity CPUs."""
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        return py_total_cpus()


total_cpus = py_total_cpus
default_data_gen_threads = py_default_data_gen_threads


class Generator:
    """python_datagen_api.rs:270-365 (PyO3 class `Generator`)."""

    def __init__(self, size: int, dedup: int = 1, compress: int = 1, threads=None,
                 chunk_size: int | None = None, seed: int | None = None):
        self._g = _Gen(size, dedup, compress, seed)
        self._chunk = int(chunk_size) if chunk_size else DEFAULT_CHUNK_SIZE

    @property
    def chunk_size(self) -> int:
        return self._chunk

    def fill_chunk(self, buffer) -> int:
        mv = memoryview(buffer)
        if mv.readonly:
            raise ValueError("Buffer must be writable")
        if not mv.c_contiguous:
            raise ValueError("Buffer must be C-contiguous")
        if mv.nbytes == 0:
            return 0
        return self._g.fill(int(np.frombuffer(mv.cast("B"), np.uint8).ctypes.data), mv.nbytes)

    def is_complete(self) -> bool:
        return bool(lib.s3dg_gen_is_complete(self._g.h))

    def reset(self) -> None:
        call("s3dg_gen_reset", self._g.h)

    # extras of the Rust ObjectGen surface
    def position(self) -> int:
        return int(lib.s3dg_gen_position(self._g.h))

    def total_size(self) -> int:
        return int(lib.s3dg_gen_total_size(self._g.h))

    @property
    def slot(self) -> int:
        """Host slot this generator runs on (s3dg_gen_slot; not in the reference)."""
        return int(lib.s3dg_gen_slot(self._g.h))


# ---- Rust streaming API (src/data_gen.rs:232-371) ---------------------------------

class ObjectGen:
    """src/data_gen.rs:308-371 (wraps ObjectGenAlt, src/data_gen_alt.rs:89-149)."""

    def __init__(self, total_size: int, dedup: int, compress: int, entropy: int):
        self._g = _Gen(total_size, dedup, compress, entropy)

    def fill_chunk(self, chunk_size: int):
        if chunk_size <= 0:
            raise AssertionError("Chunk size must be greater than 0")   # :328
        n = min(chunk_size, self.total_size() - self.position())
        if n == 0:
            return None
        out = bytearray(n)
        w = self._g.fill(int(np.frombuffer(out, np.uint8).ctypes.data), n)
        return bytes(out[:w])

    def is_complete(self) -> bool:
        return bool(lib.s3dg_gen_is_complete(self._g.h))

    def reset(self) -> None:
        call("s3dg_gen_reset", self._g.h)

    def position(self) -> int:
        return int(lib.s3dg_gen_position(self._g.h))

    def total_size(self) -> int:
        return int(lib.s3dg_gen_total_size(self._g.h))

    def fill_remaining(self) -> bytes:
        out = []
        while not self.is_complete():
            c = self.fill_chunk(32 << 20)                                # :360
            if c is None:
                break
            out.append(c)
        return b"".join(out)


class DataGenerator:
    """src/data_gen.rs:253-305: seed None -> time + per-instance counter."""

    _counter = 0

    def __init__(self, seed: int | None = None):
        if seed is None:
            import time
            DataGenerator._counter += 1
            seed = (time.time_ns() + DataGenerator._counter) & (2**64 - 1)
        self.instance_entropy = int(seed)

    @classmethod
    def new(cls, seed: int | None = None) -> "DataGenerator":
        """DataGenerator::new(Option<u64>) (src/data_gen.rs:262-264)."""
        return cls(seed)

    @classmethod
    def new_with_seed(cls, seed: int) -> "DataGenerator":
        return cls(seed)

    @classmethod
    def default(cls) -> "DataGenerator":
        """impl Default for DataGenerator: new(None) (src/data_gen.rs:301-305)."""
        return cls(None)

    def begin_object(self, size: int, dedup: int, compress: int) -> ObjectGen:
        return ObjectGen(size, dedup, compress, self.instance_entropy)


def generate_controlled_data_streaming(size: int, dedup: int, compress: int,
                                       chunk_size: int) -> bytes:
    """src/data_gen.rs:232-249."""
    obj = DataGenerator(None).begin_object(size, dedup, compress)
    parts = []
    while not obj.is_complete():
        c = obj.fill_chunk(chunk_size)
        if c is None:
            break
        parts.append(c)
    return b"".join(parts)


def generate_controlled_data_alt(size: int, dedup: int, compress: int, seed: int | None = None):
    """src/data_gen_alt.rs:66-80 (dedup/compress .max(1))."""
    return _new_bytes(size, max(1, dedup), max(1, compress), seed)


def optimal_chunk_size(total_size: int) -> int:
    """src/data_gen_alt.rs:42-52."""
    for lim in (64 << 20, 32 << 20, 16 << 20):
        if total_size >= lim:
            return lim
    return total_size


# ---- data_gen_alt / dgen-data re-exports (src/data_gen_alt.rs:14-150) --------------

import enum as _enum
from dataclasses import dataclass as _dataclass


class NumaMode(_enum.Enum):
    """dgen_data::NumaMode -- accepted for signature compatibility; generation runs
    on the GPU, so there is no host NUMA placement to choose."""
    AUTO = "auto"
    FORCE = "force"
    DISABLED = "disabled"


@_dataclass
class GeneratorConfig:
    """dgen_data::GeneratorConfig (fields: python_datagen_api.rs:59-68)."""
    size: int
    dedup_factor: int = 1
    compress_factor: int = 1
    numa_mode: NumaMode = NumaMode.AUTO
    max_threads: int | None = None
    numa_node: int | None = None
    block_size: int | None = None
    seed: int | None = None

    def _check(self):
        if self.block_size not in (None, DGEN_BLOCK_SIZE):
            raise ValueError(f"block_size must be {DGEN_BLOCK_SIZE} (the DG1 layout's 1 MiB blocks)")
        if self.size < 0:
            raise ValueError("size must be >= 0")


class DataBuffer:
    """dgen_data::DataBuffer: owned generated bytes (.into_bytes(), .as_slice(), .as_ptr())."""

    def __init__(self, view):
        self._v = view            # BytesView

    def into_bytes(self):
        return self._v

    def as_slice(self) -> memoryview:
        return self._v.memoryview()

    def as_ptr(self) -> int:
        return int(np.frombuffer(self._v, np.uint8).ctypes.data) if len(self._v) else 0

    def __len__(self) -> int:
        return len(self._v)

    def __bytes__(self) -> bytes:
        return self._v.to_bytes()


def generate_data_from_config(config: GeneratorConfig) -> DataBuffer:
    """dgen_data::generate_data(GeneratorConfig) -> DataBuffer.  Unlike the
    reference's batch path (data_gen_alt.rs:63-64) the seed is honoured."""
    config._check()
    return DataBuffer(_new_bytes(config.size, max(1, config.dedup_factor),
                                 max(1, config.compress_factor), config.seed))


def generate_data_simple(size: int, dedup: int, compress: int) -> DataBuffer:
    """dgen_data::generate_data_simple."""
    return generate_data_from_config(GeneratorConfig(size, dedup, compress))


def generate_data_with_config(config: GeneratorConfig):
    """src/data_gen_alt.rs:56-59 (Bytes = read-only zero-copy BytesView)."""
    return generate_data_from_config(config).into_bytes()


class ObjectGenAlt:
    """src/data_gen_alt.rs:89-149: streaming generator over one object,
    fill_chunk(buf) writes into `buf` and returns the byte count (0 when done)."""

    def __init__(self, total_size: int, dedup: int, compress: int, seed: int | None = None):
        if seed is None:   # :98-104 system-time seed
            import time
            seed = time.time_ns() & (2**64 - 1)
        self._g = _Gen(total_size, max(1, dedup), max(1, compress), seed)

    @classmethod
    def new(cls, total_size: int, dedup: int, compress: int) -> "ObjectGenAlt":
        return cls(total_size, dedup, compress)

    @classmethod
    def new_with_seed(cls, total_size: int, dedup: int, compress: int, seed: int) -> "ObjectGenAlt":
        return cls(total_size, dedup, compress, seed)

    def fill_chunk(self, buf) -> int:
        ptr, n = _writable(buf)
        return self._g.fill(ptr, n) if n else 0

    def is_complete(self) -> bool:
        return bool(lib.s3dg_gen_is_complete(self._g.h))

    def reset(self) -> None:
        call("s3dg_gen_reset", self._g.h)

    def position(self) -> int:
        return int(lib.s3dg_gen_position(self._g.h))

    def total_size(self) -> int:
        return int(lib.s3dg_gen_total_size(self._g.h))
