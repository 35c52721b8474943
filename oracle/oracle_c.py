"""ctypes wrapper around the C oracle (oracle/s3dg_oracle.c).

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "s3dg_oracle.c")
LIB = os.path.join(HERE, "_build", "libs3dg_oracle.so")

u64 = ctypes.c_uint64
u8p = ctypes.POINTER(ctypes.c_uint8)


def build(force: bool = False) -> str:
    """Compile the oracle with gcc (portable x86-64-v2 code: the .so travels
    to the GPU box, whose CPU may differ from this container's)."""
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        subprocess.check_call(["gcc", "-O3", "-march=x86-64-v2", "-std=c11", "-fPIC",
                               "-shared", "-Wall", "-o", LIB, SRC, "-lpthread", "-lm"])
    return LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        L.s3dgo_splitmix64_next.argtypes = [ctypes.POINTER(u64)]
        L.s3dgo_splitmix64_next.restype = u64
        L.s3dgo_xoshiro_seed.argtypes = [ctypes.POINTER(u64), u64]
        L.s3dgo_xoshiro_next.argtypes = [ctypes.POINTER(u64)]
        L.s3dgo_xoshiro_next.restype = u64
        L.s3dgo_fill_bytes.argtypes = [ctypes.POINTER(u64), u8p, ctypes.c_size_t]
        L.s3dgo_base_block.argtypes = [u64, u8p]
        L.s3dgo_unique_blocks.argtypes = [u64, u64]
        L.s3dgo_unique_blocks.restype = u64
        L.s3dgo_fill_controlled.argtypes = [u8p, u64, u64, u64, u64, u64, u8p]
        L.s3dgo_object_entropy.argtypes = [u64, u64]
        L.s3dgo_object_entropy.restype = u64
        L.s3dgo_fill_stream.argtypes = [u8p, u64, u64, u64, u64, u64, u64, u64, u64, u8p]
        L.s3dgo_fill_stream_mt.argtypes = [u8p, u64, u64, u64, u64, u64, u64, u64, u64,
                                           u8p, ctypes.c_int]
        L.s3dgo_fill_stream_mt.restype = ctypes.c_int
        L.s3dgo_pool_fill_controlled.argtypes = [u8p, u64, u64, u64, u64, u64, u8p, ctypes.c_int]
        L.s3dgo_pool_fill_controlled.restype = ctypes.c_int
        L.s3dgo_xoshiro_chunks.argtypes = [u8p, u64, u64, u64]
        L.s3dgo_dgen_fill.argtypes = [u8p, u64, u64, u64, u64, u64]
        L.s3dgo_random_data.argtypes = [u8p, u64, u64, u8p]
        L.s3dgo_dgen_stream_init.argtypes = [ctypes.c_void_p, u64, u64, u64, u64, u64]
        L.s3dgo_dgen_stream_fill.argtypes = [ctypes.c_void_p, u8p, u64]
        L.s3dgo_dgen_stream_fill.restype = u64
        L.s3dgo_dgen_chunk_bench.argtypes = [ctypes.c_int, u64, u64, u64, u64, u64, u64, ctypes.c_double,
                                             ctypes.POINTER(ctypes.c_double)]
        L.s3dgo_dgen_chunk_bench.restype = u64
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(u8p)


def splitmix64(state: int, n: int) -> list[int]:
    x = u64(state)
    return [lib().s3dgo_splitmix64_next(ctypes.byref(x)) for _ in range(n)]


def xoshiro_stream(state, n: int) -> list[int]:
    s = (u64 * 4)(*state)
    return [lib().s3dgo_xoshiro_next(s) for _ in range(n)]


def xoshiro_seeded_stream(seed: int, n: int) -> list[int]:
    s = (u64 * 4)()
    lib().s3dgo_xoshiro_seed(s, seed)
    return [lib().s3dgo_xoshiro_next(s) for _ in range(n)]


def base_block(seed: int) -> np.ndarray:
    out = np.empty(4096, np.uint8)
    lib().s3dgo_base_block(seed, _ptr(out))
    return out


def unique_blocks(nblocks: int, dedup: int) -> int:
    return lib().s3dgo_unique_blocks(nblocks, dedup)


def object_entropy(seed_base: int, j: int) -> int:
    return lib().s3dgo_object_entropy(seed_base, j)


def fill_controlled(length: int, dedup: int, f_num: int, f_den: int, entropy: int,
                    base: np.ndarray) -> np.ndarray:
    out = np.empty(length, np.uint8)
    base = np.ascontiguousarray(base, np.uint8)
    lib().s3dgo_fill_controlled(_ptr(out), length, dedup, f_num, f_den, entropy, _ptr(base))
    return out


def pool_fill_controlled(out: np.ndarray, dedup: int, f_num: int, f_den: int, entropy: int,
                         base: np.ndarray, threads: int) -> int:
    """One fill_controlled_data call on `out` over a persistent thread pool
    (the CPU baseline of the reference's criterion shape); returns threads used."""
    base = np.ascontiguousarray(base, np.uint8)
    return lib().s3dgo_pool_fill_controlled(_ptr(out), out.size, dedup, f_num, f_den,
                                            entropy & (2**64 - 1), _ptr(base), threads)


def fill_stream(obj_size: int, n: int, dedup: int, f_num: int, f_den: int,
                seed_base: int, first_obj: int, base: np.ndarray,
                stride: int | None = None, threads: int = 1,
                out: np.ndarray | None = None) -> np.ndarray:
    stride = obj_size if stride is None else stride
    if out is None:
        out = np.zeros(stride * n, np.uint8)
    base = np.ascontiguousarray(base, np.uint8)
    if threads > 1:
        lib().s3dgo_fill_stream_mt(_ptr(out), obj_size, stride, n, dedup, f_num, f_den,
                                   seed_base, first_obj, _ptr(base), threads)
    else:
        lib().s3dgo_fill_stream(_ptr(out), obj_size, stride, n, dedup, f_num, f_den,
                                seed_base, first_obj, _ptr(base))
    return out


def xoshiro_chunks(length: int, chunk: int, seed_base: int, out: np.ndarray | None = None) -> np.ndarray:
    out = np.empty(length, np.uint8) if out is None else out
    lib().s3dgo_xoshiro_chunks(_ptr(out), length, chunk, seed_base)
    return out


def dgen_fill(size: int, dedup: int, f_num: int, f_den: int, seed: int,
              out: np.ndarray | None = None) -> np.ndarray:
    out = np.empty(size, np.uint8) if out is None else out
    lib().s3dgo_dgen_fill(_ptr(out), size, dedup, f_num, f_den, seed & (2**64 - 1))
    return out


def random_data(size: int, entropy: int, base: np.ndarray) -> np.ndarray:
    out = np.empty(size, np.uint8)
    base = np.ascontiguousarray(base, np.uint8)
    lib().s3dgo_random_data(_ptr(out), size, entropy & (2**64 - 1), _ptr(base))
    return out


def dgen_stream(size: int, dedup: int, f_num: int, f_den: int, seed: int, chunk: int) -> np.ndarray:
    """DG1 produced chunk by chunk by the CPU streaming port (s3dgo_dgen_stream_fill)."""
    st = (ctypes.c_uint64 * 16)()
    lib().s3dgo_dgen_stream_init(st, size, dedup, f_num, f_den, seed & (2**64 - 1))
    out = np.empty(size, np.uint8)
    pos = 0
    while pos < size:
        w = lib().s3dgo_dgen_stream_fill(st, ctypes.cast(out.ctypes.data + pos, ctypes.POINTER(ctypes.c_uint8)),
                                         chunk)
        if w == 0:
            break
        pos += w
    return out


def dgen_chunk_bench(threads: int, obj_size: int, chunk: int, dedup: int, f_num: int, f_den: int,
                     seed_base: int, seconds: float) -> tuple[int, float]:
    """(bytes, elapsed s) of `threads` CPU threads streaming DG1 objects chunk by chunk."""
    el = ctypes.c_double()
    b = lib().s3dgo_dgen_chunk_bench(threads, obj_size, chunk, dedup, f_num, f_den, seed_base & (2**64 - 1),
                                     seconds, ctypes.byref(el))
    return b, el.value
