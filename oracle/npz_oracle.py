"""Independent restatement of generate_npz_bytes_raw (TEST INFRASTRUCTURE ONLY).

Follows /root/reference/src/data_formats/npz.rs:216-434 with Python's
struct/zlib (zlib.crc32 is the same IEEE CRC-32 as crc32fast) and the C
oracle's keystream for the x-array (npz.rs:376-383).  Parity of the framing
is pinned by construction against the reference's own code; the keystream by
the PRNG KATs.  Validated further by numpy.load / zipfile reading the result.
"""
from __future__ import annotations

import struct
import zlib

from . import oracle_c


def npy_header(shape, dtype: str) -> bytes:                    # npz.rs:216-241
    dims = ", ".join(str(int(d)) for d in shape)
    tup = f"({dims},)" if len(shape) == 1 else f"({dims})"
    d = "{'descr': '" + dtype + "', 'fortran_order': False, 'shape': " + tup + ", }"
    hl = len(d) + 1
    pad = (64 - ((6 + 2 + 2 + hl) % 64)) % 64
    return b"\x93NUMPY\x01\x00" + struct.pack("<H", hl + pad) + d.encode() + b" " * pad + b"\n"


def dtype_element_size(dtype: str) -> int:                      # npz.rs:244-252
    for ch in reversed(dtype):
        if ch.isdigit():
            return int(ch)
    return 4


def local_header(name: bytes, crc: int, size: int) -> bytes:   # npz.rs:256-270
    return (b"PK\x03\x04" + struct.pack("<HHHHHIIIHH", 20, 0, 0, 0, 0, crc, size, size, len(name), 0)
            + name)


def central_entry(name: bytes, size: int, crc: int, off: int) -> bytes:   # npz.rs:273-297
    return (b"PK\x01\x02" + struct.pack("<HHHHHHIIIHHHHHII", 20, 20, 0, 0, 0, 0, crc, size, size,
                                        len(name), 0, 0, 0, 0, 0, off) + name)


def generate_npz_bytes_raw(shape, dtype: str = "<f4", num_samples: int = 1) -> bytes:
    hx = npy_header(shape, dtype)
    hy = npy_header([num_samples], "<i8")
    n = 1
    for d in shape:
        n *= int(d)
    x_data = bytes(oracle_c.xoshiro_chunks(n * dtype_element_size(dtype), 2 * 1024 * 1024, 0)) \
        if n * dtype_element_size(dtype) else b""
    x_npy = hx + x_data
    y_npy = hy + bytes(num_samples * 8)
    crc_x, crc_y = zlib.crc32(x_npy), zlib.crc32(y_npy)
    m32 = 0xFFFFFFFF
    lx = local_header(b"x.npy", crc_x, len(x_npy) & m32) + x_npy
    off_y = len(lx)
    ly = local_header(b"y.npy", crc_y, len(y_npy) & m32) + y_npy
    cd = central_entry(b"x.npy", len(x_npy) & m32, crc_x, 0) + \
        central_entry(b"y.npy", len(y_npy) & m32, crc_y, off_y)
    off_cd = len(lx) + len(ly)
    eocd = b"PK\x05\x06" + struct.pack("<HHHHIIH", 0, 0, 2, 2, len(cd), off_cd & m32, 0)
    return lx + ly + cd + eocd
