"""TEST INFRASTRUCTURE ONLY — CPU restatement of s3dlio's object framing.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it.

    build_raw                 src/data_formats/raw.rs:7-9
    build_tfrecord(_with_index) src/data_formats/tfrecord.rs:10-75
        record = u64le len | masked_crc(len bytes) | data | masked_crc(data)
        masked_crc(c) = ((c >> 15) | (c << 17)) + 0xa282ead8 (mod 2^32)  :10-12
        index entry = u64le offset | u64le record length                  :60-66
    build_npz (legacy single-array)  src/data_formats/npz.rs:92-132
        "data.npy" ('|u1', shape (elements,)) in a stored ZIP.  The reference
        uses the `zip` crate's ZipWriter whose header fields (version-made-by,
        DOS time) are not pinned by any fixture; the build-defined layout here
         fixes them to: version 10/20, time 0, date 0x21.
        The reference test (tests/object_format_tests.rs:27-58) checks only the
        archive's structure and payload, which this layout satisfies.
Pinned by the reference's own fixtures in tests/object_format_tests.rs:19-125.
"""
from __future__ import annotations

import struct
import zlib


def masked_crc(crc: int) -> int:
    return ((((crc >> 15) | (crc << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def build_raw(data: bytes) -> bytes:
    return bytes(data)


def build_tfrecord_with_index(records: int, record_size: int, data: bytes) -> tuple[bytes, bytes]:
    out, idx = bytearray(), bytearray()
    lb = struct.pack("<Q", record_size)
    for i in range(records):
        d = bytes(data[i * record_size:(i + 1) * record_size])
        idx += struct.pack("<QQ", len(out), 16 + record_size)
        out += lb + struct.pack("<I", masked_crc(zlib.crc32(lb))) + d
        out += struct.pack("<I", masked_crc(zlib.crc32(d)))
    return bytes(out), bytes(idx)


def build_tfrecord(records: int, record_size: int, data: bytes) -> bytes:
    return build_tfrecord_with_index(records, record_size, data)[0]


def npy_header_u1(elements: int) -> bytes:
    """make_npy_header (npz.rs:92-109): padded so 10 + len(dict + '\\n') % 16 == 0."""
    d = "{'descr': '|u1', 'fortran_order': False, 'shape': (%d,)}" % elements
    d += " " * ((16 - (10 + len(d) + 1) % 16) % 16) + "\n"
    return b"\x93NUMPY\x01\x00" + struct.pack("<H", len(d)) + d.encode()


def build_npz(elements: int, data: bytes) -> bytes:
    npy = npy_header_u1(elements) + bytes(data)
    crc, n, name = zlib.crc32(npy), len(npy), b"data.npy"
    local = b"PK\x03\x04" + struct.pack("<HHHHHIIIHH", 10, 0, 0, 0, 0x21, crc, n, n, len(name), 0) + name
    cd = b"PK\x01\x02" + struct.pack("<HHHHHHIIIHHHHHII", 20, 10, 0, 0, 0, 0x21, crc, n, n,
                                      len(name), 0, 0, 0, 0, 0, 0) + name
    eocd = b"PK\x05\x06" + struct.pack("<HHHHIIH", 0, 0, 1, 1, len(cd), len(local) + n, 0)
    return local + npy + cd + eocd
