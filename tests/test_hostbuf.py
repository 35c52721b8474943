"""Recycled host output buffers (s3dlio_amd/hostbuf.py) -- host logic, no GPU."""
import gc

import pytest


def test_pool_recycles_after_last_view_dies():
    from s3dlio_amd import hostbuf
    n = 37 << 20                          # a size no other test uses
    a = hostbuf.empty(n)
    a[:] = 7
    addr = a.ctypes.data
    mv = hostbuf.readonly(a)
    del a
    gc.collect()
    b = hostbuf.empty(n)                  # mv still holds the first buffer
    addr_b = b.ctypes.data
    assert addr_b != addr
    del b
    gc.collect()
    m = memoryview(mv)
    assert bytes(m[:4]) == b"\x07" * 4 and bytes(m[-4:]) == b"\x07" * 4
    del m
    idle0 = hostbuf.pool_stats()["idle_buffers"]
    del mv
    gc.collect()
    assert hostbuf.pool_stats()["idle_buffers"] == idle0 + 1
    c, d = hostbuf.empty(n), hostbuf.empty(n)   # both come back from the pool
    assert {c.ctypes.data, d.ctypes.data} == {addr, addr_b}


def test_readonly_export_semantics():
    from s3dlio_amd import hostbuf
    a = hostbuf.empty(4096)
    bv = hostbuf.readonly(a)
    mv = memoryview(bv)
    assert mv.readonly and mv.nbytes == 4096 and len(bv) == 4096
    with pytest.raises(TypeError):
        mv[0] = 1
    import ctypes
    with pytest.raises((BufferError, TypeError)):     # writable export refused
        (ctypes.c_char * 4096).from_buffer(bv)
    import numpy as np
    assert not np.frombuffer(bv, np.uint8).flags.writeable


def test_bytesview_surface_like_reference():
    """tests/test_zero_copy.py of the reference: len, repr, memoryview() twice
    shares one pointer, to_bytes() is a copy, data outlives the last Python
    reference to the owner (python_core_api.rs:300-462)."""
    import numpy as np
    import s3dlio_amd as S
    from s3dlio_amd import hostbuf
    a = hostbuf.empty(1024)
    a[:] = np.arange(1024) % 251
    bv = hostbuf.readonly(a)
    del a
    gc.collect()
    assert isinstance(bv, S.BytesView)
    assert len(bv) == 1024 and "BytesView" in repr(bv) and "1024" in repr(bv)
    p1 = np.frombuffer(bv.memoryview(), np.uint8).ctypes.data
    p2 = np.frombuffer(bv.memoryview(), np.uint8).ctypes.data
    assert p1 == p2
    tb = bv.to_bytes()
    assert isinstance(tb, bytes) and tb == bytes(bv)
    assert np.frombuffer(tb, np.uint8).ctypes.data != p1
    mv = bv.memoryview()
    del bv
    gc.collect()
    assert bytes(mv[:5]) == bytes([0, 1, 2, 3, 4])


def test_zero_size():
    from s3dlio_amd import hostbuf
    bv = hostbuf.readonly(hostbuf.empty(0))
    assert len(bv) == 0 and bytes(bv) == b"" and memoryview(bv).nbytes == 0
