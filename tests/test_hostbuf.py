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
    assert bytes(mv[:4]) == b"\x07" * 4 and bytes(mv[-4:]) == b"\x07" * 4
    idle0 = hostbuf.pool_stats()["idle_buffers"]
    del mv
    gc.collect()
    assert hostbuf.pool_stats()["idle_buffers"] == idle0 + 1
    c, d = hostbuf.empty(n), hostbuf.empty(n)   # both come back from the pool
    assert {c.ctypes.data, d.ctypes.data} == {addr, addr_b}


def test_readonly_export_semantics():
    from s3dlio_amd import hostbuf
    a = hostbuf.empty(4096)
    mv = hostbuf.readonly(a)
    assert mv.readonly and mv.nbytes == 4096
    with pytest.raises(TypeError):
        mv[0] = 1
    import numpy as np
    assert not np.frombuffer(mv, np.uint8).flags.writeable


def test_zero_size():
    from s3dlio_amd import hostbuf
    assert hostbuf.readonly(hostbuf.empty(0)).nbytes == 0
