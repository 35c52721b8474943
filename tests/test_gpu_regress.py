"""GPU regression tests for context-cache lifetime bugs.

A batch whose tile map had to grow used to free the context's cached jump
tables and CRC tables while leaving the pointers cached (use after free): a
later K2 / DG1 / CRC call on the same context then read freed memory.  The
order below (cache -> batch -> reuse) reproduces it on a fresh context.
"""
import zlib

import numpy as np
import pytest


@pytest.mark.gpu
def test_batch_growth_keeps_cached_tables(oracle):
    import torch
    import s3dlio_amd as S
    ctx = S.Context(0, base_seed=S.DEFAULT_BASE_SEED)
    MiB = 1 << 20
    n = 3 * MiB + 5
    buf = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    exp_dg = oracle.dgen_fill(n, 2, 1, 2, 77).tobytes()
    exp_ks = oracle.xoshiro_chunks(n, 2 * MiB, 9).tobytes()

    def check():
        ctx.dgen_fill(buf, n, dedup=2, compress=2, seed=77)
        ctx.sync()
        assert bytes(buf[:n].cpu().numpy()) == exp_dg
        ctx.xoshiro_fill(buf, n, 2 * MiB, seed_base=9)
        ctx.sync()
        host = buf[:n].cpu().numpy().tobytes()
        assert host == exp_ks
        assert S.crc32_device(ctx, buf, n) == zlib.crc32(host)

    check()                                           # caches jump tables + CRC tables
    big = torch.empty(64 * MiB, dtype=torch.uint8, device="cuda")
    for nobj in (4, 300):                             # first batch allocates, second grows the map
        objs = [(k * 4 * 4096, 4 * 4096 - 3, k, 1, 1) for k in range(nobj)]
        ctx.fill_batch(big, objs)
        ctx.sync()
        check()                                       # the cached tables must still be valid
    del ctx


@pytest.mark.gpu
def test_no_device_or_host_leak_across_repeated_calls(tmp_path):
    """Repeated generate_data / generate_npz_bytes / Generator / contexts /
    put_objects / batches must not grow device memory or pinned host memory:
    every cache is bounded and every context frees what it allocated."""
    import gc
    import resource
    import torch
    import s3dlio_amd as S

    def dev_used():
        torch.cuda.synchronize()
        free, total = torch.cuda.mem_get_info()
        return total - free

    def round_():
        for _ in range(20):
            assert len(S.generate_data(3 << 20, 2, 2)) == 3 << 20
        S.generate_npz_bytes([256, 256, 3])
        for _ in range(20):
            g = S.Generator(5 << 20, 1, 3, seed=1)
            b = bytearray(1 << 20)
            while g.fill_chunk(b):
                pass
        for _ in range(5):
            with S.Context(0) as c:
                t = torch.empty(1 << 20, dtype=torch.uint8, device="cuda")
                c.fill_batch(t, [(0, 4096 * 3 + 7, 1, 2, 3), (16384, 100000, 2, 1, 1)])
                c.xoshiro_fill(t, 1 << 20)
                c.sync()
                del t
        S.put_objects([f"file://{tmp_path}/o{j}" for j in range(8)], 70000, seed=3)
        gc.collect()

    round_()                                   # first use creates the bounded caches
    d0 = dev_used()
    r0 = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss
    for _ in range(3):
        round_()
    d1 = dev_used()
    r1 = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss
    assert d1 - d0 < 64 << 20, (d0, d1)        # device memory flat (allocator noise only)
    assert (r1 - r0) * 1024 < 512 << 20, (r0, r1)


@pytest.mark.gpu
def test_stream_release_frees_per_stream_state(oracle):
    """tiled launches on many short-lived streams keep one launch
    state each until s3dg_stream_release; after release the count drops, device
    memory returns, and a reused stream starts fresh with exact bytes."""
    import torch
    import s3dlio_amd as S
    MiB = 1 << 20
    ctx = S.Context(0, base_seed=S.DEFAULT_BASE_SEED)
    buf = torch.empty(80 * MiB, dtype=torch.uint8, device="cuda")
    exp = oracle.fill_controlled(80 * MiB, 1, 0, 1, 5, oracle.base_block(S.DEFAULT_BASE_SEED))

    def dev_used():
        torch.cuda.synchronize()
        free, total = torch.cuda.mem_get_info()
        return total - free

    before = ctx.stream_state_count()
    streams = [torch.cuda.Stream() for _ in range(6)]
    for s in streams:                       # >= 64 MiB: the tiled path, one tile map per stream
        ctx.fill_controlled(buf, 80 * MiB, dedup=1, compress=1, entropy=5, stream=s)
        ctx.fill_batch(buf, [(0, 3 * MiB, 1, 1, 1)], stream=s)
    torch.cuda.synchronize()
    assert ctx.stream_state_count() >= before + 6
    used = dev_used()
    for s in streams:
        ctx.release_stream(s)
    assert ctx.stream_state_count() == before
    assert dev_used() <= used
    ctx.release_stream(streams[0])          # unknown now: no-op
    ctx.fill_controlled(buf, 80 * MiB, dedup=1, compress=1, entropy=5, stream=streams[0])
    torch.cuda.synchronize()
    assert np.array_equal(buf.cpu().numpy(), exp)
    del ctx
