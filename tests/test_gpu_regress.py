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
