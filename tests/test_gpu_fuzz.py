"""GPU: seeded random cases through every generation entry point, each
checked byte for byte against the C oracle (oracle/s3dg_oracle.c), with guard
bytes around every output.  Complements the fixed edge-case fixtures: random
sizes (ragged tails, 1..7-byte tails, block and chunk boundaries), dedup
factors, integer and rational compress ratios, entropies near 2^64, random
base blocks and random launch knobs (waves, occupancy, store floor, store policy,
prefetch, batch tile size, keystream shape).  Reference semantics: src/data_gen.rs:151-224
(fill), :102-132 (random-data layout), src/data_formats/npz.rs:376-383 (K2).
"""
import os
import random

import numpy as np
import pytest

from oracle import oracle_py as P

pytestmark = pytest.mark.gpu
GUARD = 0xA7
SOAK = max(1, int(os.environ.get("S3DG_FUZZ_SOAK", "1")))   # soak runs: seeds x SOAK


@pytest.fixture(scope="module")
def torch():
    import torch as t
    return t


def _size(rnd):
    k = rnd.random()
    if k < 0.3:
        return rnd.randint(1, 5000)
    if k < 0.6:
        return rnd.choice([4096, 8192, 2048, 2049, 2047]) * rnd.randint(1, 40) + rnd.randint(-7, 7)
    return rnd.randint(5000, 6 << 20)


def _compress(rnd):
    return rnd.choice([1, 1, 2, 3, 4, 7, 16, (3, 2), (5, 3), (9, 4)])


def _knobs(ctx, rnd):
    ctx.set_waves_per_block(rnd.choice([0, 1, 2, 4]))
    occ = rnd.choice([-1, 0, 4, 9, 14, 24])
    ctx.set_occupancy(occ, occ)
    sp = rnd.choice([-1, 0, 1, 2, 3])
    ctx.set_store_policy(sp, sp)
    ctx.set_batch_prefetch(rnd.choice([-1, 0, 1, 7, 128, 256, 1 << 20]))
    ctx.set_batch_tile(rnd.choice([0, 0, 1, 2, 4, 8, 16, 32, 64]))
    ctx.set_batch_pace(rnd.choice([-1, -1, 0, 50, 200]))   # wall-clock store floor (per-launch default: -1)
    ctx.set_batch_split(rnd.choice([-1, -1, 0, 8, 64]))    # small objects' own launch


def _reset(ctx):
    ctx.set_waves_per_block(0)
    ctx.set_occupancy(-1, -1)
    ctx.set_store_policy(-1, -1)
    ctx.set_batch_prefetch(-1)
    ctx.set_batch_tile(0)
    ctx.set_batch_pace(-1)
    ctx.set_batch_split(-1)
    ctx.set_stream_tiles(-1)
    ctx.set_keystream_shape(0)
    ctx.set_keystream_shape(1)
    ctx.set_keystream_xcd_group(0, 0)
    ctx.set_keystream_xcd_group(1, 0)


@pytest.mark.parametrize("seed", range(12 * SOAK))
def test_fuzz_controlled_stream_batch(gpu_ctx, torch, oracle, seed):
    rnd = random.Random(1000 + seed)
    orig = gpu_ctx.base_block
    base = np.frombuffer(rnd.randbytes(4096), np.uint8).copy()
    gpu_ctx.set_base_block(base.tobytes())
    try:
        for _ in range(6):
            _knobs(gpu_ctx, rnd)
            L, d, c = _size(rnd), rnd.choice([0, 1, 2, 3, 5, 64, 1 << 20]), _compress(rnd)
            e = rnd.getrandbits(64)
            fn, fd = P.compress_ratio(c)
            t = torch.full((L + 48,), GUARD, dtype=torch.uint8, device="cuda")
            gpu_ctx.fill_controlled(t, L, dedup=d, compress=c, entropy=e)
            h = t.cpu().numpy()
            assert np.array_equal(h[:L], oracle.fill_controlled(L, d, fn, fd, e, base)), (L, d, c, e)
            assert (h[L:] == GUARD).all()
            # a stream of equal objects at a padded stride
            n, sz = rnd.randint(1, 9), _size(rnd) % (1 << 20) + 1
            stride = (sz + 15) // 16 * 16 + 16 * rnd.randint(0, 3)
            sb, first = rnd.getrandbits(64), rnd.randint(0, 1 << 20)
            t = torch.full((n * stride + 32,), GUARD, dtype=torch.uint8, device="cuda")
            gpu_ctx.fill_stream(t, obj_size=sz, n_objs=n, stride=stride, dedup=d, compress=c, seed_base=sb,
                                first_obj=first)
            h = t.cpu().numpy()
            for j in range(n):
                exp = oracle.fill_controlled(sz, d, fn, fd, P.object_entropy(sb, first + j), base)
                assert np.array_equal(h[j * stride:j * stride + sz], exp), (sz, j, d, c)
                assert (h[j * stride + sz:(j + 1) * stride] == GUARD).all()
            # a mixed batch with per-object parameters and guard gaps
            objs, off = [], 0
            for j in range(rnd.randint(1, 12)):
                sz = _size(rnd)
                objs.append((off, sz, rnd.getrandbits(64), rnd.choice([1, 2, 4, 9]), _compress(rnd)))
                off += (sz + 15) // 16 * 16 + 16 * rnd.randint(1, 3)
            t = torch.full((off + 16,), GUARD, dtype=torch.uint8, device="cuda")
            gpu_ctx.fill_batch(t, objs)
            h = t.cpu().numpy()
            ends = [o[0] for o in objs[1:]] + [off + 16]
            for (o, sz, e, d2, c2), end in zip(objs, ends):
                f2n, f2d = P.compress_ratio(c2)
                assert np.array_equal(h[o:o + sz], oracle.fill_controlled(sz, d2, f2n, f2d, e, base)), (sz, d2, c2)
                assert (h[o + sz:end] == GUARD).all()
    finally:
        gpu_ctx.set_base_block(orig)
        _reset(gpu_ctx)


@pytest.mark.parametrize("seed", range(6 * SOAK))
def test_fuzz_tiled_streams(gpu_ctx, torch, oracle, seed):
    """Large uniform streams (>= 16384 blocks) take the tiled batch kernel:
    random ragged sizes, 32 KiB-multiple strides, random destination offsets
    (so every XCD lead 0..7 occurs) and random launch knobs."""
    rnd = random.Random(3000 + seed)
    base = np.frombuffer(gpu_ctx.base_block, np.uint8)
    try:
        for _ in range(3):
            _knobs(gpu_ctx, rnd)
            gpu_ctx.set_stream_tiles(1)
            sz = rnd.randint(4096, 4 << 20) + rnd.choice([0, 0, 1, 7, 15, 4095])
            stride = ((sz + 32767) // 32768 + rnd.randint(0, 2)) * 32768
            blocks = (sz + 4095) // 4096
            n = max(1, (16384 + blocks - 1) // blocks + rnd.randint(0, 8))
            while n > 1 and n * stride > (160 << 20):
                n -= 1
            off = 16 * rnd.randint(0, 4096)
            d, c = rnd.choice([1, 2, 3, 5, 64]), _compress(rnd)
            fn, fd = P.compress_ratio(c)
            sb, first = rnd.getrandbits(64), rnd.randint(0, 1 << 20)
            t = torch.full((off + n * stride + 32,), GUARD, dtype=torch.uint8, device="cuda")
            gpu_ctx.fill_stream(t[off:], obj_size=sz, n_objs=n, stride=stride, dedup=d, compress=c,
                                seed_base=sb, first_obj=first)
            h = t.cpu().numpy()
            assert (h[:off] == GUARD).all()
            g = h[off:]
            exp = oracle.fill_stream(sz, n, d, fn, fd, sb, first, base, stride=stride, threads=8)
            for j in range(n):
                o = j * stride
                assert np.array_equal(g[o:o + sz], exp[o:o + sz]), (sz, stride, n, off, j, d, c)
                assert (g[o + sz:o + stride] == GUARD).all(), (sz, j)
            assert (g[n * stride:] == GUARD).all()
    finally:
        _reset(gpu_ctx)


@pytest.mark.parametrize("seed", range(8 * SOAK))
def test_fuzz_random_layout_keystream_dgen(gpu_ctx, torch, oracle, seed):
    rnd = random.Random(2000 + seed)
    base = np.frombuffer(gpu_ctx.base_block, np.uint8)
    try:
        for _ in range(5):
            L, e = _size(rnd), rnd.getrandbits(64)
            t = torch.full((L + 40,), GUARD, dtype=torch.uint8, device="cuda")
            gpu_ctx.random_data(t, L, entropy=e)
            h = t.cpu().numpy()
            assert np.array_equal(h[:L], oracle.random_data(L, e, base)), (L, e)
            assert (h[L:] == GUARD).all()
            for mode in (0, 1):
                gpu_ctx.set_keystream_shape(mode, rnd.choice([0, 16, 32, 64]), rnd.choice([0, 1, 2, 4]),
                                            rnd.choice([0, 0, 1, 3]), rnd.choice([0, 64, 512, 4096]),
                                            rnd.choice([-1, 0, 1, 2, 3]))
                gpu_ctx.set_keystream_xcd_group(mode, rnd.choice([0, 1, 2, 8, 16, 64, 256]))
            L = _size(rnd)
            chunk = rnd.choice([128, 1152, 65536, 2 << 20, (rnd.randint(1, 4096)) * 128])
            sb = rnd.getrandbits(64)
            t = torch.full((L + 40,), GUARD, dtype=torch.uint8, device="cuda")
            gpu_ctx.xoshiro_fill(t, L, chunk_bytes=chunk, seed_base=sb)
            h = t.cpu().numpy()
            assert np.array_equal(h[:L], oracle.xoshiro_chunks(L, chunk, sb)), (L, chunk, sb)
            assert (h[L:] == GUARD).all()
            L, d, c, sd = _size(rnd) + rnd.randint(0, 3 << 20), rnd.choice([1, 2, 3, 8]), _compress(rnd), rnd.getrandbits(64)
            fn, fd = P.compress_ratio(c)
            t = torch.full((L + 40,), GUARD, dtype=torch.uint8, device="cuda")
            gpu_ctx.dgen_fill(t, L, dedup=d, compress=c, seed=sd)
            h = t.cpu().numpy()
            assert np.array_equal(h[:L], oracle.dgen_fill(L, d, fn, fd, sd)), (L, d, c, sd)
            assert (h[L:] == GUARD).all()
    finally:
        _reset(gpu_ctx)
