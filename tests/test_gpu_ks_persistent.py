"""GPU: persistent keystream launches (k_keystream over per-XCD unit queues,
launches of more than one round of resident waves) write exactly the bytes of
the static grid.  The reference is the same keystream cut into launches of
less than one round (static grid, other lane splits) and the oracle on sample
chunks.  Covers 1-wave (K2, DG1 c1) and 4-wave (DG1 with a zero prefix)
workgroups, ragged object ends, several objects per launch, back-to-back
persistent launches on one stream (the queue counter sets alternate) and on
two streams.  A context with s3dg_set_keystream_persist(1) forces the
persistent grid from one round up (both workgroup shapes); the default rule
(1-wave workgroups from 6 rounds) is covered at 6 GiB."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
MiB, GiB = 1 << 20, 1 << 30


@pytest.fixture(scope="module")
def S():
    import s3dlio_amd
    return s3dlio_amd


@pytest.fixture(scope="module")
def pctx(S, gpu_ctx):
    """Persistent keystream launches from one round of resident waves up."""
    c = S.Context(0, base_seed=S.DEFAULT_BASE_SEED)
    c.set_keystream_persist(1)
    return c


def _pieces_dgen(ctx, dst, size, d, c, seed, per=128):
    nb = (size + MiB - 1) // MiB
    for lo in range(0, nb, per):
        ctx.dgen_fill(dst[lo * MiB:], size, lo, min(lo + per, nb), dedup=d, compress=c, seed=seed)


@pytest.mark.parametrize("size,d,c", [(2 * GiB + 777, 1, 1), (2 * GiB + 4093, 2, 2), (1280 * MiB + 3, 3, 3)])
def test_dgen_persistent_equals_static_pieces(S, oracle, gpu_ctx, pctx, size, d, c):
    import torch
    seed = 0xC0FFEE + d
    a = torch.full((size + 64,), 0xAB, dtype=torch.uint8, device="cuda")
    b = torch.full_like(a, 0xAB)
    for _ in range(3):   # three persistent launches in a row: counter sets 0, 1, 0
        pctx.dgen_fill(a, size, dedup=d, compress=c, seed=seed)
    _pieces_dgen(gpu_ctx, b, size, d, c, seed)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    if d == 1:
        # without dedup a block depends only on (seed, index, length): the first
        # 8 MiB are those of an 8 MiB object
        fn, fd = S.compress_ratio(c)
        exp = np.frombuffer(oracle.dgen_fill(8 * MiB, d, fn, fd, seed), dtype=np.uint8)
        assert np.array_equal(a[:8 * MiB].cpu().numpy(), exp)
    assert (a[size:].cpu().numpy() == 0xAB).all()


def test_dgen_stream_persistent_vs_per_object(S, oracle, gpu_ctx, pctx):
    import torch
    size, stride, n, sb = 300 * MiB + 17, 301 * MiB, 7, 0x5EED000000000001
    a = torch.full((n * stride + 64,), 0xAB, dtype=torch.uint8, device="cuda")
    pctx.dgen_fill_stream(a, size, n, stride=stride, dedup=2, compress=2, seed_base=sb, first_obj=3)
    b = torch.full_like(a, 0xAB)
    for j in range(n):
        _pieces_dgen(gpu_ctx, b[j * stride:], size, 2, 2, S.object_entropy(sb, 3 + j))
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    exp = oracle.dgen_fill(size, 2, 1, 2, S.object_entropy(sb, 3 + n - 1))
    assert bytes(a[(n - 1) * stride:(n - 1) * stride + size].cpu().numpy()) == bytes(exp)


def test_keystream_persistent_equals_static_pieces(S, oracle, gpu_ctx, pctx):
    """K2 (npz.rs:376-383): 3 GiB + 100 B of 2 MiB chunks in one launch against
    launches of 128 chunks (chunk index = seed), twice on one stream."""
    import torch
    n = 3 * GiB + 100
    a = torch.full((n + 64,), 0xAB, dtype=torch.uint8, device="cuda")
    b = torch.full_like(a, 0xAB)
    pctx.xoshiro_fill(a, n)
    pctx.xoshiro_fill(a, n)
    per = 128 * 2 * MiB
    for off in range(0, n, per):
        gpu_ctx.xoshiro_fill(b[off:], min(per, n - off), seed_base=off // (2 * MiB))
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    last = (n - 1) // (2 * MiB)
    exp = oracle.xoshiro_chunks(n - last * 2 * MiB, 2 * MiB, last)
    assert bytes(a[last * 2 * MiB:n].cpu().numpy()) == bytes(exp)
    assert (a[n:].cpu().numpy() == 0xAB).all()


def test_persistent_launches_on_two_streams(S, gpu_ctx, pctx):
    """Each stream has its own counter sets: persistent launches alternating
    between two streams (and overlapping in time) write the static bytes."""
    import torch
    size = 1536 * MiB
    ref = torch.empty(size, dtype=torch.uint8, device="cuda")
    _pieces_dgen(gpu_ctx, ref, size, 1, 1, 77)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outs = [torch.empty(size, dtype=torch.uint8, device="cuda") for _ in range(2)]
    torch.cuda.synchronize()
    for k in range(4):
        st = (s1, s2)[k & 1]
        with torch.cuda.stream(st):
            pctx.dgen_fill(outs[k & 1], size, dedup=1, compress=1, seed=77, stream=st)
    torch.cuda.synchronize()
    for o in outs:
        assert torch.equal(o, ref)


def test_default_rule_six_rounds(S, oracle, gpu_ctx):
    """The default context: a 6 GiB + 5 B DG1 c1 object (6145 one-wave units,
    six rounds) runs persistent; its bytes equal the static pieces and the
    oracle on its first and last blocks."""
    import torch
    size = 6 * GiB + 5
    a = torch.full((size + 64,), 0xAB, dtype=torch.uint8, device="cuda")
    gpu_ctx.dgen_fill(a, size, dedup=1, compress=1, seed=4242)
    b = torch.full_like(a, 0xAB)
    _pieces_dgen(gpu_ctx, b, size, 1, 1, 4242)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    exp = np.frombuffer(oracle.dgen_fill(2 * MiB, 1, 0, 1, 4242), dtype=np.uint8)
    assert np.array_equal(a[:2 * MiB].cpu().numpy(), exp)
    assert (a[size:].cpu().numpy() == 0xAB).all()
    del a, b


def test_persist_knob_off_and_bad_args(S):
    c = S.Context(0, base_seed=S.DEFAULT_BASE_SEED)
    c.set_keystream_persist(0)
    c.set_keystream_persist(-5)      # default rule
    c.set_keystream_persist(3)


@pytest.mark.parametrize("case", range(int(os.environ.get("S3DG_PERSIST_FUZZ", "8"))))
def test_persistent_fuzz_shapes(S, gpu_ctx, case):
    """Seeded draws of object size (1.1-2.3 GiB, ragged), dedup, compress,
    workgroup waves, XCD group and lane length, DG1 or K2, through a context
    that runs every launch of one round or more persistent; bytes equal the
    default context's static pieces of less than one round.  S3DG_PERSIST_FUZZ
    sets the number of draws (default 8)."""
    import random
    import torch
    rng = random.Random(9000 + case)
    c = S.Context(0, base_seed=S.DEFAULT_BASE_SEED)
    c.set_keystream_persist(1)
    mode = rng.choice((0, 1))
    waves = rng.choice((1, 2, 4))
    c.set_keystream_shape(mode, 64, waves, 0, rng.choice((512, 1024, 2048)), -1)
    c.set_keystream_xcd_group(mode, rng.choice((1, 4, 16, 64)))
    size = int(rng.uniform(1.1, 2.3) * GiB) + rng.randrange(1, 4096)
    a = torch.full((size + 64,), 0xAB, dtype=torch.uint8, device="cuda")
    b = torch.full_like(a, 0xAB)
    if mode == 1:
        d, cc, seed = rng.choice((1, 2, 3)), rng.choice((1, 2, 3)), rng.getrandbits(64)
        c.dgen_fill(a, size, dedup=d, compress=cc, seed=seed)
        c.dgen_fill(a, size, dedup=d, compress=cc, seed=seed)
        _pieces_dgen(gpu_ctx, b, size, d, cc, seed)
    else:
        size = size // 16 * 16
        sb = rng.getrandbits(40)
        c.xoshiro_fill(a, size, seed_base=sb)
        per = 128 * 2 * MiB
        for off in range(0, size, per):
            gpu_ctx.xoshiro_fill(b[off:], min(per, size - off), seed_base=sb + off // (2 * MiB))
    torch.cuda.synchronize()
    assert torch.equal(a, b), (mode, waves, size)


@pytest.mark.parametrize("size,d,c", [(6 * GiB, 1, 1), (6 * GiB + 5, 2, 1), (6 * GiB, 2, 2), (5 * GiB, 1, 3)])
def test_tail_half_lanes_equal(S, gpu_ctx, size, d, c):
    """One-object DG1 launches on the persistent grid hand out their last
    blocks as half-length lanes (s3dg_set_keystream_tail): the default, a
    long tail (1000 blocks) and none (0: the round-4 launch, pinned to the
    oracle by the tests above) write the same bytes, and nothing past the
    object."""
    import torch
    outs = []
    for tail in (-1, 1000, 0):
        ctx = S.Context(0, base_seed=S.DEFAULT_BASE_SEED)
        ctx.set_keystream_tail(tail)
        a = torch.full((size + 64,), 0xAB, dtype=torch.uint8, device="cuda")
        ctx.dgen_fill(a, size, dedup=d, compress=c, seed=0xBEEF + c)
        torch.cuda.synchronize()
        outs.append(a)
        ctx.close()
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    assert (outs[0][size:].cpu().numpy() == 0xAB).all()
    del outs
