"""GPU: DG1 launches with a zero prefix split into a zero-prefix launch in the
fill's store shape (k_zero_prefix) plus a keystream launch over the blocks'
tails (k_keystream with the draw offset z0; s3dg_set_dgen_zero_split) write
exactly the bytes of the single keystream launch, which the oracle pins
(oracle/dgen_oracle: the DG1 contract of src/data_gen_alt.rs:66-80,
src/python_api/python_datagen_api.rs:58-70; parity unpinned by construction,
DESIGN.md §5.3).  Covers compress 2, 3, 4, 8 and ratios whose prefix ends
inside a granule, dedup 1-3, block ranges of ragged objects (the split needs
every block of the launch full length), several objects per launch (the
chunk -> object division), the zero launch's 65 535-chunk grid pieces, its
workgroup shapes, store policies, occupancy caps and side-stream overlap,
and launches below the threshold."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
MiB, GiB = 1 << 20, 1 << 30


@pytest.fixture(scope="module")
def S():
    import s3dlio_amd
    return s3dlio_amd


@pytest.fixture(scope="module")
def one(S):
    """The reference: one keystream launch, never split."""
    c = S.Context(0, base_seed=S.DEFAULT_BASE_SEED)
    c.set_dgen_zero_split(0)
    return c


@pytest.fixture(scope="module")
def split(S):
    """Split from one block up."""
    c = S.Context(0, base_seed=S.DEFAULT_BASE_SEED)
    c.set_dgen_zero_split(1)
    return c


def _pair(torch, n):
    a = torch.full((n + 4096,), 0xAB, dtype=torch.uint8, device="cuda")
    return a, torch.full_like(a, 0xCD)


@pytest.mark.parametrize("size,d,c", [
    (96 * MiB, 1, 2), (96 * MiB, 2, 2), (130 * MiB, 3, 3), (64 * MiB, 1, 4), (80 * MiB, 2, 8),
    (72 * MiB, 1, (3, 2)), (72 * MiB, 2, (5, 4)), (200 * MiB, 1, 7),
])
def test_split_equals_single_launch(S, oracle, one, split, size, d, c):
    import torch
    seed = 0xD6E5 + d
    a, b = _pair(torch, size)
    split.dgen_fill(a, size, dedup=d, compress=c, seed=seed)
    one.dgen_fill(b, size, dedup=d, compress=c, seed=seed)
    torch.cuda.synchronize()
    assert torch.equal(a[:size], b[:size])
    assert (a[size:].cpu().numpy() == 0xAB).all()          # nothing past the object
    fn, fd = S.compress_ratio(c)
    exp = np.frombuffer(oracle.dgen_fill(size, d, fn, fd, seed), dtype=np.uint8)
    got = a[:size].cpu().numpy()
    assert np.array_equal(got[:8 * MiB], exp[:8 * MiB]) and np.array_equal(got[-8 * MiB:], exp[-8 * MiB:])


@pytest.mark.parametrize("size", [100 * MiB + 17, 77 * MiB + 4096 * 3 + 5])
def test_ragged_objects_ranges(S, one, split, size):
    """A ragged object: a whole-object launch keeps one keystream launch (its
    last block is short); block ranges that end before it split."""
    import torch
    nb = (size + MiB - 1) // MiB
    a, b = _pair(torch, size)
    for lo, hi in ((0, nb - 1), (nb - 1, nb), (0, nb)):
        split.dgen_fill(a[lo * MiB:], size, lo, hi, dedup=2, compress=2, seed=99)
        one.dgen_fill(b[lo * MiB:], size, lo, hi, dedup=2, compress=2, seed=99)
    torch.cuda.synchronize()
    assert torch.equal(a[:size], b[:size])
    lo = 5
    split.dgen_fill(a[lo * MiB:], size, lo, lo + 40, dedup=1, compress=3, seed=7)
    one.dgen_fill(b[lo * MiB:], size, lo, lo + 40, dedup=1, compress=3, seed=7)
    torch.cuda.synchronize()
    assert torch.equal(a[:size], b[:size])


def test_stream_of_objects(S, oracle, one, split):
    """Several objects per launch at a stride: chunk -> object by fastdiv."""
    import torch
    size, stride, n, sb = 37 * MiB, 39 * MiB + 4096, 9, 0x5EED000000000001
    a, b = _pair(torch, n * stride)
    split.dgen_fill_stream(a, size, n, stride=stride, dedup=2, compress=2, seed_base=sb, first_obj=4)
    one.dgen_fill_stream(b, size, n, stride=stride, dedup=2, compress=2, seed_base=sb, first_obj=4)
    torch.cuda.synchronize()
    for j in range(n):
        assert torch.equal(a[j * stride:j * stride + size], b[j * stride:j * stride + size]), j
        assert (a[j * stride + size:(j + 1) * stride].cpu().numpy() == 0xAB).all(), j   # gaps untouched
    exp = oracle.dgen_fill(size, 2, 1, 2, S.object_entropy(sb, 4 + n - 1))
    assert bytes(a[(n - 1) * stride:(n - 1) * stride + size].cpu().numpy()) == bytes(exp)


@pytest.mark.parametrize("waves,store,occ,overlap", [
    (1, 0, 0, 0), (1, 1, 0, 1), (2, 2, 29, 0), (4, 3, 14, 1), (4, 2, 4, 0), (4, 2, 8, 1)])
def test_zero_launch_knobs(S, one, waves, store, occ, overlap):
    import torch
    c = S.Context(0, base_seed=S.DEFAULT_BASE_SEED)
    c.set_dgen_zero_split(1, waves, occ, store, overlap)
    size = 48 * MiB
    a, b = _pair(torch, size)
    c.dgen_fill(a, size, dedup=1, compress=2, seed=5)
    one.dgen_fill(b, size, dedup=1, compress=2, seed=5)
    torch.cuda.synchronize()
    assert torch.equal(a[:size], b[:size])


def test_default_threshold(S, gpu_ctx, one):
    """The default context splits from 64 blocks: 63 and 64 blocks both equal
    the single launch."""
    import torch
    for nb in (63, 64, 640):
        size = nb * MiB
        a, b = _pair(torch, size)
        gpu_ctx.dgen_fill(a, size, dedup=3, compress=4, seed=nb)
        one.dgen_fill(b, size, dedup=3, compress=4, seed=nb)
        torch.cuda.synchronize()
        assert torch.equal(a[:size], b[:size]), nb


def test_zero_grid_pieces(S, one, split):
    """70 000 blocks in one launch: the zero launch's grid in 65 535-chunk pieces."""
    import torch
    n, size = 7, 10000 * MiB
    a = torch.full((n * size,), 0xAB, dtype=torch.uint8, device="cuda")
    b = torch.full_like(a, 0xCD)
    split.dgen_fill_stream(a, size, n, dedup=1, compress=2, seed_base=11)
    one.dgen_fill_stream(b, size, n, dedup=1, compress=2, seed_base=11)
    torch.cuda.synchronize()
    piece = 2 * GiB
    for off in range(0, n * size, piece):
        assert torch.equal(a[off:off + piece], b[off:off + piece]), off
    del a, b


@pytest.mark.parametrize("size,c", [(70 * MiB + 3, 2), (65 * MiB + 4095, 3)])
def test_ragged_stream_splits_full_blocks(S, oracle, one, gpu_ctx, size, c):
    """Objects with a short last block (the default context, >= 64 full
    blocks per object): the full blocks split, the short last blocks in a
    launch of their own; equal to the single launch, gaps untouched."""
    import torch
    stride, n, sb = 72 * MiB, 3, 0x5EED000000000001
    a, b = _pair(torch, n * stride)
    gpu_ctx.dgen_fill_stream(a, size, n, stride=stride, dedup=2, compress=c, seed_base=sb, first_obj=1)
    one.dgen_fill_stream(b, size, n, stride=stride, dedup=2, compress=c, seed_base=sb, first_obj=1)
    torch.cuda.synchronize()
    for j in range(n):
        assert torch.equal(a[j * stride:j * stride + size], b[j * stride:j * stride + size]), j
        assert (a[j * stride + size:(j + 1) * stride].cpu().numpy() == 0xAB).all(), j
    fn, fd = S.compress_ratio(c)
    exp = oracle.dgen_fill(size, 2, fn, fd, S.object_entropy(sb, 1 + n - 1))
    assert bytes(a[(n - 1) * stride:(n - 1) * stride + size].cpu().numpy()) == bytes(exp)


@pytest.mark.parametrize("ctxname", ["gpu_ctx", "split"])
@pytest.mark.parametrize("c", [2, 3])
def test_one_full_block_per_object(S, oracle, one, request, ctxname, c):
    """Objects of 1 MiB + 100 B at a 4 KiB-rounded stride: the full blocks
    split as one chunk per object (cpo = 1, the zero launch's fastdiv
    special case), the 100-B tails in a launch of their own.  Equal to the
    single launch and the oracle, the gaps between objects untouched."""
    import torch
    ctx = request.getfixturevalue(ctxname)
    size, n, sb = MiB + 100, 80, 0x5EED000000000003
    stride = (size + 4095) // 4096 * 4096
    a, b = _pair(torch, n * stride)
    ctx.dgen_fill_stream(a, size, n, stride=stride, dedup=1, compress=c, seed_base=sb, first_obj=2)
    one.dgen_fill_stream(b, size, n, stride=stride, dedup=1, compress=c, seed_base=sb, first_obj=2)
    torch.cuda.synchronize()
    ha = a.cpu().numpy()
    hb = b.cpu().numpy()
    fn, fd = S.compress_ratio(c)
    for j in range(n):
        o = j * stride
        assert np.array_equal(ha[o:o + size], hb[o:o + size]), j
        assert (ha[o + size:o + stride] == 0xAB).all(), j
    for j in (0, n // 2, n - 1):
        exp = oracle.dgen_fill(size, 1, fn, fd, S.object_entropy(sb, 2 + j))
        assert bytes(ha[j * stride:j * stride + size]) == bytes(exp), j
