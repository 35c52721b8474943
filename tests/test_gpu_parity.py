"""GPU parity: the gfx950 kernels through the C ABI vs the golden fixtures and
the C oracle (bit-exact; integer/byte work, no tolerance)."""
import hashlib
import json
import os
import random

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import oracle_py as P

pytestmark = pytest.mark.gpu

SEED_BASE = 0x5EED000000000001
GUARD = 0xAB


def sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def torch():
    import torch
    return torch


@pytest.fixture(scope="module")
def base(golden_base):
    return np.frombuffer(golden_base, np.uint8)


def test_base_block_matches_fixture(gpu_ctx, golden_base):
    assert gpu_ctx.base_block == golden_base


def test_cfg1_golden_digests(gpu_ctx, torch):
    g = load("cfg1_1000x64KiB.json")
    n, size = g["objects"], g["size"]
    out = torch.empty(n * size, dtype=torch.uint8, device="cuda")
    gpu_ctx.fill_stream(out, obj_size=size, n_objs=n, seed_base=int(g["seed_base"], 16))
    torch.cuda.synchronize()
    host = out.cpu().numpy()
    digests = [sha(host[j * size:(j + 1) * size]) for j in range(n)]
    assert digests == g["sha256"]


def test_edge_case_fixtures_with_guards(gpu_ctx, torch):
    cases = load("edge_cases.json")["cases"]
    maxlen = max(c["len"] for c in cases)
    buf = torch.empty(maxlen + 256, dtype=torch.uint8, device="cuda")
    bad = []
    for c in cases:
        buf.fill_(GUARD)
        gpu_ctx.fill_controlled(buf, c["len"], dedup=c["dedup"],
                                compress=(c["f_den"], c["f_den"] - c["f_num"]) if c["f_num"] else 1,
                                entropy=int(c["entropy"]))
        h = buf[:c["len"] + 256].cpu().numpy()
        if sha(h[:c["len"]]) != c["sha256"] or not (h[c["len"]:] == GUARD).all():
            bad.append(c)
    assert not bad, bad[:3]


def test_blob_fixtures(gpu_ctx, torch):
    for name, (L, d, comp, e) in {"blob_4097_d1_c3": (4097, 1, 3, 11),
                                  "blob_12288_d2_c2": (12288, 2, 2, 12),
                                  "blob_8192_d1_c1": (8192, 1, 1, 13)}.items():
        with open(os.path.join(GOLDEN, name + ".bin"), "rb") as f:
            exp = f.read()
        t = torch.empty(L, dtype=torch.uint8, device="cuda")
        gpu_ctx.fill_controlled(t, L, dedup=d, compress=comp, entropy=e)
        assert bytes(t.cpu().numpy()) == exp, name


@pytest.mark.parametrize("size,stride,n,d,c,first", [
    (8 * 2**20, 8 * 2**20, 24, 1, 1, 0),
    (8 * 2**20, 8 * 2**20, 24, 4, 2, 7),
    (8 * 2**20, 8 * 2**20, 24, 2, 3, 123456),
    (4096 * 70 + 1000, 4096 * 72, 9, 3, 5, 3),
    (4096 * 64, 4096 * 64, 5, 1, 2, 0),
    (1, 16, 33, 1, 1, 0),
    (4095, 4096, 17, 2, 129, 2**20),
])
def test_stream_vs_oracle(gpu_ctx, torch, oracle, base, size, stride, n, d, c, first):
    fn, fd = P.compress_ratio(c)
    out = torch.full((stride * n + 64,), GUARD, dtype=torch.uint8, device="cuda")
    gpu_ctx.fill_stream(out, obj_size=size, n_objs=n, stride=stride, dedup=d, compress=c,
                        seed_base=SEED_BASE, first_obj=first)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    exp = oracle.fill_stream(size, n, d, fn, fd, SEED_BASE, first, base, stride=stride, threads=8)
    for j in range(n):
        o = j * stride
        assert np.array_equal(got[o:o + size], exp[o:o + size]), j
        assert (got[o + size:o + stride] == GUARD).all(), f"gap overwritten after object {j}"
    assert (got[stride * n:] == GUARD).all()


@pytest.mark.parametrize("size,stride,n,d,c,off,tile", [
    (8 * 2**20, 8 * 2**20, 9, 1, 1, 4096 * 3, 0),            # lead 3
    (2**20 + 123, 2**20 + 32768, 70, 3, (3, 2), 4096 * 7, 0), # ragged tail, lead 7
    (2**20 + 123, 2**20 + 32768, 70, 3, (3, 2), 4096 * 5, 8),
    (3 * 2**20 + 4096 * 5, 4 * 2**20, 20, 2, 3, 16, 16),     # dst 16 B past a granule
    (80 * 2**20 + 9, 80 * 2**20 + 16, 1, 5, 7, 4096, 32),    # one large object
    (2**16, 2**16, 1100, 1, 2, 0, 0),                       # 16-block objects: small tiles
])
def test_stream_tiled_vs_oracle_and_2d(gpu_ctx, torch, oracle, base, size, stride, n, d, c, off, tile):
    """Large uniform streams run through the tiled batch kernel (device-built
    records, XCD lead from the destination address); every byte against the
    oracle and against the 2D stream kernel, guard bytes around every object."""
    fn, fd = P.compress_ratio(c)
    out = torch.full((off + stride * n + 64,), GUARD, dtype=torch.uint8, device="cuda")
    gpu_ctx.set_batch_tile(tile)
    try:
        gpu_ctx.fill_stream(out[off:], obj_size=size, n_objs=n, stride=stride, dedup=d, compress=c,
                            seed_base=SEED_BASE, first_obj=11)
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        gpu_ctx.set_stream_tiles(0)
        out2 = torch.full_like(out, GUARD)
        gpu_ctx.fill_stream(out2[off:], obj_size=size, n_objs=n, stride=stride, dedup=d, compress=c,
                            seed_base=SEED_BASE, first_obj=11)
        torch.cuda.synchronize()
        assert bool(torch.equal(out, out2)), "tiled and 2D stream kernels differ"
    finally:
        gpu_ctx.set_stream_tiles(-1)
        gpu_ctx.set_batch_tile(0)
    exp = oracle.fill_stream(size, n, d, fn, fd, SEED_BASE, 11, base, stride=stride, threads=8)
    assert (got[:off] == GUARD).all()
    g = got[off:]
    for j in range(n):
        o = j * stride
        assert np.array_equal(g[o:o + size], exp[o:o + size]), j
        assert (g[o + size:o + stride] == GUARD).all(), f"gap overwritten after object {j}"
    assert (g[stride * n:] == GUARD).all()


@pytest.mark.parametrize("L,d,c,off", [(70 * 2**20 + 13, 3, (5, 3), 4096 * 5), (64 * 2**20, 1, 1, 0),
                                       (96 * 2**20 + 4095, 2, 4, 48)])
def test_large_fill_controlled_tiled(gpu_ctx, torch, oracle, base, L, d, c, off):
    """A whole buffer >= 64 MiB runs as a one-object tiled stream; against the
    oracle and the 2D kernel, with guard bytes."""
    fn, fd = P.compress_ratio(c)
    e = P.object_entropy(SEED_BASE, 77)
    t = torch.full((off + L + 32,), GUARD, dtype=torch.uint8, device="cuda")
    gpu_ctx.fill_controlled(t[off:], L, dedup=d, compress=c, entropy=e)
    torch.cuda.synchronize()
    h = t.cpu().numpy()
    try:
        gpu_ctx.set_stream_tiles(0)
        t2 = torch.full_like(t, GUARD)
        gpu_ctx.fill_controlled(t2[off:], L, dedup=d, compress=c, entropy=e)
        torch.cuda.synchronize()
        assert bool(torch.equal(t, t2)), "tiled and 2D kernels differ"
    finally:
        gpu_ctx.set_stream_tiles(-1)
    assert (h[:off] == GUARD).all() and (h[off + L:] == GUARD).all()
    assert np.array_equal(h[off:off + L], oracle.fill_controlled(L, d, fn, fd, e, base))


@pytest.mark.parametrize("L,off", [(80 * 2**20 + 5, 4096 * 3), (64 * 2**20, 0)])
def test_large_random_data_tiled(gpu_ctx, torch, oracle, base, L, off):
    """Random-data layout (A6 analogue) at >= 64 MiB: tiled kernel vs oracle and 2D kernel."""
    e = 0x1234567890ABCDEF
    t = torch.full((off + L + 32,), GUARD, dtype=torch.uint8, device="cuda")
    gpu_ctx.random_data(t[off:], L, entropy=e)
    torch.cuda.synchronize()
    h = t.cpu().numpy()
    try:
        gpu_ctx.set_stream_tiles(0)
        t2 = torch.full_like(t, GUARD)
        gpu_ctx.random_data(t2[off:], L, entropy=e)
        torch.cuda.synchronize()
        assert bool(torch.equal(t, t2)), "tiled and 2D kernels differ"
    finally:
        gpu_ctx.set_stream_tiles(-1)
    assert (h[:off] == GUARD).all() and (h[off + L:] == GUARD).all()
    assert np.array_equal(h[off:off + L], oracle.random_data(L, e, base))


def test_tile_map_shared_across_streams(gpu_ctx, torch, oracle, base):
    """A batch on one stream and a tiled stream on another, back to back with
    no host sync: each stream has its own tile map and batch staging, so the
    two launches share nothing.  Repeated with growth."""
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    rnd = random.Random(99)
    for rep in range(3):
        sizes = [rnd.randint(1, 3 << 20) for _ in range(40 + 40 * rep)]
        objs, off = [], 0
        for j, sz in enumerate(sizes):
            objs.append((off, sz, P.object_entropy(SEED_BASE, j), 2, 3))
            off += (sz + 4095) // 4096 * 4096
        a = torch.full((off,), GUARD, dtype=torch.uint8, device="cuda")
        n, size = 12 + 4 * rep, 8 << 20
        b = torch.full((n * size,), GUARD, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        gpu_ctx.fill_batch(a, objs, stream=s1)
        gpu_ctx.fill_stream(b, obj_size=size, n_objs=n, dedup=1, compress=1, seed_base=SEED_BASE + rep,
                            stream=s2)
        torch.cuda.synchronize()
        ha, hb = a.cpu().numpy(), b.cpu().numpy()
        fn, fd = P.compress_ratio(3)
        for (o, sz, e, d, c) in objs:
            assert np.array_equal(ha[o:o + sz], oracle.fill_controlled(sz, d, fn, fd, e, base)), (rep, o)
        exp = oracle.fill_stream(size, n, 1, 0, 1, SEED_BASE + rep, 0, base, threads=8)
        assert np.array_equal(hb, exp), rep


@pytest.mark.parametrize("waves,occ,pf,sp,tile", [
    (1, -1, 128, -1, 0), (2, -1, 128, 0, 64), (4, -1, 128, 1, 8), (1, 0, 0, 0, 16), (1, 20, 1, 1, 32),
    (2, 12, 3, 2, 8), (1, -1, 100000, -1, 64), (2, 14, 64, 3, 0), (1, -1, 128, -1, 8), (1, 26, 0, -1, 16),
    (1, -1, 256, -1, 2), (2, -1, 256, 3, 4)])
def test_batch_mixed_sizes_vs_oracle(gpu_ctx, torch, oracle, base, waves, occ, pf, sp, tile):
    gpu_ctx.set_waves_per_block(waves)
    gpu_ctx.set_occupancy(occ, occ)
    gpu_ctx.set_batch_prefetch(pf)
    gpu_ctx.set_store_policy(sp, sp)
    gpu_ctx.set_batch_tile(tile)
    rnd = random.Random(7)
    sizes = [0, 1, 5, 31, 32, 33, 4095, 4096, 4097, 2**20 + 3, 3 * 2**20, 65536 * 64 + 11]
    sizes += [int(np.exp(rnd.uniform(np.log(4096), np.log(4 * 2**20)))) for _ in range(40)]
    objs, off = [], 0
    for j, sz in enumerate(sizes):
        d = rnd.choice([0, 1, 2, 3, 4, 100])
        c = rnd.choice([1, 2, 3, 7, (3, 2), (5, 3)])
        objs.append((off, sz, P.object_entropy(SEED_BASE, j), d, c))
        off += (sz + 16 + 4095) // 4096 * 4096          # a guard gap after each object
    out = torch.full((off,), GUARD, dtype=torch.uint8, device="cuda")
    gpu_ctx.fill_batch(out, objs)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    nxt = [o[0] for o in objs[1:]] + [off]
    for (o, sz, e, d, c), end in zip(objs, nxt):
        fn, fd = P.compress_ratio(c)
        exp = oracle.fill_controlled(sz, d, fn, fd, e, base)
        assert np.array_equal(got[o:o + sz], exp), (waves, o, sz, d, c)
        assert (got[o + sz:end] == GUARD).all()
    gpu_ctx.set_waves_per_block(0)
    gpu_ctx.set_occupancy(-1, -1)
    gpu_ctx.set_batch_prefetch(-1)
    gpu_ctx.set_store_policy(-1, -1)
    gpu_ctx.set_batch_tile(0)


def test_range_pieces_compose(gpu_ctx, torch, oracle, base):
    L = 4096 * 300 + 77
    full = torch.empty(L, dtype=torch.uint8, device="cuda")
    gpu_ctx.fill_controlled(full, L, dedup=3, compress=3, entropy=31337)
    pieces = torch.empty(L, dtype=torch.uint8, device="cuda")
    for lo, hi in [(0, 1), (1, 65), (65, 130), (130, 301)]:
        view = pieces[lo * 4096:]
        gpu_ctx.fill_range(view, L, lo, hi, dedup=3, compress=3, entropy=31337)
    torch.cuda.synchronize()
    assert torch.equal(full, pieces)
    assert bytes(full.cpu().numpy()) == bytes(oracle.fill_controlled(L, 3, 2, 3, 31337, base))


def test_store_modes_and_occupancy_agree(gpu_ctx, torch):
    n, size = 40, 2**20 + 4096 * 3
    ref = torch.empty(n * size, dtype=torch.uint8, device="cuda")
    gpu_ctx.fill_stream(ref, obj_size=size, n_objs=n, dedup=2, compress=3, seed_base=5)
    for sp in (-1, 0, 1, 2, 3):
        for waves in (1, 2, 4):
            for cap in (-1, 0, 3, 12, 40):
                gpu_ctx.set_store_policy(sp, sp)
                gpu_ctx.set_waves_per_block(waves)
                gpu_ctx.set_occupancy(cap, cap)
                t = torch.zeros_like(ref)
                gpu_ctx.fill_stream(t, obj_size=size, n_objs=n, dedup=2, compress=3, seed_base=5)
                assert torch.equal(t, ref), (sp, waves, cap)
    gpu_ctx.set_nontemporal(True)
    t = torch.zeros_like(ref)
    gpu_ctx.fill_stream(t, obj_size=size, n_objs=n, dedup=2, compress=3, seed_base=5)
    assert torch.equal(t, ref)
    gpu_ctx.set_nontemporal(False)
    gpu_ctx.set_waves_per_block(0)
    gpu_ctx.set_occupancy(-1, -1)


def test_batch_store_floor_identical(gpu_ctx, torch, oracle, base):
    """The batch kernel's wall-clock store floor (s3dg_set_batch_pace; default
    100 ticks for mid-line zero prefixes of >= half a block, e.g. compress 3)
    never changes bytes: a tiled uniform stream and a batch, floors 0..1000."""
    n, size = 20, 8 * 2**20 + 4096 * 5 + 123          # 20 x 2054 blocks: the tiled batch kernel
    stride = 8 * 2**20 + 32 * 1024                     # a multiple of 32 KiB: one granule lead
    ref = torch.empty(n * stride, dtype=torch.uint8, device="cuda")
    gpu_ctx.set_batch_pace(0)
    gpu_ctx.fill_stream(ref, obj_size=size, n_objs=n, dedup=2, compress=3, seed_base=11, stride=stride)
    torch.cuda.synchronize()
    h = ref.cpu().numpy()
    for j in (0, n - 1):
        exp = oracle.fill_controlled(size, 2, 2, 3, P.object_entropy(11, j), base)
        assert np.array_equal(h[j * stride:j * stride + size], exp), j
    for ticks in (-1, 1, 100, 1000):
        gpu_ctx.set_batch_pace(ticks)
        t = torch.zeros_like(ref)
        gpu_ctx.fill_stream(t, obj_size=size, n_objs=n, dedup=2, compress=3, seed_base=11, stride=stride)
        torch.cuda.synchronize()
        for j in range(n):
            assert torch.equal(t[j * stride:j * stride + size], ref[j * stride:j * stride + size]), (ticks, j)
    rnd = random.Random(3)
    objs, off = [], 0
    for j in range(60):
        sz = int(np.exp(rnd.uniform(np.log(4096), np.log(2 * 2**20))))
        objs.append((off, sz, P.object_entropy(SEED_BASE, j), rnd.choice([1, 2, 4]), rnd.choice([3, 3, 5, 2, 1])))
        off += (sz + 16 + 4095) // 4096 * 4096
    for ticks in (-1, 0, 300):
        gpu_ctx.set_batch_pace(ticks)
        out = torch.full((off,), GUARD, dtype=torch.uint8, device="cuda")
        gpu_ctx.fill_batch(out, objs)
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        for (o, sz, e, d, c) in objs:
            fn, fd = P.compress_ratio(c)
            assert np.array_equal(got[o:o + sz], oracle.fill_controlled(sz, d, fn, fd, e, base)), (ticks, o)
    gpu_ctx.set_batch_pace(-1)
    with pytest.raises(Exception):
        gpu_ctx.set_batch_pace(100001)          # more than 1 ms per block is refused
    gpu_ctx.set_batch_pace(-1)


def test_occupancy_cap_is_applied(gpu_ctx):
    # stream default 14 resident 2-wave workgroups per CU, uncapped batch (1 wave),
    # 29 for batch launches with line-aligned zero prefixes (cap 30)
    assert gpu_ctx.query_occupancy(batch=False) == 14
    assert gpu_ctx.query_occupancy(batch=True) >= 30
    assert gpu_ctx.query_occupancy(batch=True, zero_lines=True) == 29
    for cap in (8, 10, 16):
        gpu_ctx.set_occupancy(cap, cap)
        assert gpu_ctx.query_occupancy(batch=False) == cap
        assert gpu_ctx.query_occupancy(batch=True) == cap
        assert gpu_ctx.query_occupancy(batch=True, zero_lines=True) == cap
    gpu_ctx.set_occupancy(-1, -1)
    assert gpu_ctx.query_occupancy(batch=False) == 14


def test_host_dropin_seeded_multi_chunk(oracle, base):
    import s3dlio_amd as S
    L = 150 * 2**20 + 5                      # > two 64 MiB device chunks, ragged tail
    buf = bytearray(L)
    S.fill_controlled_data_seeded(buf, 2, 3, entropy=77, base_block=bytes(base))
    exp = oracle.fill_controlled(L, 2, 2, 3, 77, base)
    assert sha(buf) == sha(exp)
    arr = np.zeros(12345, np.uint8)
    S.fill_controlled_data_seeded(arr, 1, 1, entropy=9)          # default base block
    assert np.array_equal(arr, oracle.fill_controlled(12345, 1, 0, 1, 9, base))


def test_host_dropin_unseeded_contract():
    """Reference unit tests (src/data_gen.rs:405-458): size preserved, not all
    zero, two calls differ, empty buffer ok, dedup/compress accepted."""
    import s3dlio_amd as S
    a, b = bytearray(2**20), bytearray(2**20)
    S.fill_controlled_data(a, 1, 1)
    S.fill_controlled_data(b, 1, 1)
    assert len(a) == 2**20 and any(a) and a != b
    S.fill_controlled_data(bytearray(), 1, 1)
    c = bytearray(4 * 2**20)
    S.fill_controlled_data(c, 4, 1)
    blocks = {bytes(c[i:i + 4096]) for i in range(0, len(c), 4096)}
    assert len(blocks) == 256
    z = bytearray(2 * 2**20)
    S.fill_controlled_data(z, 1, 4)
    assert abs(z.count(0) / len(z) - 0.75) < 0.01


def test_full_size_structure_cfg2(gpu_ctx, torch, base):
    """Size-independent properties at BASELINE cfg2 object size on 1000 x 8 MiB
    (7.8 GiB): every block equals the base block outside the two 32-byte
    windows [0,32) and [2048,2080); windows differ between blocks."""
    n, size = 1000, 8 * 2**20
    out = torch.empty(n * size, dtype=torch.uint8, device="cuda")
    gpu_ctx.fill_stream(out, obj_size=size, n_objs=n, seed_base=SEED_BASE)
    blocks = out.view(-1, 4096)
    bt = torch.from_numpy(base.copy()).cuda()
    mask = torch.ones(4096, dtype=torch.bool, device="cuda")
    mask[0:32] = False
    mask[2048:2080] = False
    assert torch.equal(blocks[:, mask], bt[mask].expand(blocks.shape[0], -1))
    w = blocks[:, 0:8].contiguous().view(torch.int64).flatten()
    assert torch.unique(w).numel() == w.numel()          # 2,048,000 distinct first words
    del out, blocks


def test_full_size_structure_cfg3(gpu_ctx, torch, oracle, base):
    """cfg3 (dedup=4, compress=2) at 8 MiB: U=512 unique blocks repeating with
    period 512, zero prefix exactly 2048 B, sampled objects bit-exact."""
    n, size = 200, 8 * 2**20
    out = torch.empty(n * size, dtype=torch.uint8, device="cuda")
    gpu_ctx.fill_stream(out, obj_size=size, n_objs=n, dedup=4, compress=2, seed_base=SEED_BASE)
    v = out.view(n, 4, 512, 4096)
    for r in range(1, 4):
        assert torch.equal(v[:, 0], v[:, r])
    assert int(v[..., :2048].count_nonzero()) == 0
    for j in (0, 57, n - 1):
        exp = oracle.fill_controlled(size, 4, 1, 2, P.object_entropy(SEED_BASE, j), base)
        assert bytes(out[j * size:(j + 1) * size].cpu().numpy()) == bytes(exp)


def test_write_ceiling_kernel(gpu_ctx, torch):
    t = torch.zeros(2**24, dtype=torch.uint8, device="cuda")
    gpu_ctx.write_ceiling(t, pattern=0x01020304)
    torch.cuda.synchronize()
    w = t.view(torch.int32).view(-1, 4)
    assert int(w[:, 0].eq(0x01020304).all()) == 1


def test_write_ceiling_tiled_kernel(gpu_ctx, torch):
    t = torch.zeros(2**26, dtype=torch.uint8, device="cuda")
    gpu_ctx.write_ceiling_tiled(t, pattern=0x0A0B0C0D)
    torch.cuda.synchronize()
    w = t.view(torch.int32).view(-1, 4)
    assert int(w[:, 0].eq(0x0A0B0C0D).all()) == 1 and int(w[:, 3].eq(~0x0A0B0C0D).all()) == 1


def test_invalid_arguments_raise(gpu_ctx, torch):
    t = torch.empty(4096 + 16, dtype=torch.uint8, device="cuda")
    with pytest.raises(ValueError, match="aligned"):
        gpu_ctx.fill_controlled(int(t.data_ptr()) + 1, 100)
    with pytest.raises(ValueError):
        gpu_ctx.fill_stream(t, obj_size=4096, n_objs=2, stride=100)
    for bad in (3, 9, 128):
        with pytest.raises(ValueError, match="tile"):
            gpu_ctx.set_batch_tile(bad)


def test_keystream_golden_fixtures(gpu_ctx, torch):
    for c in load("xoshiro_chunks.json"):
        t = torch.full((c["len"] + 64,), GUARD, dtype=torch.uint8, device="cuda")
        gpu_ctx.xoshiro_fill(t, c["len"], chunk_bytes=c["chunk"], seed_base=c["seed_base"])
        h = t.cpu().numpy()
        assert sha(h[:c["len"]]) == c["sha256"], c
        assert (h[c["len"]:] == GUARD).all()


@pytest.mark.parametrize("length,chunk,sb", [
    (64 * 2**20 + 5, 2 * 2**20, 0),        # npz.rs chunking, ragged 1..4-byte tail
    (3 * 2**20 + 6, 2 * 2**20, 9),         # 5..7-byte tail
    (2**20 + 4, 256 * 1024, 3),
    (10 * 1152 + 7, 1152, 77),             # one lane per chunk
    (2 * 2**20 + 128, 2 * 2**20 + 128, 1),
    (1, 128, 0),
])
def test_keystream_vs_oracle(gpu_ctx, torch, oracle, length, chunk, sb):
    t = torch.full((length + 64,), GUARD, dtype=torch.uint8, device="cuda")
    gpu_ctx.xoshiro_fill(t, length, chunk_bytes=chunk, seed_base=sb)
    h = t.cpu().numpy()
    exp = oracle.xoshiro_chunks(length, chunk, sb)
    assert np.array_equal(h[:length], exp)
    assert (h[length:] == GUARD).all()


KS_SHAPES = [(16, 4, 0, 0, -1), (16, 1, 0, 0, 2), (32, 2, 0, 0, 1), (64, 4, 0, 0, 2), (64, 1, 3, 0, 0),
             (64, 2, 0, 4096, -1), (32, 4, 1, 64, 2), (16, 2, 0, 128, 1)]


@pytest.mark.parametrize("shape", KS_SHAPES)
def test_keystream_shapes_vs_oracle(gpu_ctx, torch, oracle, shape):
    """Every k_keystream launch shape (stage depth, waves per workgroup,
    occupancy cap, lanes per chunk) writes the same bytes, in both modes."""
    gpu_ctx.set_keystream_shape(0, *shape)
    gpu_ctx.set_keystream_shape(1, *shape)
    try:
        for length, chunk, sb in [(8 * 2**20 + 5, 2 * 2**20, 4), (2**20 + 6, 256 * 1024, 9),
                                  (10 * 1152 + 3, 1152, 77)]:
            t = torch.full((length + 64,), GUARD, dtype=torch.uint8, device="cuda")
            gpu_ctx.xoshiro_fill(t, length, chunk_bytes=chunk, seed_base=sb)
            h = t.cpu().numpy()
            assert np.array_equal(h[:length], oracle.xoshiro_chunks(length, chunk, sb)), (shape, length)
            assert (h[length:] == GUARD).all()
        for size, d, c, seed in [(5 * 2**20 + 7, 2, 3, 5), (3 * 2**20, 1, 1, 11), (2**20 + 3, 1, 2, 2**64 - 1)]:
            t = torch.full((size + 64,), GUARD, dtype=torch.uint8, device="cuda")
            gpu_ctx.dgen_fill(t, size, dedup=d, compress=c, seed=seed)
            h = t.cpu().numpy()
            fn, fd = P.compress_ratio(c)
            assert np.array_equal(h[:size], oracle.dgen_fill(size, d, fn, fd, seed)), (shape, size)
            assert (h[size:] == GUARD).all()
    finally:
        gpu_ctx.set_keystream_shape(0)
        gpu_ctx.set_keystream_shape(1)


@pytest.mark.parametrize("waves,xcd", [(4, 1), (4, 16), (4, 64), (1, 16), (1, 256), (2, 8)])
def test_keystream_xcd_groups_vs_oracle(gpu_ctx, torch, oracle, waves, xcd):
    """XCD-grouped workgroup remap (s3dg_set_keystream_xcd_group): full groups
    plus a ragged last group write the same bytes as the dealing order, K2 and
    DG1, every byte against the oracle."""
    try:
        for mode in (0, 1):
            gpu_ctx.set_keystream_shape(mode, 64, waves)
            gpu_ctx.set_keystream_xcd_group(mode, xcd)
        length, chunk, sb = 300 * 2**20 + 5, 2 * 2**20, 31
        t = torch.full((length + 64,), GUARD, dtype=torch.uint8, device="cuda")
        gpu_ctx.xoshiro_fill(t, length, chunk_bytes=chunk, seed_base=sb)
        h = t.cpu().numpy()
        assert np.array_equal(h[:length], oracle.xoshiro_chunks(length, chunk, sb))
        assert (h[length:] == GUARD).all()
        size, d, c, seed = 200 * 2**20 + 3, 2, 1, 77
        t = torch.full((size + 64,), GUARD, dtype=torch.uint8, device="cuda")
        gpu_ctx.dgen_fill(t, size, dedup=d, compress=c, seed=seed)
        h = t.cpu().numpy()
        fn, fd = P.compress_ratio(c)
        assert np.array_equal(h[:size], oracle.dgen_fill(size, d, fn, fd, seed))
        assert (h[size:] == GUARD).all()
    finally:
        for mode in (0, 1):
            gpu_ctx.set_keystream_shape(mode)
            gpu_ctx.set_keystream_xcd_group(mode, 0)


def test_keystream_two_chunks_per_wave_vs_oracle(gpu_ctx, torch, oracle):
    """32 lanes per chunk (4096-draw lanes over 1 MiB chunks): every wave holds
    two chunks, so the lanes take the per-lane vector jump.  Large enough that
    the launch keeps 32 lanes per chunk; K2 and DG1, every byte vs the oracle.
    (Two scalar sequences per wave were tried: DG1 at 4096 draws ran no faster
    than at 2048, profiles/r02/diag/ks/dg1_two_chunk_waves_ab.log.)"""
    try:
        for mode in (0, 1):
            gpu_ctx.set_keystream_shape(mode, 64, 1, 0, 4096)
        length, chunk, sb = 2 * 2**30 + 5, 2**20, 5
        t = torch.full((length + 64,), GUARD, dtype=torch.uint8, device="cuda")
        gpu_ctx.xoshiro_fill(t, length, chunk_bytes=chunk, seed_base=sb)
        h = t.cpu().numpy()
        assert np.array_equal(h[:length], oracle.xoshiro_chunks(length, chunk, sb))
        assert (h[length:] == GUARD).all()
        del t, h
        size = 2 * 2**30 + 3
        t = torch.full((size + 64,), GUARD, dtype=torch.uint8, device="cuda")
        gpu_ctx.dgen_fill(t, size, dedup=2, compress=1, seed=17)
        h = t.cpu().numpy()
        assert np.array_equal(h[:size], oracle.dgen_fill(size, 2, 0, 1, 17))
        assert (h[size:] == GUARD).all()
    finally:
        for mode in (0, 1):
            gpu_ctx.set_keystream_shape(mode)


def test_keystream_full_size_properties(gpu_ctx, torch, oracle):
    """8 GiB of 2 MiB chunks: sampled chunks bit-exact, bytes ~uniform."""
    n = 8 * 2**30
    t = torch.empty(n, dtype=torch.uint8, device="cuda")
    gpu_ctx.xoshiro_fill(t, chunk_bytes=2 * 2**20, seed_base=0)
    for k in (0, 1, 1000, 4095):
        exp = oracle.xoshiro_chunks(2 * 2**20, 2 * 2**20, k)
        assert np.array_equal(t[k * 2**21:(k + 1) * 2**21].cpu().numpy(), exp), k
    hist = torch.bincount(t[:2**30].to(torch.int32), minlength=256).double()
    assert float((hist.max() - hist.min()) / hist.mean()) < 0.01


def test_launch_splitting_large_grids(gpu_ctx, torch, oracle, base):
    """Large grids: a 17 GiB object and 17.5 GiB batches with 1, 2 and 4 waves
    per block (AQL grid sizes are 32-bit work-item counts; batch launches are
    capped at the largest multiple of 256 workgroups that fits, the 2D stream
    kernel at 2^22 per dimension); checked against the oracle."""
    size = 17 * 2**30 + 4096 * 3 + 5
    t = torch.empty(size, dtype=torch.uint8, device="cuda")
    gpu_ctx.fill_controlled(t, size, dedup=1, compress=3, entropy=123)
    torch.cuda.synchronize()
    exp = oracle.fill_controlled(size, 1, 2, 3, 123, base)
    for lo, hi in [(0, 2**24), (2**34 - 2**20, 2**34 + 2**20), (size - 2**24, size)]:
        assert np.array_equal(t[lo:hi].cpu().numpy(), exp[lo:hi]), (lo, hi)
    del t, exp
    for waves in (1, 2, 4):
        gpu_ctx.set_waves_per_block(waves)
        osz = 5 * 2**29 + 100                                  # 2.5 GiB + 100 B
        stride = (osz + 4095) // 4096 * 4096
        objs = [(k * stride, osz, P.object_entropy(SEED_BASE, k), 2, 2) for k in range(7)]
        out = torch.empty(7 * stride, dtype=torch.uint8, device="cuda")
        gpu_ctx.fill_batch(out, objs)
        torch.cuda.synchronize()
        exp = oracle.fill_controlled(osz, 2, 1, 2, P.object_entropy(SEED_BASE, 6), base)
        assert np.array_equal(out[6 * stride:6 * stride + osz].cpu().numpy(), exp), waves
        del out, exp
    gpu_ctx.set_waves_per_block(0)


def test_block_windows_equal_rand_crate_vectors(gpu_ctx, torch):
    """Pinned without the oracle: block 0 at entropy 0 is seeded
    SmallRng::seed_from_u64(0) (src/data_gen.rs:202-203), so its two 32-byte
    windows (:217, :220) are next_u64 outputs 0-3 and 4-7 of rand 0.9's own
    `stable_seed_from_u64` test, little-endian; block 1 at entropy 2^64-1 is
    seed 0 again (u + E wraps)."""
    kat = load("kat.json")["rand_seed_from_u64_0_x10"]
    want1 = b"".join(v.to_bytes(8, "little") for v in kat[:4])
    want2 = b"".join(v.to_bytes(8, "little") for v in kat[4:8])
    t = torch.empty(2 * 4096, dtype=torch.uint8, device="cuda")
    gpu_ctx.fill_controlled(t, 4096, dedup=1, compress=1, entropy=0)
    torch.cuda.synchronize()
    h = bytes(t[:4096].cpu().numpy())
    assert h[:32] == want1 and h[2048:2080] == want2
    u = torch.empty(2 * 4096, dtype=torch.uint8, device="cuda")
    gpu_ctx.fill_controlled(u, 2 * 4096, dedup=1, compress=1, entropy=2**64 - 1)
    torch.cuda.synchronize()
    h = bytes(u[4096:].cpu().numpy())
    assert h[:32] == want1 and h[2048:2080] == want2


def test_batch_launch_split_path(tmp_path):
    """The split path of batch launches, forced in a child process with a small
    cap (S3DG_BATCH_GRID_CAP=2^20 workgroups): a 5 GiB tiled fill and a batch
    of 3 x 1.5 GiB objects cross several launch boundaries; every byte of the
    boundary windows and the last object equals the oracle."""
    import subprocess
    import sys
    script = r'''
import sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import torch
import s3dlio_amd as S
from oracle import oracle_c as OC
from oracle import oracle_py as P
base = OC.base_block(S.DEFAULT_BASE_SEED)
ctx = S.Context(0, base_seed=S.DEFAULT_BASE_SEED)
size = 5 * 2**30 + 4096 + 7
t = torch.empty(size, dtype=torch.uint8, device="cuda")
ctx.fill_controlled(t, size, dedup=3, compress=2, entropy=55)
torch.cuda.synchronize()
exp = OC.fill_controlled(size, 3, 1, 2, 55, base)
for k in range(1, 6):                      # every 2^20-block (4 GiB) launch boundary +- 1 MiB
    lo = max(0, k * 2**32 - 2**20); hi = min(size, k * 2**32 + 2**20)
    if lo < size:
        assert np.array_equal(t[lo:hi].cpu().numpy(), exp[lo:hi]), k
assert np.array_equal(t[size - 2**20:].cpu().numpy(), exp[size - 2**20:])
del t, exp
osz = 3 * 2**29 + 9
stride = (osz + 4095) // 4096 * 4096
objs = [(k * stride, osz, P.object_entropy(0x5EED000000000001, k), 1, 1) for k in range(3)]
out = torch.empty(3 * stride, dtype=torch.uint8, device="cuda")
ctx.fill_batch(out, objs)
torch.cuda.synchronize()
exp = OC.fill_controlled(osz, 1, 0, 1, P.object_entropy(0x5EED000000000001, 2), base)
assert np.array_equal(out[2 * stride:2 * stride + osz].cpu().numpy(), exp)
print("split ok")
'''
    p = tmp_path / "split.py"
    p.write_text(script)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, S3DG_BATCH_GRID_CAP=str(1 << 20))
    r = subprocess.run([sys.executable, str(p), root], env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0 and "split ok" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]
