"""GPU: BASELINE configurations at full size, every byte checked against the
C oracle (oracle/s3dg_oracle.c; src/data_gen.rs:151-224 semantics).

The GPU writes the whole configuration (78 GiB for configs 2/3, 69 GB for
config 4) into HBM exactly as bench.py does; the oracle regenerates it on the
host threads in 2 GiB windows, each window is uploaded and compared on the
device with torch.equal.  Config 5 (100 000 objects, 839 GB) is checked whole,
as ten 10 000-object ring passes (bench.py's N=1 ring).

Every buffer is poisoned (0xA5) before the fill, so a block the kernel never
wrote cannot pass for one a previous fill left behind, and the stream
configurations sit between two 64 MiB guard regions that must still hold the
poison afterwards (no store outside the objects).
"""
import concurrent.futures as cf
import ctypes
import os

import pytest

from oracle import oracle_py as P

pytestmark = pytest.mark.gpu
MiB = 1 << 20
SEED_BASE = 0x5EED000000000001        # bench.py / SURVEY.md §8d
BASE_SEED = 0xBA5EB10C00000000
WINDOW = 2 << 30
GUARD = 64 * MiB
POISON = 0xA5
THREADS = max(1, min(16, os.cpu_count() or 1))


@pytest.fixture(scope="module")
def env():
    import torch
    import s3dlio_amd as S
    from oracle import oracle_c as OC
    ctx = S.Context(0, base_seed=BASE_SEED)
    base = OC.base_block(BASE_SEED)
    host = torch.empty(WINDOW, dtype=torch.uint8).pin_memory()
    chk = torch.empty(WINDOW, dtype=torch.uint8, device="cuda")
    yield torch, S, OC, ctx, base, host, chk
    ctx.close()


def _compare(torch, host, chk, dev_slice, nbytes):
    chk[:nbytes].copy_(host[:nbytes])
    return bool(torch.equal(chk[:nbytes], dev_slice))


@pytest.mark.parametrize("cfg,n,first,d,c", [
    (2, 10000, 0, 1, 1),
    (3, 10000, 0, 4, 2),
] + [(5, 10000, f, 2, 3) for f in range(0, 100000, 10000)])
def test_stream_config_every_byte(env, cfg, n, first, d, c):
    torch, S, OC, ctx, base, host, chk = env
    size = 8 * MiB
    fn, fd = P.compress_ratio(c)
    whole = torch.empty(n * size + 2 * GUARD, dtype=torch.uint8, device="cuda")
    whole.fill_(POISON)
    dev = whole[GUARD:GUARD + n * size]
    ctx.fill_stream(dev, obj_size=size, n_objs=n, dedup=d, compress=c, seed_base=SEED_BASE, first_obj=first)
    torch.cuda.synchronize()
    assert int((whole[:GUARD] != POISON).sum()) == 0, "store before the buffer"
    assert int((whole[GUARD + n * size:] != POISON).sum()) == 0, "store past the buffer"
    per = WINDOW // size
    hnp = host.numpy()
    for s0 in range(0, n, per):
        k = min(per, n - s0)
        OC.fill_stream(size, k, d, fn, fd, SEED_BASE, first + s0, base, threads=THREADS, out=hnp[:k * size])
        assert _compare(torch, host, chk, dev[s0 * size:(s0 + k) * size], k * size), (cfg, s0)
    del dev, whole


def test_batch_config4_every_byte(env):
    torch, S, OC, ctx, base, host, chk = env
    from bench import log_uniform_sizes
    n = 10000
    sizes = log_uniform_sizes(n)
    fn, fd = P.compress_ratio((3, 2))
    offs, cur = [], 0
    for sz in sizes:
        offs.append(cur)
        cur += (sz + 4095) // 4096 * 4096
    dev = torch.empty(cur, dtype=torch.uint8, device="cuda")
    dev.fill_(POISON)
    ctx.fill_batch(dev, [(offs[j], sizes[j], P.object_entropy(SEED_BASE, j), 2, (3, 2)) for j in range(n)])
    torch.cuda.synchronize()
    lib = OC.lib()
    bptr = base.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
    hbase = host.data_ptr()
    j = 0
    with cf.ThreadPoolExecutor(THREADS) as pool:
        while j < n:
            w0 = offs[j]                      # window [w0, w1) of whole objects
            k = j
            while k < n and offs[k] + sizes[k] - w0 <= WINDOW:
                k += 1
            assert k > j, "an object larger than the window"
            w1 = offs[k - 1] + sizes[k - 1]

            def one(q):
                p = ctypes.cast(hbase + offs[q] - w0, ctypes.POINTER(ctypes.c_uint8))
                lib.s3dgo_fill_controlled(p, sizes[q], 2, fn, fd, P.object_entropy(SEED_BASE, q), bptr)
            list(pool.map(one, range(j, k)))
            # the gaps between objects are not generated: copy them from the device side
            for q in range(j, k - 1):
                a, b = offs[q] + sizes[q], offs[q + 1]
                if b > a:
                    host[a - w0:b - w0].copy_(dev[a:b])
            assert _compare(torch, host, chk, dev[w0:w1], w1 - w0), (j, k)
            j = k
    del dev


def test_keystream_config6_every_byte(env):
    """bench.py --config 6: 10 000 x 8 MiB written as 2 MiB Xoshiro256++ chunks
    (the npz x-fill, src/data_formats/npz.rs:376-383), chunk k seeded k."""
    torch, S, OC, ctx, base, host, chk = env
    total, chunk = 10000 * 8 * MiB, 2 * MiB
    dev = torch.empty(total, dtype=torch.uint8, device="cuda")
    dev.fill_(POISON)
    ctx.xoshiro_fill(dev, total, chunk_bytes=chunk, seed_base=0)
    torch.cuda.synchronize()
    lib = OC.lib()
    hbase = host.data_ptr()
    per_task = 64 * chunk

    def one(args):
        off, k0, n = args
        lib.s3dgo_xoshiro_chunks(ctypes.cast(hbase + off, ctypes.POINTER(ctypes.c_uint8)), n, chunk, k0)
    with cf.ThreadPoolExecutor(THREADS) as pool:
        for w0 in range(0, total, WINDOW):
            n = min(WINDOW, total - w0)
            tasks = [(o, (w0 + o) // chunk, min(per_task, n - o)) for o in range(0, n, per_task)]
            list(pool.map(one, tasks))
            assert _compare(torch, host, chk, dev[w0:w0 + n], n), w0
    del dev
