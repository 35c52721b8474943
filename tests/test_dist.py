"""CPU, world_size=2 over gloo: the N>1 path shards objects with no data-path
collective.  Each rank generates its own object range (oracle as the CPU
stand-in for the device fill, which has identical per-object semantics); the
concatenation must equal the single-process stream, and the control plane
(barrier, max/sum) must agree across ranks."""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from s3dlio_amd.shard import object_range

SEED_BASE = 0x5EED000000000001


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_total, size, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from oracle import oracle_c as OC
    from s3dlio_amd.shard import ControlPlane
    cp = ControlPlane()
    lo, hi = object_range(n_total, cp.rank, cp.world)
    base = OC.base_block(0xBA5EB10C00000000)
    out = OC.fill_stream(size, hi - lo, 2, 2, 3, SEED_BASE, lo, base)
    cp.barrier()
    mx = cp.max(float(rank + 1))
    tot = cp.sum(float(hi - lo))
    q.put((rank, lo, hi, hashlib.sha256(out.tobytes()).hexdigest(), mx, tot))
    cp.close()


@pytest.mark.parametrize("n_total,world", [(7, 2), (64, 2), (37, 4), (83, 8)])
def test_two_rank_sharding_matches_single_stream(oracle, n_total, world):
    size = 4096 * 3 + 100
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, size, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    base = oracle.base_block(0xBA5EB10C00000000)
    full = oracle.fill_stream(size, n_total, 2, 2, 3, SEED_BASE, 0, base)
    for rank, lo, hi, digest, mx, tot in res:
        assert digest == hashlib.sha256(full[lo * size:hi * size].tobytes()).hexdigest()
        assert mx == float(world) and tot == float(n_total)
    assert res[0][1] == 0 and res[-1][2] == n_total
    assert all(res[k][2] == res[k + 1][1] for k in range(world - 1))


@pytest.mark.parametrize("n,w", [(0, 1), (1, 8), (7, 2), (100000, 8), (12500, 3)])
def test_object_range_partition(n, w):
    rs = [object_range(n, r, w) for r in range(w)]
    assert rs[0][0] == 0 and rs[-1][1] == n
    assert all(rs[k][1] == rs[k + 1][0] for k in range(w - 1))
    sizes = [hi - lo for lo, hi in rs]
    assert max(sizes) - min(sizes) <= 1


def test_entropy_independent_of_world_size(oracle):
    """Object j's bytes depend only on (seed_base, j): any GPU count gives the
    same objects."""
    base = oracle.base_block(0xBA5EB10C00000000)
    a = oracle.fill_stream(8192, 6, 1, 0, 1, SEED_BASE, 0, base)
    b = np.concatenate([oracle.fill_stream(8192, 2, 1, 0, 1, SEED_BASE, k, base) for k in (0, 2, 4)])
    assert np.array_equal(a, b)


def test_bench_config_math():
    """bench.py's config 4 sizes follow SURVEY.md §8d (log-uniform 4 KiB..64 MiB,
    SplitMix64(seed 4), mean (b-a)/ln(b/a) ~= 6.9 MB) and config 5 splits
    100 000 objects over 8 ranks as 12 500 each."""
    import math
    import bench
    s = bench.log_uniform_sizes(10000)
    assert min(s) >= 4096 and max(s) <= 64 << 20
    mean = (64 * 2**20 - 4096) / math.log(64 * 2**20 / 4096)
    assert abs(sum(s) / len(s) - mean) / mean < 0.05
    assert s == bench.log_uniform_sizes(10000)                  # deterministic
    assert sum(s) == 68647437822                                 # the bytes bench.py and the profiles report
    assert [object_range(100000, r, 8) for r in (0, 7)] == [(0, 12500), (87500, 100000)]
