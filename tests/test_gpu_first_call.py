"""GPU: the first keystream call of a fresh context builds its lane jump
table on the host (x^(z0 + k*span) mod P for every lane k of a chunk).  Round
5 builds it with one product mod P per lane (word-wise GF(2) products) where
round 4 raised one power per lane bit by bit (~3 ms each, ~1.6 s for a
512-lane table).  A first small DG1 / K2 call (the small-launch rule spreads
a chunk over up to 512 lanes) now returns within a fraction of a second, with
the same bytes as the oracle."""
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
MiB = 1 << 20


@pytest.mark.parametrize("kind", ["dgen", "k2"])
def test_first_small_call_latency(kind, oracle, gpu_ctx):
    import torch
    import s3dlio_amd as S
    buf = torch.zeros(3 * MiB + 64, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    ctx = S.Context(0, base_seed=S.DEFAULT_BASE_SEED)
    t0 = time.perf_counter()
    if kind == "dgen":
        ctx.dgen_fill(buf, 3 * MiB + 5, dedup=1, compress=1, seed=31337)
    else:
        ctx.xoshiro_fill(buf, 3 * MiB, seed_base=99)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ctx.close()
    if kind == "dgen":
        exp = np.frombuffer(oracle.dgen_fill(3 * MiB + 5, 1, 0, 1, 31337), dtype=np.uint8)
        assert np.array_equal(buf[:3 * MiB + 5].cpu().numpy(), exp)
    else:
        exp = oracle.xoshiro_chunks(3 * MiB, 2 * MiB, 99)
        assert bytes(buf[:3 * MiB].cpu().numpy()) == bytes(exp)
    assert dt < 0.5, f"first {kind} call took {dt:.3f} s"
