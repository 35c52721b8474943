"""GPU: the N>1 launcher path of bench.py on the HIP library (VERDICT r05
next #4).  `bench.py --gpus 2` outside torch.distributed.run starts the ranks
as a child torch.distributed.run before anything touches the GPU
(bench.py:launch_ranks); each rank generates its own object range with no
collective on the data path (the fan-out of
src/s3_utils.rs:1824-1868) and verifies its last writes against the C
oracle; rank 0 prints one line with every rank's range.  On the one-GPU box
both ranks share device 0 (--device-override 0, rehearsal only)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=240):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device-override", "0",
           "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-ceiling"] + args
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-4000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-3000:]
    return json.loads(lines[0])


def _disjoint(ranks, per_rank):
    rs = sorted(tuple(r["object_range"]) for r in ranks)
    assert [r["rank"] for r in ranks] == [0, 1]
    assert all(hi - lo == per_rank for lo, hi in rs), rs
    assert rs[0][1] <= rs[1][0], rs


def test_two_ranks_config2():
    j = _run(["--config", "2", "--objects", "32", "--no-d2h"])
    assert j["n_gpus"] == 2 and j["verified_vs_oracle"] is True
    assert j["config"]["objects_per_rank"] == 32
    assert j["config"]["bytes_per_step_all_ranks"] == 2 * 32 * 8 * (1 << 20)
    _disjoint(j["ranks"], 32)


def test_two_ranks_config5_d2h_full():
    j = _run(["--config", "5", "--objects", "64", "--d2h-full"])
    assert j["n_gpus"] == 2 and j["verified_vs_oracle"] is True
    d = j["d2h_inclusive"]
    assert d and d["verified_vs_oracle"] is True and d["whole_job_GiBps"] > 0
    # config 5 shards one object stream (strong scaling): 64 objects over 2 ranks
    per = j["config"]["objects_per_rank"]
    _disjoint(j["ranks"], per)
    assert per == 32 and sum(r["object_range"][1] - r["object_range"][0] for r in j["ranks"]) == 64
