"""Object-stream sharding across GPUs.

Objects are independent (per-object entropy, §8a A9), so each rank owns a
contiguous object-index range and no collective touches the data path.  The
only inter-rank traffic is control: a barrier and a max over per-rank
elapsed times, on a CPU (gloo) process group.
"""
from __future__ import annotations

import os


def object_range(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """[lo, hi) object indices owned by `rank` (contiguous, sizes differ by <= 1)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    q, r = divmod(n_total, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def dist_env() -> tuple[int, int, int]:
    """(rank, world, local_rank) from torchrun's environment (1 process: 0,1,0)."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


class ControlPlane:
    """Barrier + max-reduce over ranks (gloo, CPU tensors only)."""

    def __init__(self):
        self.rank, self.world, self.local_rank = dist_env()
        self.pg = None
        if self.world > 1:
            import torch.distributed as dist
            if not dist.is_initialized():
                dist.init_process_group("gloo")
            self.pg = dist

    def barrier(self) -> None:
        if self.pg is not None:
            self.pg.barrier()

    def max(self, x: float) -> float:
        if self.pg is None:
            return float(x)
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64)
        self.pg.all_reduce(t, op=self.pg.ReduceOp.MAX)
        return float(t.item())

    def sum(self, x: float) -> float:
        if self.pg is None:
            return float(x)
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64)
        self.pg.all_reduce(t, op=self.pg.ReduceOp.SUM)
        return float(t.item())

    def gather(self, obj) -> list:
        """Every rank's `obj` (a small picklable value), in rank order."""
        if self.pg is None:
            return [obj]
        out = [None] * self.world
        self.pg.all_gather_object(out, obj)
        return out

    def close(self) -> None:
        if self.pg is not None and self.pg.is_initialized():
            self.pg.destroy_process_group()
