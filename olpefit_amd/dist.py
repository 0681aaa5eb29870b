"""Host-side orchestration of the walker-sharded multi-GPU run.

One process per GPU.  Walkers are independent, so rank r owns a contiguous range of
global walker indices and seeds walker w with ``base + w``: the chains do not depend
on the GPU count.  Ranks talk only through the host group (barrier, timing max, the
128-byte RCCL id) and, at the end, through RCCL in libolpe (all-gather of states,
all-reduce of moments).  The host group is torch.distributed over gloo (CPU); it
carries no sampling data.
"""
from __future__ import annotations

import os

import numpy as np


def env():
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard(total: int, world: int, rank: int):
    """Contiguous shard [w0, w0 + n) of ``total`` walkers for ``rank`` (strong split)."""
    lo = (rank * total) // world
    hi = ((rank + 1) * total) // world
    return lo, hi - lo


def walker_seeds(base: int, w0: int, n: int) -> np.ndarray:
    """np.random.seed values of walkers w0 .. w0+n-1 (global index -> seed)."""
    return ((int(base) + w0 + np.arange(n, dtype=np.int64)) & 0xFFFFFFFF).astype(np.uint32)


class HostGroup:
    """Barrier / max / broadcast over gloo; a no-op group when world == 1."""

    def __init__(self, rank: int, world: int, timeout_min: float = 10.0):
        self.rank, self.world = rank, world
        self.dist = None
        if world > 1:
            import datetime

            import torch.distributed as dist
            if not dist.is_initialized():
                dist.init_process_group("gloo", rank=rank, world_size=world,
                                        timeout=datetime.timedelta(minutes=timeout_min))
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def allmax(self, x: float) -> float:
        if not self.dist:
            return float(x)
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def broadcast(self, obj, src: int = 0):
        if not self.dist:
            return obj
        box = [obj if self.rank == src else None]
        self.dist.broadcast_object_list(box, src=src)
        return box[0]

    def close(self):
        if self.dist and self.dist.is_initialized():
            self.dist.destroy_process_group()
