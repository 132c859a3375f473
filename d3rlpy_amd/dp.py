"""Data-parallel CQL (K4): one learner process per GPU.

Every CQL loss is a batch mean (cql_impl.py:217, ensemble_q_function.py:105,
sac_impl.py:121,138), so the mean over R ranks of the gradients of R disjoint
256-row shards is the gradient of the global R*256-row batch.  Per update
there are three gradient exchanges, in dependency order, each a SUM
all-reduce over RCCL (xGMI) followed by a 1/R scale inside the consumer
kernel (exact for power-of-two R):

  1  {temp, alpha} scalar gradients (8 B)      -> d3a_cql_loss phase 2
  2  critic gradient (one copy, ~606 KB)        -> Adam (critic)
  3  actor gradient (~310 KB)                   -> Adam (actor)

plus one for the logged losses.  Parameters, optimiser state and targets stay
bit-identical across ranks (identical all-reduce results, deterministic
kernels), so the soft target updates need no communication.  The index
stream is global: rank k gathers draws [k*B, (k+1)*B) of each step
(RandomIterator(shard=(k, R))).  Each rank draws its own policy noise
(independent Philox streams: the same distribution as slicing one global draw).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist


class DataParallel:
    """The exchange used by an Impl's update pipeline (any torch.distributed
    backend; RCCL ``nccl`` on the GPU path, where the collectives are
    captured into the update's HIP graph together with the kernels)."""

    def __init__(self, group: Optional[dist.ProcessGroup] = None):
        if not dist.is_initialized():
            raise RuntimeError("torch.distributed must be initialised for data parallelism")
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        # 1/world is exact for power-of-two worlds; otherwise the average
        # carries one extra rounding of the scale
        self.scale = 1.0 / self.world

    def all_reduce_sum(self, t: torch.Tensor) -> None:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> None:
        dist.broadcast(t, src=src, group=self.group)


def shard_rows(global_batch: int, rank: int, world: int) -> slice:
    """Rows of the global batch that ``rank`` owns."""
    if global_batch % world:
        raise ValueError("global batch must divide evenly over the ranks")
    b = global_batch // world
    return slice(rank * b, (rank + 1) * b)
