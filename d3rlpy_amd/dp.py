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
(RandomIterator(shard=(k, R)), whose seed is rank 0's, broadcast).  Each rank
draws its own policy noise: rank 0's workspace seed is broadcast and the rank
is folded in (``rank_seed``), so the ranks' Philox streams are distinct even
when every process called ``torch.manual_seed`` with the same value (the same
distribution as slicing one global draw).
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

    def shared_seed(self, seed: int) -> int:
        """Rank 0's ``seed`` on every rank."""
        return broadcast_seed(seed, self.group)

    def rank_seed(self, seed: int) -> int:
        """A per-rank Philox key derived from rank 0's ``seed``."""
        return fold_rank(self.shared_seed(seed), self.rank)


_M64 = (1 << 64) - 1


def _splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & _M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _M64
    return x ^ (x >> 31)


def fold_rank(seed: int, rank: int) -> int:
    """Distinct 62-bit keys per rank (rank 0 keeps a mixed copy of ``seed``)."""
    return _splitmix64((int(seed) & _M64) ^ _splitmix64(int(rank))) >> 2


def broadcast_seed(seed: int, group: Optional[dist.ProcessGroup] = None) -> int:
    """Rank 0's integer ``seed`` on every rank of ``group`` (a one-element
    int64 tensor on the device the backend needs)."""
    dev = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.tensor([int(seed)], dtype=torch.int64, device=dev)
    dist.broadcast(t, src=0, group=group)
    return int(t.item())


def shard_rows(global_batch: int, rank: int, world: int) -> slice:
    """Rows of the global batch that ``rank`` owns."""
    if global_batch % world:
        raise ValueError("global batch must divide evenly over the ranks")
    b = global_batch // world
    return slice(rank * b, (rank + 1) * b)
