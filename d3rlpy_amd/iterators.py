"""Minibatch iterators over an HBM-resident dataset.

Same names, constructor arguments and epoch semantics as
d3rlpy/iterators/{base,random_iterator,round_iterator}.py, but ``__next__``
returns a ``DeviceBatch`` filled by one gather launch instead of building a
Python list of Transition objects and a host TransitionMiniBatch
(iterators/base.py:46-64).

Index streams:
  RandomIterator  index_source="device" (default): Philox on the GPU,
                  i.i.d. uniform over transitions (statistically the
                  reference's stream, not bit-identical);
                  index_source="numpy": exactly the reference's stream — one
                  ``np.random.randint(len(transitions))`` per sample from
                  numpy's global RNG (random_iterator.py:38-41) — uploaded
                  each step (B int64 values).
  RoundIterator   ``np.random.shuffle(np.arange(n))`` once per epoch
                  (round_iterator.py:39-48), uploaded once per epoch; each
                  step gathers a contiguous slice of it.
"""
from __future__ import annotations

from typing import Tuple, Optional

import numpy as np
import torch

from .dataset import DeviceDataset


class TransitionIterator:
    def __init__(self, dataset: DeviceDataset, batch_size: int, n_steps: int = 1,
                 gamma: float = 0.99, n_frames: int = 1, real_ratio: float = 1.0,
                 generated_maxlen: int = 100000, out=None):
        if real_ratio != 1.0:
            raise NotImplementedError("generated-transition mixing (model-based) is out of scope")
        self._dataset = dataset
        self._batch_size = batch_size
        self._n_steps = n_steps
        self._gamma = gamma
        self._n_frames = n_frames
        self._real_ratio = real_ratio
        self._real_batch_size = batch_size
        self._count = 0
        self._out = out if out is not None else dataset.alloc_batch(batch_size, n_frames)

    def __iter__(self):
        self.reset()
        return self

    def __next__(self):
        if self._has_finished():
            raise StopIteration
        self._gather(self._out)
        self._count += 1
        return self._out

    def reset(self) -> None:
        self._count = 0
        self._reset()

    def _reset(self) -> None:
        pass

    def _gather(self, out) -> None:
        raise NotImplementedError

    def _has_finished(self) -> bool:
        raise NotImplementedError

    def __len__(self) -> int:
        raise NotImplementedError

    def size(self) -> int:
        return len(self._dataset)

    @property
    def dataset(self) -> DeviceDataset:
        return self._dataset

    @property
    def batch(self):
        return self._out


class RandomIterator(TransitionIterator):
    def __init__(self, dataset: DeviceDataset, n_steps_per_epoch: int, batch_size: int,
                 n_steps: int = 1, gamma: float = 0.99, n_frames: int = 1,
                 real_ratio: float = 1.0, generated_maxlen: int = 100000,
                 index_source: str = "device", seed: Optional[int] = None, out=None,
                 shard: Tuple[int, int] = (0, 1)):
        """``shard=(rank, world)``: this learner's slice [rank*B, (rank+1)*B)
        of one global stream of world*B indices per step (every rank must use
        the same ``seed``) — the data-parallel sampler of SURVEY §8e.  With
        world > 1 and ``seed=None`` rank 0's seed is broadcast over the
        initialised torch.distributed group (an error if there is none)."""
        super().__init__(dataset, batch_size, n_steps, gamma, n_frames, real_ratio,
                         generated_maxlen, out)
        self._rank, self._world = int(shard[0]), int(shard[1])
        if not 0 <= self._rank < self._world:
            raise ValueError("shard must be (rank, world) with 0 <= rank < world")
        self._n_steps_per_epoch = n_steps_per_epoch
        if index_source not in ("device", "numpy"):
            raise ValueError("index_source must be 'device' or 'numpy'")
        self._index_source = index_source
        if seed is None and index_source == "numpy":
            seed = 0  # unused: the numpy stream draws from numpy's global RNG,
            # which must not be advanced here (the reference draws nothing at
            # construction, random_iterator.py:18-36)
        if seed is None:
            seed = int(np.random.randint(0, 2**62))
            if self._world > 1:
                import torch.distributed as dist
                if not dist.is_initialized():
                    raise ValueError("shard world > 1 needs an explicit seed shared by every "
                                     "rank, or an initialised torch.distributed group")
                from .dp import broadcast_seed
                seed = broadcast_seed(seed)
        self._seed = int(seed)
        self.indices = torch.zeros(batch_size, dtype=torch.int64, device=dataset.device)

    def _gather(self, out) -> None:
        if self._index_source == "numpy":
            idx = np.array([np.random.randint(len(self._dataset))
                            for _ in range(self._batch_size * self._world)], dtype=np.int64)
            idx = idx[self._rank * self._batch_size:(self._rank + 1) * self._batch_size]
            self.indices.copy_(torch.from_numpy(idx), non_blocking=False)
            self._dataset.gather(out, self.indices, self._n_steps, self._gamma, self._n_frames)
        else:
            self._dataset.gather(out, None, self._n_steps, self._gamma, self._n_frames,
                                 seed=self._seed, idx_out=self.indices,
                                 row_offset=self._rank * self._batch_size)

    def _has_finished(self) -> bool:
        return self._count >= self._n_steps_per_epoch

    def __len__(self) -> int:
        return self._n_steps_per_epoch


class RoundIterator(TransitionIterator):
    def __init__(self, dataset: DeviceDataset, batch_size: int, n_steps: int = 1,
                 gamma: float = 0.99, n_frames: int = 1, real_ratio: float = 1.0,
                 generated_maxlen: int = 100000, shuffle: bool = True, out=None):
        super().__init__(dataset, batch_size, n_steps, gamma, n_frames, real_ratio,
                         generated_maxlen, out)
        self._shuffle = shuffle
        self._perm = torch.arange(len(dataset), dtype=torch.int64, device=dataset.device)
        self._index = 0

    def _reset(self) -> None:
        indices = np.arange(len(self._dataset))
        if self._shuffle:
            np.random.shuffle(indices)
        self._perm.copy_(torch.from_numpy(indices))
        self._index = 0

    def _gather(self, out) -> None:
        idx = self._perm[self._index:self._index + self._batch_size]
        self._dataset.gather(out, idx, self._n_steps, self._gamma, self._n_frames)
        self._index += self._batch_size

    def _has_finished(self) -> bool:
        # full batches only (the reference's __len__ is n // batch_size)
        return self._index + self._batch_size > len(self._dataset)

    def __len__(self) -> int:
        return len(self._dataset) // self._real_batch_size
