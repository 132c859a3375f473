"""MDP dataset model and its HBM-resident form.

Host data model (API of d3rlpy/dataset.pyx): ``MDPDataset`` (:125) splits the
flat arrays into ``Episode``s (:44-67, :602), each exposing linked
``Transition``s (:70-116, :792).  These are plain Python/numpy objects used
to *describe* the data and to build scalers; they are not on the update path.

Device form: ``DeviceDataset`` uploads the dataset once as a structure of
arrays plus a transition table, and ``gather`` fills a ``DeviceBatch`` with
one kernel launch (d3a_gather_batch) — the replacement of
TransitionMiniBatch/_assign_to_batch (dataset.pyx:1139-1342) and of the
per-sample ``np.random.randint`` of RandomIterator (iterators/random_iterator.py:38-41).

HBM layout (n_rows = steps stored, n_trans = transitions):
    obs      [n_rows][D] f32        or frames [n_rows][C*H*W] u8
    act      [n_rows][A] f32        or act_i  [n_rows] i32
    rew      [n_rows] f32
    t_row, t_ep_start, t_ep_last    [n_trans] i64
    t_terminal                      [n_trans] u8
Transitions of an episode are consecutive (next_transition = i + 1 unless
i == t_ep_last[i]); a non-terminal episode of length L has L-1 transitions
and a terminal one L, the last pointing at the all-zero dummy observation
(dataset.pyx:85-95).
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch


def _check_discrete_action(actions) -> bool:
    """dataset.pyx:119-122."""
    float_actions = np.array(actions, dtype=np.float32)
    int_actions = np.array(actions, dtype=np.int32)
    return bool(np.all(float_actions == int_actions))


class Transition:
    """dataset.pyx:792-1033 (host object; links built by Episode)."""

    __slots__ = ("observation_shape", "action_size", "observation", "action", "reward",
                 "next_observation", "terminal", "prev_transition", "next_transition", "_index")

    def __init__(self, observation_shape, action_size, observation, action, reward,
                 next_observation, terminal, prev_transition=None, next_transition=None):
        self.observation_shape = tuple(observation_shape)
        self.action_size = action_size
        self.observation = observation
        self.action = action
        self.reward = reward
        self.next_observation = next_observation
        self.terminal = terminal
        self.prev_transition = prev_transition
        self.next_transition = next_transition
        self._index = None

    def get_observation_shape(self):
        return self.observation_shape

    def get_action_size(self):
        return self.action_size

    @property
    def is_discrete(self) -> bool:
        return not isinstance(self.action, np.ndarray)

    def clear_links(self) -> None:
        self.prev_transition = None
        self.next_transition = None


class Episode:
    """dataset.pyx:602-790."""

    def __init__(self, observation_shape, action_size, observations, actions, rewards,
                 terminal=True):
        self.observation_shape = tuple(observation_shape)
        self.action_size = action_size
        self._observations = observations
        self._actions = actions
        self._rewards = np.asarray(rewards, dtype=np.float32).reshape(-1)
        self._terminal = bool(terminal)
        self._transitions: Optional[List[Transition]] = None

    @property
    def observations(self):
        return self._observations

    @property
    def actions(self):
        return self._actions

    @property
    def rewards(self):
        return self._rewards

    @property
    def terminal(self) -> bool:
        return self._terminal

    def __len__(self) -> int:
        return len(self._observations)

    def size(self) -> int:
        return len(self.transitions)

    def get_observation_shape(self):
        return self.observation_shape

    def get_action_size(self):
        return self.action_size

    def compute_return(self) -> float:
        """Undiscounted episode return (dataset.pyx:763-774)."""
        return float(np.sum(self._rewards))

    def n_transitions(self) -> int:
        L = len(self._observations)
        return L if self._terminal else max(L - 1, 0)

    @property
    def transitions(self) -> List[Transition]:
        """_to_transitions (dataset.pyx:70-116)."""
        if self._transitions is None:
            rets: List[Transition] = []
            n = len(self._observations)
            prev = None
            for i in range(n):
                if i == n - 1:
                    if self._terminal:
                        next_observation = np.zeros_like(self._observations[i])
                    else:
                        break
                else:
                    next_observation = self._observations[i + 1]
                env_terminal = float(self._terminal) if i == n - 1 else 0.0
                t = Transition(self.observation_shape, self.action_size, self._observations[i],
                               self._actions[i], float(self._rewards[i]), next_observation,
                               env_terminal, prev_transition=prev)
                if prev is not None:
                    prev.next_transition = t
                prev = t
                rets.append(t)
            self._transitions = rets
        return self._transitions

    def __iter__(self):
        return iter(self.transitions)


class MDPDataset:
    """dataset.pyx:125-600 (flat arrays -> episodes)."""

    def __init__(self, observations, actions, rewards, terminals, episode_terminals=None,
                 discrete_action=None):
        assert isinstance(observations, np.ndarray), "Observations must be numpy array."
        if observations.ndim == 4:
            assert observations.dtype == np.uint8, "Image observation must be uint8 array."
        elif observations.dtype != np.float32:
            observations = np.asarray(observations, dtype=np.float32)
        assert not np.isnan(observations).any() if observations.dtype != np.uint8 else True
        assert not np.isnan(np.asarray(actions, dtype=np.float64)).any()
        assert not np.isnan(np.asarray(rewards, dtype=np.float64)).any()
        assert not np.isnan(np.asarray(terminals, dtype=np.float64)).any()
        self._observations = observations
        self._rewards = np.asarray(rewards, dtype=np.float32).reshape(-1)
        self._terminals = np.asarray(terminals, dtype=np.float32).reshape(-1)
        if episode_terminals is None:
            self._episode_terminals = self._terminals
        else:
            self._episode_terminals = np.asarray(episode_terminals, dtype=np.float32).reshape(-1)
        if discrete_action is None:
            discrete_action = _check_discrete_action(actions)
        self.discrete_action = bool(discrete_action)
        if self.discrete_action:
            self._actions = np.asarray(actions, dtype=np.int32).reshape(-1)
        else:
            self._actions = np.asarray(actions, dtype=np.float32)
        self._episodes: Optional[List[Episode]] = None
        # bumped by every in-place change; device copies are keyed by it
        self._version = 0

    @property
    def version(self) -> int:
        return self._version

    @property
    def observations(self):
        return self._observations

    @property
    def actions(self):
        return self._actions

    @property
    def rewards(self):
        return self._rewards

    @property
    def terminals(self):
        return self._terminals

    @property
    def episode_terminals(self):
        return self._episode_terminals

    def episode_bounds(self) -> List[Tuple[int, int, bool]]:
        """(start, end_exclusive, terminal) per episode (_to_episodes, dataset.pyx:44-67)."""
        ends = np.nonzero(self._episode_terminals)[0]
        out, head = [], 0
        for i in ends:
            out.append((head, int(i) + 1, bool(self._terminals[i])))
            head = int(i) + 1
        return out

    @property
    def episodes(self) -> List[Episode]:
        if self._episodes is None:
            shape, asize = self.get_observation_shape(), self.get_action_size()
            self._episodes = [
                Episode(shape, asize, self._observations[s:e], self._actions[s:e],
                        self._rewards[s:e], terminal=t)
                for s, e, t in self.episode_bounds()
            ]
        return self._episodes

    def size(self) -> int:
        return len(self.episodes)

    def __len__(self) -> int:
        return self.size()

    def get_observation_shape(self):
        return tuple(self._observations.shape[1:])

    def get_action_size(self) -> int:
        if self.discrete_action:
            return int(np.max(self._actions) + 1)
        return int(self._actions.shape[1])

    def is_action_discrete(self) -> bool:
        return self.discrete_action

    def __iter__(self):
        return iter(self.episodes)

    def __getitem__(self, index):
        return self.episodes[index]

    def build_episodes(self) -> None:
        """Rebuild the episode view (dataset.pyx:552-566)."""
        self._episodes = None
        _ = self.episodes

    # -- growing the dataset (dataset.pyx:424-509) ------------------------------
    def append(self, observations, actions, rewards, terminals, episode_terminals=None):
        """Append flat arrays; episodes are re-derived from the new terminals."""
        observations = np.asarray(observations)
        shape = self.get_observation_shape()
        assert observations.shape[1:] == shape, f"Observation shape must be {shape}."
        if self.discrete_action:
            actions = np.asarray(actions).reshape(-1)
            if actions.size and int(actions.max()) >= self.get_action_size():
                import warnings
                warnings.warn(f"New action size is higher than {self.get_action_size()}.")
            self._actions = np.concatenate([self._actions, actions.astype(np.int32)])
        else:
            actions = np.asarray(actions, dtype=np.float32)
            assert actions.shape[1:] == (self.get_action_size(),), \
                f"Action size must be {self.get_action_size()}."
            self._actions = np.concatenate([self._actions, actions])
        if observations.dtype != self._observations.dtype:
            observations = observations.astype(self._observations.dtype)
        self._observations = np.concatenate([self._observations, observations])
        terminals = np.asarray(terminals, dtype=np.float32).reshape(-1)
        self._rewards = np.concatenate(
            [self._rewards, np.asarray(rewards, dtype=np.float32).reshape(-1)])
        self._terminals = np.concatenate([self._terminals, terminals])
        ep_terms = terminals if episode_terminals is None else \
            np.asarray(episode_terminals, dtype=np.float32).reshape(-1)
        self._episode_terminals = np.concatenate([self._episode_terminals, ep_terms])
        self._episodes = None
        self._version += 1

    def extend(self, dataset: "MDPDataset") -> None:
        """dataset.pyx:488-509."""
        assert self.is_action_discrete() == dataset.is_action_discrete(), \
            "Dataset must have discrete action-space."
        assert self.get_observation_shape() == dataset.get_observation_shape(), \
            f"Observation shape must be {self.get_observation_shape()}"
        self.append(dataset.observations, dataset.actions, dataset.rewards,
                    dataset.terminals, dataset.episode_terminals)

    # -- statistics (dataset.pyx:330-422) ---------------------------------------
    def compute_stats(self) -> dict:
        """Return / reward / action / observation summaries with 20-bin histograms."""
        def summary(x, axis=None):
            return {"mean": np.mean(x, axis=axis), "std": np.std(x, axis=axis),
                    "min": np.min(x, axis=axis), "max": np.max(x, axis=axis)}

        returns = np.array([ep.compute_return() for ep in self.episodes])
        stats = {"return": dict(summary(returns), histogram=np.histogram(returns, bins=20)),
                 "reward": dict(summary(self._rewards),
                                histogram=np.histogram(self._rewards, bins=20))}
        n_act = self.get_action_size()
        if self.discrete_action:
            counts = [int(np.count_nonzero(self._actions == a)) for a in range(n_act)]
            stats["action"] = {"histogram": [counts, np.arange(n_act)]}
        else:
            stats["action"] = dict(summary(self._actions, axis=0), histogram=[
                np.histogram(self._actions[:, j], bins=20) for j in range(n_act)])
        stats["observation"] = summary(self._observations, axis=0)
        return stats

    # -- persistence (dataset.pyx:511-550) --------------------------------------
    _FIELDS = ("observations", "actions", "rewards", "terminals", "episode_terminals")

    def dump(self, fname: str) -> None:
        """HDF5 (same dataset names as the reference) when h5py is importable and
        the name ends in .h5/.hdf5; otherwise an uncompressed .npz with the same keys."""
        arrays = {k: getattr(self, "_" + k) for k in self._FIELDS}
        if str(fname).endswith((".h5", ".hdf5")):
            try:
                import h5py
            except ImportError as e:
                raise ImportError("h5py is required for .h5 files; use a .npz name") from e
            with h5py.File(fname, "w") as f:
                for k, v in arrays.items():
                    f.create_dataset(k, data=v)
                f.create_dataset("discrete_action", data=self.discrete_action)
                f.create_dataset("version", data="1.0")
            return
        with open(fname, "wb") as fh:
            np.savez(fh, discrete_action=np.array(self.discrete_action),
                     version=np.array("1.0"), **arrays)

    @classmethod
    def load(cls, fname: str) -> "MDPDataset":
        if str(fname).endswith((".h5", ".hdf5")):
            import h5py
            with h5py.File(fname, "r") as f:
                data = {k: f[k][()] for k in cls._FIELDS if k in f}
                discrete = bool(f["discrete_action"][()])
        else:
            with np.load(fname, allow_pickle=False) as f:
                data = {k: f[k] for k in cls._FIELDS if k in f.files}
                discrete = bool(f["discrete_action"])
        return cls(data["observations"], data["actions"], data["rewards"], data["terminals"],
                   episode_terminals=data.get("episode_terminals"), discrete_action=discrete)


def transition_table(bounds: Sequence[Tuple[int, int, bool]]) -> Tuple[np.ndarray, ...]:
    """(t_row, t_ep_start, t_ep_last, t_terminal) for the given episode bounds."""
    rows, starts, lasts, terms = [], [], [], []
    base = 0
    for s, e, term in bounds:
        L = e - s
        n = L if term else max(L - 1, 0)
        if n == 0:
            continue
        r = np.arange(s, s + n, dtype=np.int64)
        rows.append(r)
        starts.append(np.full(n, s, dtype=np.int64))
        lasts.append(np.full(n, base + n - 1, dtype=np.int64))
        t = np.zeros(n, dtype=np.uint8)
        if term:
            t[-1] = 1
        terms.append(t)
        base += n
    if not rows:
        raise ValueError("empty dataset is not supported.")
    return (np.concatenate(rows), np.concatenate(starts), np.concatenate(lasts),
            np.concatenate(terms))


class DeviceDataset:
    """An MDPDataset resident in HBM, with the minibatch gather kernel."""

    def __init__(self, dataset: MDPDataset, device=None):
        from . import _native  # noqa: F401  (fail loudly if the library is missing)
        if not torch.cuda.is_available():
            raise RuntimeError("DeviceDataset needs a HIP device (no CPU fallback)")
        dev = torch.device(device if device is not None else torch.cuda.current_device())
        self.device = dev
        obs = dataset.observations
        self.is_image = obs.ndim == 4
        self.observation_shape = tuple(obs.shape[1:])
        self.discrete = dataset.is_action_discrete()
        self.action_size = dataset.get_action_size()
        t_row, t_s, t_l, t_t = transition_table(dataset.episode_bounds())
        self.n_trans = int(t_row.shape[0])
        self.n_rows = int(obs.shape[0])
        up = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        if self.is_image:
            self.frames = up(obs.reshape(self.n_rows, -1))
            self.obs = None
            self.frame_bytes = int(np.prod(obs.shape[1:]))
        else:
            self.obs = up(obs.reshape(self.n_rows, -1).astype(np.float32))
            self.frames = None
            self.frame_bytes = 0
        if self.discrete:
            self.act_i = up(dataset.actions.astype(np.int32))
            self.act = None
        else:
            self.act = up(dataset.actions.astype(np.float32))
            self.act_i = None
        self.rew = up(dataset.rewards.astype(np.float32))
        self.t_row, self.t_ep_start, self.t_ep_last, self.t_terminal = (up(t_row), up(t_s),
                                                                        up(t_l), up(t_t))
        self.ctr = torch.zeros(1, dtype=torch.int64, device=dev)
        self._draws = 0  # host draw counter of the vector-observation sampler
        self.ticket = torch.zeros(1, dtype=torch.int32, device=dev)

    def __len__(self) -> int:
        return self.n_trans

    def alloc_batch(self, batch_size: int, n_frames: int = 1):
        from .algos.impl_base import DeviceBatch
        dev, B = self.device, batch_size
        if self.is_image:
            c = self.observation_shape[0]
            shape = (B, n_frames * c) + tuple(self.observation_shape[1:])
            obs = torch.zeros(shape, dtype=torch.uint8, device=dev)
            nobs = torch.zeros(shape, dtype=torch.uint8, device=dev)
        else:
            obs = torch.zeros((B,) + self.observation_shape, device=dev)
            nobs = torch.zeros((B,) + self.observation_shape, device=dev)
        act = (torch.zeros(B, dtype=torch.int32, device=dev) if self.discrete
               else torch.zeros(B, self.action_size, device=dev))
        z = lambda: torch.zeros(B, device=dev)  # noqa: E731
        return DeviceBatch(obs, act, z(), nobs, z(), z())

    def gather(self, out, indices: Optional[torch.Tensor] = None, n_steps: int = 1,
               gamma: float = 0.99, n_frames: int = 1, seed: int = 0,
               idx_out: Optional[torch.Tensor] = None, row_offset: int = 0) -> None:
        """Fill ``out`` (DeviceBatch) with the transitions ``indices`` (device
        int64), or with indices drawn on device (Philox, ``seed``, advancing
        this dataset's sampler counter) when ``indices`` is None; drawn row b
        is draw ``row_offset + b`` of the step (a data-parallel shard of one
        global index stream)."""
        from . import _native as N
        from . import ops
        B = out.batch_size
        d = N.GatherDesc()
        d.obs = ops.ptr(self.obs)
        d.frames = ops.ptr(self.frames)
        d.act = ops.ptr(self.act)
        d.act_i = ops.ptr(self.act_i)
        d.rew = ops.ptr(self.rew)
        d.t_row, d.t_ep_start = ops.ptr(self.t_row), ops.ptr(self.t_ep_start)
        d.t_ep_last, d.t_terminal = ops.ptr(self.t_ep_last), ops.ptr(self.t_terminal)
        d.n_trans = self.n_trans
        d.D = 0 if self.is_image else int(np.prod(self.observation_shape))
        d.A = 0 if self.discrete else self.action_size
        d.frame_bytes = self.frame_bytes
        d.n_frames = n_frames if self.is_image else 1
        d.n_steps = n_steps
        d.set_gamma(gamma, n_steps)
        if indices is not None:
            assert indices.dtype == torch.int64 and indices.is_cuda and indices.numel() >= B
            d.idx = ops.ptr(indices)
        else:
            if idx_out is None:
                idx_out = torch.zeros(B, dtype=torch.int64, device=self.device)
            d.idx_out = ops.ptr(idx_out)
            d.seed = C.c_uint64(seed & 0xFFFFFFFFFFFFFFFF).value
            if self.is_image:
                d.ctr = ops.ptr(self.ctr)
                d.ticket = ops.ptr(self.ticket)
            else:
                # the draw counter by value (this host call is the only
                # consumer): the one-wave-per-row kernel, no device ticket
                d.ctr_value = self._draws
                self._draws += 1
            d.row_offset = row_offset
        d.B = B
        if self.is_image:
            d.o_frames, d.o_next_frames = ops.ptr(out.obs), ops.ptr(out.next_obs)
        else:
            d.o_obs, d.o_next_obs = ops.ptr(out.obs), ops.ptr(out.next_obs)
        if self.discrete:
            d.o_act_i = ops.ptr(out.act)
        else:
            d.o_act = ops.ptr(out.act)
        d.o_rew, d.o_term, d.o_n_steps = ops.ptr(out.rew), ops.ptr(out.term), ops.ptr(out.n_steps)
        ops.call_desc("d3a_gather_batch", d)
