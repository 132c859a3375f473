"""Online training: HBM-resident replay buffer, explorers and the single-env
loop behind ``fit_online``.

Reference: d3rlpy/online/buffers.py (ReplayBuffer, FIFOQueue in containers.py),
online/explorers.py, online/iterators.py:99-278 (train_single_env).

Replay layout (host mirror + HBM copy, structure of arrays over ring slots):
transition in slot ``s`` owns two step rows, ``2s`` (its observation, action,
reward) and ``2s+1`` (its next observation, zeros after a terminal step).  The
transition table handed to the gather kernel (``d3a_gather_batch``) is then
``t_row[s] = 2s``, ``t_ep_start[s] = 2s``, ``t_terminal[s] = 0`` (the zero
next observation is stored), ``t_term_value[s]`` = the transition's terminal
flag, and ``t_ep_last[s] = s`` iff the transition has no successor in the next
slot (``(s+1) % maxlen``), so the kernel's n-step walk (successor slot until
``nt_i == t_ep_last``)
follows the reference's ``next_transition`` links and reads the next
observation at ``2(s+k)+1``.  Appends land in the host mirror; ``sample``
uploads only the slots written since the previous sample, then gathers on
device.  Sampling draws ``np.random.choice(len(buffer), batch_size)`` from
numpy's global RNG over raw slot indices, the reference's stream
(buffers.py:213).

Differences from the reference, by construction:
* ``n_frames > 1`` (frame stacking across the ring) is not supported:
  ``sample`` raises ``NotImplementedError``.
* ``to_mdp_dataset`` traces episodes through stored transitions only; the
  reference may also reach transitions already overwritten in the ring but
  still linked from a stored successor (buffers.py:115-121).
"""
from __future__ import annotations

import time
from collections import defaultdict
from typing import Callable, Dict, List, Optional

import numpy as np
import torch

from .dataset import Episode, MDPDataset


def get_action_size_from_env(env) -> int:
    """online/utility.py:7-10 (Discrete -> n, Box -> shape[0])."""
    space = env.action_space
    if hasattr(space, "n"):
        return int(space.n)
    return int(space.shape[0])


def _is_discrete_env(env) -> bool:
    return hasattr(env.action_space, "n")


class ReplayBuffer:
    """buffers.py:219-318 — standard FIFO replay buffer, HBM-resident."""

    def __init__(self, maxlen: int, env=None, episodes: Optional[List[Episode]] = None,
                 device=None):
        if env is not None:
            obs_shape = tuple(env.observation_space.shape)
            action_size = get_action_size_from_env(env)
            discrete = _is_discrete_env(env)
        elif episodes:
            obs_shape = tuple(episodes[0].get_observation_shape())
            action_size = episodes[0].get_action_size()
            discrete = episodes[0].actions.ndim == 1
        else:
            raise ValueError("env or episodes are required to determine shape.")
        assert maxlen >= 1
        self._maxlen = maxlen
        self._observation_shape = obs_shape
        self._action_size = action_size
        self._discrete = discrete
        self._is_image = len(obs_shape) == 3
        width = int(np.prod(obs_shape))
        self._width = width
        R = 2 * maxlen
        # host mirror
        self._h_obs = np.zeros((R, width), np.uint8 if self._is_image else np.float32)
        self._h_act = (np.zeros(R, np.int32) if discrete
                       else np.zeros((R, action_size), np.float32))
        self._h_rew = np.zeros(R, np.float32)
        self._h_last = np.arange(maxlen, dtype=np.int64)
        self._h_term = np.zeros(maxlen, np.float32)
        # links by global transition id (slot = id % maxlen); -1 = none
        self._prev_id = np.full(maxlen, -1, np.int64)
        self._next_id = np.full(maxlen, -1, np.int64)
        self._n_total = 0
        self._size = 0
        self._dirty: set = set()
        self._device = None
        self._req_device = device
        self._prev_observation = None
        self._prev_action = None
        self._prev_reward = 0.0
        self._prev_terminal = 0.0
        self._prev_tid = -1
        if episodes:
            for ep in episodes:
                self.append_episode(ep)

    # ------------------------------------------------------------ host side
    def _live(self, tid: int) -> bool:
        return tid >= 0 and tid >= self._n_total - self._size

    def _push(self, obs, act, rew, next_obs, terminal: float, prev_tid: int) -> int:
        tid = self._n_total
        s = tid % self._maxlen
        if self._size == self._maxlen:
            # the overwritten transition's successor loses its predecessor link
            # (the reference keeps the dropped object reachable; see module doc)
            nxt = int(self._next_id[s])
            if self._live(nxt):
                self._prev_id[nxt % self._maxlen] = -1
        self._h_obs[2 * s] = np.asarray(obs).reshape(-1)
        self._h_obs[2 * s + 1] = np.asarray(next_obs).reshape(-1)
        self._h_act[2 * s] = act
        self._h_rew[2 * s] = np.float32(rew)
        self._h_term[s] = terminal
        self._h_last[s] = s
        self._prev_id[s] = prev_tid
        self._next_id[s] = -1
        self._dirty.add(s)
        # liveness in the post-push window [tid - maxlen + 1, tid]: with
        # maxlen 1 the predecessor was just overwritten by this transition
        if prev_tid >= 0 and prev_tid > tid - self._maxlen:
            ps = prev_tid % self._maxlen
            self._next_id[ps] = tid
            # the kernel's n-step walk steps to slot (ps + 1) % maxlen
            self._h_last[ps] = s if s == (ps + 1) % self._maxlen else ps
            self._dirty.add(ps)
        self._n_total += 1
        self._size = min(self._size + 1, self._maxlen)
        return tid

    def append(self, observation, action, reward, terminal, clip_episode=None) -> None:
        """buffers.py:235-293."""
        if clip_episode is None:
            clip_episode = bool(terminal)
        assert tuple(np.asarray(observation).shape) == self._observation_shape
        if isinstance(action, np.ndarray) and action.ndim >= 1:
            assert action.shape[0] == self._action_size
        else:
            action = int(action)
            assert action < self._action_size
        assert not (terminal and not clip_episode)
        if self._prev_observation is not None:
            if isinstance(terminal, bool):
                terminal = 1.0 if terminal else 0.0
            self._prev_tid = self._push(self._prev_observation, self._prev_action,
                                        self._prev_reward, observation, float(terminal),
                                        self._prev_tid)
        self._prev_observation = np.asarray(observation)
        self._prev_action = action
        self._prev_reward = reward
        self._prev_terminal = terminal
        if clip_episode:
            if terminal:
                self._add_last_step()
            self.clip_episode()

    def _add_last_step(self) -> None:
        """buffers.py:302-318: (s_T, a_T, r_T) -> zeros, terminal 1."""
        assert self._prev_terminal
        assert self._prev_observation is not None
        self._push(self._prev_observation, self._prev_action, self._prev_reward,
                   np.zeros_like(self._prev_observation), 1.0, self._prev_tid)

    def clip_episode(self) -> None:
        self._prev_observation = None
        self._prev_action = None
        self._prev_reward = 0.0
        self._prev_terminal = 0.0
        self._prev_tid = -1

    def append_episode(self, episode: Episode) -> None:
        """buffers.py:56-66: every transition of ``episode``, linked."""
        assert tuple(episode.get_observation_shape()) == self._observation_shape
        assert episode.get_action_size() == self._action_size
        prev = -1
        for t in episode.transitions:
            prev = self._push(t.observation, t.action, t.reward, t.next_observation,
                              float(t.terminal), prev)

    def size(self) -> int:
        return self._size

    def __len__(self) -> int:
        return self._size

    @property
    def maxlen(self) -> int:
        return self._maxlen

    def to_mdp_dataset(self) -> MDPDataset:
        """buffers.py:115-165: episodes traced back from every stored tail."""
        obs, act, rew, term, ep = [], [], [], [], []
        for s in range(self._size):
            if self._next_id[s] >= 0 and self._live(int(self._next_id[s])):
                continue
            chain = [s]
            while True:
                p = int(self._prev_id[chain[-1]])
                if not self._live(p):
                    break
                chain.append(p % self._maxlen)
            chain.reverse()
            for i, c in enumerate(chain):
                obs.append(self._h_obs[2 * c])
                act.append(self._h_act[2 * c])
                rew.append(self._h_rew[2 * c])
                term.append(self._h_term[c])
                ep.append(i == len(chain) - 1)
        observations = np.asarray(obs).reshape((-1,) + self._observation_shape)
        if self._is_image:
            observations = observations.astype(np.uint8)
        else:
            observations = observations.astype(np.float32)
        return MDPDataset(observations, np.asarray(act), np.asarray(rew, np.float32),
                          np.asarray(term, np.float32),
                          episode_terminals=np.asarray(ep, np.float32),
                          discrete_action=self._discrete)

    # ---------------------------------------------------------- device side
    def _ensure_device(self) -> None:
        if self._device is not None:
            return
        from . import _native  # noqa: F401  (fail loudly if the library is missing)
        if not torch.cuda.is_available():
            raise RuntimeError("ReplayBuffer.sample needs a HIP device (no CPU fallback)")
        dev = torch.device(self._req_device if self._req_device is not None
                           else torch.cuda.current_device())
        self._device = dev
        M = self._maxlen
        up = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        # step rows start as zeros on the device; every slot written so far is
        # still in the dirty set, so the first _sync uploads exactly those (a
        # 1M-slot pixel ring never copies, or faults in, its unused host pages)
        zeros = lambda a: torch.zeros(a.shape, dtype=torch.from_numpy(a[:1]).dtype,  # noqa: E731
                                      device=dev)
        self._d_obs = zeros(self._h_obs)
        self._d_act = zeros(self._h_act)
        self._d_rew = zeros(self._h_rew)
        self._d_last = up(self._h_last)
        self._d_term = zeros(self._h_term)
        self._d_row = torch.arange(0, 2 * M, 2, dtype=torch.int64, device=dev)
        self._d_ep_start = self._d_row
        self._d_terminal = torch.zeros(M, dtype=torch.uint8, device=dev)

    def _sync(self) -> None:
        """Upload the slots written since the last sample (one copy per field)."""
        if not self._dirty:
            return
        slots = np.fromiter(self._dirty, dtype=np.int64, count=len(self._dirty))
        self._dirty.clear()
        rows = np.concatenate([2 * slots, 2 * slots + 1])
        dev = self._device
        ds = torch.from_numpy(slots).to(dev, non_blocking=False)
        dr = torch.from_numpy(rows).to(dev, non_blocking=False)
        self._d_obs.index_copy_(0, dr, torch.from_numpy(self._h_obs[rows]).to(dev))
        self._d_act.index_copy_(0, dr, torch.from_numpy(self._h_act[rows]).to(dev))
        self._d_rew.index_copy_(0, dr, torch.from_numpy(self._h_rew[rows]).to(dev))
        self._d_last.index_copy_(0, ds, torch.from_numpy(self._h_last[slots]).to(dev))
        self._d_term.index_copy_(0, ds, torch.from_numpy(self._h_term[slots]).to(dev))

    def alloc_batch(self, batch_size: int):
        from .algos.impl_base import DeviceBatch
        self._ensure_device()
        dev, B = self._device, batch_size
        dt = torch.uint8 if self._is_image else torch.float32
        obs = torch.zeros((B,) + self._observation_shape, dtype=dt, device=dev)
        nobs = torch.zeros((B,) + self._observation_shape, dtype=dt, device=dev)
        act = (torch.zeros(B, dtype=torch.int32, device=dev) if self._discrete
               else torch.zeros(B, self._action_size, device=dev))
        z = lambda: torch.zeros(B, device=dev)  # noqa: E731
        return DeviceBatch(obs, act, z(), nobs, z(), z())

    def sample(self, batch_size: int, n_frames: int = 1, n_steps: int = 1,
               gamma: float = 0.99, out=None, indices: Optional[np.ndarray] = None):
        """buffers.py:206-216: ``np.random.choice(len(self), batch_size)`` raw
        slots, gathered on device into a DeviceBatch (``out`` if given)."""
        if n_frames > 1:
            raise NotImplementedError("frame stacking is not supported by the device "
                                      "replay buffer")
        assert self._size > 0, "buffer is empty"
        if indices is None:
            indices = np.random.choice(self._size, batch_size)
        indices = np.asarray(indices, dtype=np.int64)
        assert indices.shape == (batch_size,) and indices.min() >= 0 \
            and indices.max() < self._size
        self._ensure_device()
        self._sync()
        if out is None:
            out = self.alloc_batch(batch_size)
        assert out.batch_size == batch_size
        from . import _native as N
        from . import ops
        idx = torch.from_numpy(indices).to(self._device)
        d = N.GatherDesc()
        if self._is_image:
            d.frames = ops.ptr(self._d_obs)
            d.frame_bytes = self._width
        else:
            d.obs = ops.ptr(self._d_obs)
            d.D = self._width
        if self._discrete:
            d.act_i = ops.ptr(self._d_act)
        else:
            d.act = ops.ptr(self._d_act)
            d.A = self._action_size
        d.rew = ops.ptr(self._d_rew)
        d.t_row, d.t_ep_start = ops.ptr(self._d_row), ops.ptr(self._d_ep_start)
        d.t_ep_last, d.t_terminal = ops.ptr(self._d_last), ops.ptr(self._d_terminal)
        d.t_term_value = ops.ptr(self._d_term)
        d.n_trans = self._maxlen
        d.n_frames = 1
        d.n_steps = n_steps
        d.set_gamma(gamma, n_steps)
        d.idx = ops.ptr(idx)
        d.B = batch_size
        if self._is_image:
            d.o_frames, d.o_next_frames = ops.ptr(out.obs), ops.ptr(out.next_obs)
        else:
            d.o_obs, d.o_next_obs = ops.ptr(out.obs), ops.ptr(out.next_obs)
        if self._discrete:
            d.o_act_i = ops.ptr(out.act)
        else:
            d.o_act = ops.ptr(out.act)
        d.o_rew, d.o_term, d.o_n_steps = ops.ptr(out.rew), ops.ptr(out.term), \
            ops.ptr(out.n_steps)
        ops.call_desc("d3a_gather_batch", d)
        return out


# ------------------------------------------------------------------ explorers
class Explorer:
    def sample(self, algo, x: np.ndarray, step: int) -> np.ndarray:
        raise NotImplementedError


class ConstantEpsilonGreedy(Explorer):
    """explorers.py:34-53."""

    def __init__(self, epsilon: float):
        self._epsilon = epsilon

    def sample(self, algo, x, step):
        greedy_actions = algo.predict(x)
        random_actions = np.random.randint(algo.action_size, size=x.shape[0])
        is_random = np.random.random(x.shape[0]) < self._epsilon
        return np.where(is_random, random_actions, greedy_actions)


class LinearDecayEpsilonGreedy(Explorer):
    """explorers.py:56-109."""

    def __init__(self, start_epsilon: float = 1.0, end_epsilon: float = 0.1,
                 duration: int = 1000000):
        self._start_epsilon = start_epsilon
        self._end_epsilon = end_epsilon
        self._duration = duration

    def sample(self, algo, x, step):
        greedy_actions = algo.predict(x)
        random_actions = np.random.randint(algo.action_size, size=x.shape[0])
        is_random = np.random.random(x.shape[0]) < self.compute_epsilon(step)
        return np.where(is_random, random_actions, greedy_actions)

    def compute_epsilon(self, step: int) -> float:
        if step >= self._duration:
            return self._end_epsilon
        base = self._start_epsilon - self._end_epsilon
        return base * (1.0 - step / self._duration) + self._end_epsilon


class NormalNoise(Explorer):
    """explorers.py:112-155 (one scalar noise draw per call, as the reference)."""

    def __init__(self, mean: float = 0.0, std: float = 0.1):
        self._mean = mean
        self._std = std

    def sample(self, algo, x, step):
        action = algo.predict(x)
        noise = np.random.normal(self._mean, self._std)
        return np.clip(action + noise, -1.0, 1.0)


# --------------------------------------------------------------- evaluation
def evaluate_on_environment(env, n_trials: int = 10, epsilon: float = 0.0
                            ) -> Callable[..., float]:
    """metrics/scorer.py evaluate_on_environment: mean undiscounted return of
    ``n_trials`` greedy (epsilon-greedy) episodes, vector observations."""
    def scorer(algo, *args) -> float:
        returns = []
        for _ in range(n_trials):
            observation = env.reset()
            episode_reward = 0.0
            while True:
                if np.random.random() < epsilon:
                    action = env.action_space.sample()
                else:
                    action = algo.predict([observation])[0]
                observation, reward, done, _ = env.step(action)
                episode_reward += reward
                if done:
                    break
            returns.append(episode_reward)
        return float(np.mean(returns))
    return scorer


# -------------------------------------------------------------- online loop
def _setup_algo(algo, env) -> None:
    """iterators.py:76-96."""
    scaler = algo.scaler
    if scaler is not None:
        fit = getattr(scaler, "fit_with_env", None)
        if fit is not None:
            fit(env)
        elif getattr(scaler, "get_type", lambda: "")() == "standard" \
                and getattr(scaler, "_mean", None) is None:
            # StandardScaler.fit_with_env (preprocessing/scalers.py) raises
            # unless mean/std were given
            raise NotImplementedError("standard scaler does not support fit_with_env.")
    if algo.impl is None:
        algo.create_impl(algo._process_observation_shape(env.observation_space.shape),
                         get_action_size_from_env(env))


def train_single_env(algo, env, buffer: ReplayBuffer, explorer: Optional[Explorer] = None,
                     n_steps: int = 1000000, n_steps_per_epoch: int = 10000,
                     update_interval: int = 1, update_start_step: int = 0,
                     random_steps: int = 0, eval_env=None, eval_epsilon: float = 0.0,
                     save_metrics: bool = True, save_interval: int = 1,
                     experiment_name: Optional[str] = None, with_timestamp: bool = True,
                     logdir: str = "d3rlpy_logs", verbose: bool = True,
                     show_progress: bool = True, tensorboard_dir=None,
                     timelimit_aware: bool = True, callback=None
                     ) -> List[Dict[str, float]]:
    """iterators.py:99-278: act, step the env, append, then one gradient step
    on a device-gathered minibatch every ``update_interval`` env steps.
    Returns the per-epoch metric means (the reference writes them to its
    logger only)."""
    from .logger import OfflineLogger
    if algo.n_frames > 1:
        raise NotImplementedError("online training with frame stacking is not supported")
    name = experiment_name or algo.__class__.__name__ + "_online"
    logger = OfflineLogger(name, save_metrics=save_metrics, root_dir=logdir,
                           verbose=verbose, with_timestamp=with_timestamp)
    _setup_algo(algo, env)
    if save_metrics:
        algo.save_params(logger.logdir)
    eval_scorer = evaluate_on_environment(eval_env, epsilon=eval_epsilon) if eval_env \
        else None
    out = algo.impl.staging_batch(algo.batch_size) \
        if hasattr(algo.impl, "staging_batch") else None
    metrics: Dict[str, List[float]] = defaultdict(list)
    history: List[Dict[str, float]] = []
    observation = env.reset()
    rollout_return = 0.0
    t0 = time.perf_counter()
    for total_step in range(1, n_steps + 1):
        observation = np.asarray(observation)
        if observation.dtype != np.uint8:
            observation = observation.astype("f4")
        if total_step < random_steps:
            action = env.action_space.sample()
        elif explorer:
            action = explorer.sample(algo, observation.reshape((1,) + observation.shape),
                                     total_step)[0]
        else:
            action = algo.sample_action([observation])[0]
        next_observation, reward, terminal, info = env.step(action)
        rollout_return += reward
        if timelimit_aware and "TimeLimit.truncated" in info:
            clip_episode = True
            terminal = False
        else:
            clip_episode = terminal
        buffer.append(observation=observation, action=action, reward=reward,
                      terminal=terminal, clip_episode=clip_episode)
        if clip_episode:
            observation = env.reset()
            metrics["rollout_return"].append(rollout_return)
            rollout_return = 0.0
        else:
            observation = next_observation
        epoch = total_step // n_steps_per_epoch
        if total_step > update_start_step and len(buffer) > algo.batch_size:
            if total_step % update_interval == 0:
                batch = buffer.sample(batch_size=algo.batch_size, n_frames=algo.n_frames,
                                      n_steps=algo.n_steps, gamma=algo.gamma, out=out)
                loss = algo.update(batch)
                for k, v in loss.items():
                    metrics[k].append(v)
        if callback:
            callback(algo, epoch, total_step)
        if epoch > 0 and total_step % n_steps_per_epoch == 0:
            if eval_scorer:
                metrics["evaluation"].append(eval_scorer(algo))
            if save_metrics and epoch % save_interval == 0:
                logger.save_model(total_step, algo)
            summary = {k: float(np.mean(v)) for k, v in metrics.items()}
            elapsed = time.perf_counter() - t0
            logger.add_epoch(epoch, total_step, summary,
                             {"time_step": elapsed / n_steps_per_epoch})
            history.append(summary)
            metrics = defaultdict(list)
            t0 = time.perf_counter()
    buffer.clip_episode()
    logger.close()
    return history


def collect(algo, env, buffer: ReplayBuffer, explorer: Optional[Explorer] = None,
            deterministic: bool = False, n_steps: int = 1000000,
            show_progress: bool = True, timelimit_aware: bool = True) -> None:
    """iterators.py:288-380: fill ``buffer`` by acting in ``env`` (greedy when
    ``deterministic``, else the explorer or the policy's sample), no updates."""
    if algo.n_frames > 1:
        raise NotImplementedError("online collection with frame stacking is not supported")
    _setup_algo(algo, env)
    observation = env.reset()
    for total_step in range(1, n_steps + 1):
        observation = np.asarray(observation)
        if observation.dtype != np.uint8:
            observation = observation.astype("f4")
        if deterministic:
            action = algo.predict([observation])[0]
        elif explorer:
            action = explorer.sample(algo, observation.reshape((1,) + observation.shape),
                                     total_step)[0]
        else:
            action = algo.sample_action([observation])[0]
        next_observation, reward, terminal, info = env.step(action)
        if timelimit_aware and "TimeLimit.truncated" in info:
            clip_episode = True
            terminal = False
        else:
            clip_episode = terminal
        buffer.append(observation=observation, action=action, reward=reward,
                      terminal=terminal, clip_episode=clip_episode)
        observation = env.reset() if clip_episode else next_observation
    buffer.clip_episode()
