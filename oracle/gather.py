"""Restatement of the minibatch gather and the index stream — TEST INFRASTRUCTURE.

Follows d3rlpy/dataset.pyx:
  _to_episodes            :44-67    (episode split on episode_terminals)
  _to_transitions         :70-116   (links; terminal episodes get a zero dummy
                                     next observation, non-terminal ones drop
                                     their last step)
  TransitionMiniBatch     :1139-1217
  _assign_to_batch        :1286-1342 (n-step return, t+n observation, terminal)
  _stack_frames           :1053-1096 (frame stacking, zero next-stack at terminals)
and RandomIterator._next (iterators/random_iterator.py:38-41): one
``np.random.randint(len(transitions))`` per sample from numpy's global RNG.

Pure Python loops over transition *objects* exactly like the reference's
pointer walk; for small cases only (the test KATs).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import numpy as np


@dataclass
class OTransition:
    observation: np.ndarray
    action: object
    reward: float
    next_observation: np.ndarray
    terminal: float
    prev: Optional["OTransition"] = None
    next: Optional["OTransition"] = None


def to_episodes(observations, actions, rewards, terminals, episode_terminals=None):
    """dataset.pyx:44-67 -> list of (obs, act, rew, terminal)."""
    terminals = np.asarray(terminals, dtype=np.float32).reshape(-1)
    ep_t = terminals if episode_terminals is None else \
        np.asarray(episode_terminals, dtype=np.float32).reshape(-1)
    rets, head = [], 0
    for i in range(len(observations)):
        if ep_t[i]:
            rets.append((observations[head:i + 1], actions[head:i + 1], rewards[head:i + 1],
                         float(terminals[i])))
            head = i + 1
    return rets


def to_transitions(observations, actions, rewards, terminal) -> List[OTransition]:
    """dataset.pyx:70-116."""
    rets: List[OTransition] = []
    n = len(observations)
    prev = None
    for i in range(n):
        if i == n - 1:
            if terminal:
                next_observation = np.zeros_like(observations[i])
            else:
                break
        else:
            next_observation = observations[i + 1]
        env_terminal = terminal if i == n - 1 else 0.0
        t = OTransition(observations[i], actions[i], float(np.float32(np.asarray(rewards[i]).reshape(-1)[0])),
                        next_observation, float(env_terminal), prev=prev)
        if prev is not None:
            prev.next = t
        prev = t
        rets.append(t)
    return rets


def _stack_frames(t: OTransition, n_frames: int, stack_next: bool) -> np.ndarray:
    """dataset.pyx:1053-1096."""
    obs = t.observation
    c, h, w = obs.shape
    stack = np.zeros((n_frames * c, h, w), dtype=np.uint8)
    if stack_next and t.terminal:
        return stack
    cur = t
    for i in range(n_frames):
        tail = n_frames * c - i * c
        head = tail - c
        src = cur.next_observation if stack_next else cur.observation
        stack[head:tail] = src
        if cur.prev is None:
            for j in range(n_frames - i - 1):
                tail = n_frames * c - (i + j + 1) * c
                head = tail - c
                stack[head:tail] = cur.observation
            break
        cur = cur.prev
    return stack


_LIBM = None


def _powf_table(g32: np.float32, n: int):
    """powf(gamma, (float)i) for i < n from the C library (ctypes)."""
    global _LIBM
    if _LIBM is None:
        import ctypes
        import ctypes.util
        _LIBM = ctypes.CDLL(ctypes.util.find_library("m"))
        _LIBM.powf.restype = ctypes.c_float
        _LIBM.powf.argtypes = [ctypes.c_float, ctypes.c_float]
    return [np.float32(_LIBM.powf(float(g32), float(i))) for i in range(n)]


def gather(transitions: List[OTransition], n_frames: int = 1, n_steps: int = 1,
           gamma: float = 0.99):
    """TransitionMiniBatch(transitions, n_frames, n_steps, gamma) -> dict of arrays."""
    size = len(transitions)
    first = transitions[0]
    is_image = first.observation.ndim == 3
    discrete = not isinstance(first.action, np.ndarray)
    obs, nobs, acts, rews, terms, nst = [], [], [], [], [], []
    g32 = np.float32(gamma)
    gpow = _powf_table(g32, n_steps)
    for t in transitions:
        ret = np.float32(0.0)
        nxt = t
        i = 0
        for i in range(n_steps):
            # n_step_return += reward * gamma ** i   (dataset.pyx:1325, float gamma,
            # int i): Cython 0.29.21 (requirements.txt:8) emits
            # `acc = acc + reward * powf(gamma, (float)i)` — fp32 throughout,
            # powf from the C library (tests/golden/cython_pow_codegen.txt)
            gp = gpow[i]
            ret = np.float32(ret + np.float32(np.float32(nxt.reward) * gp))
            if nxt.next is None or i == n_steps - 1:
                break
            nxt = nxt.next
        if is_image and n_frames > 1:
            obs.append(_stack_frames(t, n_frames, False))
            nobs.append(_stack_frames(nxt, n_frames, True))
        else:
            obs.append(np.asarray(t.observation))
            nobs.append(np.asarray(nxt.next_observation))
        acts.append(t.action)
        rews.append(ret)
        terms.append(nxt.terminal)
        nst.append(i + 1)
    out = {
        "observations": np.stack(obs),
        "next_observations": np.stack(nobs),
        "actions": (np.asarray(acts, dtype=np.int32) if discrete
                    else np.stack(acts).astype(np.float32)),
        "rewards": np.asarray(rews, dtype=np.float32).reshape(size, 1),
        "terminals": np.asarray(terms, dtype=np.float32).reshape(size, 1),
        "n_steps": np.asarray(nst, dtype=np.float32).reshape(size, 1),
    }
    return out


def random_indices(n_transitions: int, batch_size: int) -> np.ndarray:
    """RandomIterator._next x batch_size (one global-RNG randint per sample)."""
    return np.array([np.random.randint(n_transitions) for _ in range(batch_size)],
                    dtype=np.int64)


def synthetic_dataset(n_steps_total: int, obs_dim: int, act_dim: int, episode_len: int = 1000,
                      seed: int = 0, discrete: bool = False):
    """D4RL-shaped synthetic data: RandomState(seed); obs ~ N(0,1),
    actions ~ U(-1,1) (or U{0..act_dim-1}), rewards ~ N(0,1), terminal on the
    last step of every episode_len-step episode."""
    rs = np.random.RandomState(seed)
    obs = rs.randn(n_steps_total, obs_dim).astype(np.float32)
    if discrete:
        act = rs.randint(act_dim, size=n_steps_total).astype(np.int32)
    else:
        act = rs.uniform(-1.0, 1.0, size=(n_steps_total, act_dim)).astype(np.float32)
    rew = rs.randn(n_steps_total).astype(np.float32)
    term = np.zeros(n_steps_total, dtype=np.float32)
    term[episode_len - 1::episode_len] = 1.0
    term[-1] = 1.0
    return obs, act, rew, term
