"""Restatement of the online replay buffer — TEST INFRASTRUCTURE.

Follows d3rlpy/online/buffers.py and d3rlpy/containers.py:
  FIFOQueue.append / __getitem__   containers.py:35-62 (ring of ``maxlen`` slots;
                                    index = raw slot, not age order; the drop
                                    callback clears an episode's links when its
                                    last transition is overwritten)
  ReplayBuffer.append              buffers.py:235-293 (transition into the
                                    terminal observation has terminal = 1; a
                                    terminal step then adds (s_T -> zeros))
  ReplayBuffer._add_last_step      buffers.py:302-318
  BasicSampleMixin.sample          buffers.py:206-216 (np.random.choice over
                                    len(buffer), then TransitionMiniBatch)
  _Buffer.to_mdp_dataset           buffers.py:115-165
Pure Python objects, for small cases only.  Only tests/ may import this.
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np

from .gather import OTransition, gather


def _clear_back(t: Optional[OTransition]) -> None:
    """trace_back_and_clear (dataset.pyx:1036-1048)."""
    while t is not None:
        p = t.prev
        t.prev = None
        t.next = None
        t = p


class OReplayBuffer:
    def __init__(self, maxlen: int, observation_shape, action_size: int):
        self.maxlen = maxlen
        self.observation_shape = tuple(observation_shape)
        self.action_size = action_size
        self.buf: List[Optional[OTransition]] = [None] * maxlen
        self.cursor = 0
        self.size = 0
        self._prev_obs = None
        self._prev_act = None
        self._prev_rew = 0.0
        self._prev_term = 0.0
        self._prev_t: Optional[OTransition] = None

    def __len__(self) -> int:
        return self.size

    def _push(self, t: OTransition) -> None:
        cur = self.buf[self.cursor]
        if cur is not None and cur.next is None:
            _clear_back(cur)
        self.buf[self.cursor] = t
        self.cursor = (self.cursor + 1) % self.maxlen
        self.size = min(self.size + 1, self.maxlen)

    def append(self, observation, action, reward, terminal, clip_episode=None) -> None:
        if clip_episode is None:
            clip_episode = bool(terminal)
        assert not (terminal and not clip_episode)
        if not isinstance(action, np.ndarray):
            action = int(action)
        if self._prev_obs is not None:
            if isinstance(terminal, bool):
                terminal = 1.0 if terminal else 0.0
            t = OTransition(self._prev_obs, self._prev_act,
                            float(np.float32(self._prev_rew)), observation, float(terminal),
                            prev=self._prev_t)
            if self._prev_t is not None:
                self._prev_t.next = t
            self._push(t)
            self._prev_t = t
        self._prev_obs = observation
        self._prev_act = action
        self._prev_rew = reward
        self._prev_term = terminal
        if clip_episode:
            if terminal:
                t = OTransition(self._prev_obs, self._prev_act,
                                float(np.float32(self._prev_rew)),
                                np.zeros_like(self._prev_obs), 1.0, prev=self._prev_t)
                if self._prev_t is not None:
                    self._prev_t.next = t
                self._push(t)
            self.clip_episode()

    def clip_episode(self) -> None:
        self._prev_obs = None
        self._prev_act = None
        self._prev_rew = 0.0
        self._prev_term = 0.0
        self._prev_t = None

    def sample_indices(self, batch_size: int) -> np.ndarray:
        return np.random.choice(self.size, batch_size)

    def gather(self, indices, n_frames: int = 1, n_steps: int = 1, gamma: float = 0.99):
        return gather([self.buf[int(i)] for i in indices], n_frames, n_steps, gamma)

    def to_mdp_arrays(self):
        """buffers.py:115-165 -> (observations, actions, rewards, terminals,
        episode_terminals) numpy arrays."""
        tails = [t for t in self.buf[:self.size] if t.next is None]
        obs, act, rew, term, ep = [], [], [], [], []
        for tail in tails:
            chain = []
            t = tail
            while True:
                chain.append(t)
                if t.prev is None:
                    break
                t = t.prev
            chain.reverse()
            for i, t in enumerate(chain):
                obs.append(t.observation)
                act.append(t.action)
                rew.append(t.reward)
                term.append(t.terminal)
                ep.append(i == len(chain) - 1)
        return (np.asarray(obs, dtype=np.float32), np.asarray(act), np.asarray(rew),
                np.asarray(term), np.asarray(ep))
