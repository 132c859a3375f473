"""Synthetic, shape-matched stand-ins for the reference's dataset loaders.

The reference's loaders (d3rlpy/datasets.py:16-330) download D4RL / Atari
data; there is no network here, so benchmarks and examples use seeded
synthetic data with the same shapes: obs ~ N(0,1),
actions ~ U(-1,1) (or U{0..A-1}), rewards ~ N(0,1), fixed-length episodes
with the terminal flag on the last step.
"""
from __future__ import annotations

import numpy as np

from .dataset import MDPDataset

D4RL_SHAPES = {
    "hopper-medium-v0": (11, 3),
    "halfcheetah-medium-v0": (17, 6),
    "walker2d-medium-v0": (17, 6),
    "antmaze-umaze-v0": (29, 8),
    "pendulum-random": (3, 1),
}


def synthetic_arrays(n: int, obs_dim: int, act_dim: int, episode_len: int = 1000,
                     seed: int = 0, discrete: bool = False):
    rs = np.random.RandomState(seed)
    obs = rs.randn(n, obs_dim).astype(np.float32)
    if discrete:
        act = rs.randint(act_dim, size=n).astype(np.int32)
    else:
        act = rs.uniform(-1.0, 1.0, size=(n, act_dim)).astype(np.float32)
    rew = rs.randn(n).astype(np.float32)
    term = np.zeros(n, dtype=np.float32)
    term[episode_len - 1::episode_len] = 1.0
    term[-1] = 1.0
    return obs, act, rew, term


def get_synthetic_d4rl(name: str = "hopper-medium-v0", n: int = 1_000_000,
                       episode_len: int = 1000, seed: int = 0) -> MDPDataset:
    obs_dim, act_dim = D4RL_SHAPES[name]
    return MDPDataset(*synthetic_arrays(n, obs_dim, act_dim, episode_len, seed))


def get_synthetic_atari(n_frames_total: int = 100_000, action_size: int = 4,
                        episode_len: int = 2000, seed: int = 0, frame_shape=(1, 84, 84)
                        ) -> MDPDataset:
    """uint8 frames ~ U{0..255}, actions U{0..A-1}, rewards in {-1, 0, 1}."""
    rs = np.random.RandomState(seed)
    obs = rs.randint(0, 256, size=(n_frames_total,) + tuple(frame_shape), dtype=np.uint8)
    act = rs.randint(action_size, size=n_frames_total).astype(np.int32)
    rew = rs.randint(-1, 2, size=n_frames_total).astype(np.float32)
    term = np.zeros(n_frames_total, dtype=np.float32)
    term[episode_len - 1::episode_len] = 1.0
    term[-1] = 1.0
    return MDPDataset(obs, act, rew, term, discrete_action=True)
