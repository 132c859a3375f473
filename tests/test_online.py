"""Online replay buffer (online/buffers.py) and fit_online (online/iterators.py).

CPU: the HBM replay buffer's host mirror (slots, links, n-step chain table,
to_mdp_dataset) against the restated reference buffer (oracle/online.py) on
the same append sequence, with and without ring eviction.
GPU: ``ReplayBuffer.sample`` through the gather kernel, bit-exact against the
oracle's TransitionMiniBatch on the same slots (n_steps 1 and 3, vector and
pixel observations, the reference's np.random.choice stream), and
``fit_online`` end to end on toy gym-style environments.
"""
import numpy as np
import pytest
import torch

from oracle.online import OReplayBuffer
from d3rlpy_amd.online import (ConstantEpsilonGreedy, LinearDecayEpsilonGreedy, NormalNoise,
                               ReplayBuffer)


class _Box:
    def __init__(self, shape, low=-1.0, high=1.0, dtype=np.float32):
        self.shape, self.low, self.high, self.dtype = tuple(shape), low, high, dtype

    def sample(self):
        return np.random.uniform(self.low, self.high, self.shape).astype(np.float32)


class _Discrete:
    def __init__(self, n):
        self.n = n

    def sample(self):
        return int(np.random.randint(self.n))


class ToyEnv:
    """Gym-style (old API) environment: random observations, episodes of
    random length; some end terminal, some by TimeLimit truncation."""

    def __init__(self, obs_shape=(5,), action_size=2, discrete=False, seed=0, max_len=40):
        self.observation_space = _Box(obs_shape)
        self.action_space = _Discrete(action_size) if discrete else _Box((action_size,))
        self._rng = np.random.RandomState(seed)
        self._image = len(obs_shape) == 3
        self._max_len = max_len
        self._t = 0

    def _obs(self):
        if self._image:
            return self._rng.randint(0, 256, self.observation_space.shape).astype(np.uint8)
        return self._rng.randn(*self.observation_space.shape).astype(np.float32)

    def reset(self):
        self._t = 0
        self._len = int(self._rng.randint(3, self._max_len))
        return self._obs()

    def step(self, action):
        self._t += 1
        reward = float(self._rng.randn())
        done = self._t >= self._len
        info = {}
        if done and self._rng.rand() < 0.3:
            info["TimeLimit.truncated"] = True
        return self._obs(), reward, done, info


def _fill(buffers, n_steps, obs_shape=(5,), action_size=2, discrete=False, seed=0):
    """Drive the same append sequence (as train_single_env does) into every buffer."""
    env = ToyEnv(obs_shape, action_size, discrete, seed)
    rng = np.random.RandomState(seed + 1)
    obs = env.reset()
    for _ in range(n_steps):
        a = int(rng.randint(action_size)) if discrete else \
            rng.uniform(-1, 1, action_size).astype(np.float32)
        nobs, r, done, info = env.step(a)
        if "TimeLimit.truncated" in info:
            clip, done = True, False
        else:
            clip = done
        for b in buffers:
            b.append(observation=obs, action=a, reward=r, terminal=done, clip_episode=clip)
        obs = env.reset() if clip else nobs


def _check_host(buf: ReplayBuffer, ob: OReplayBuffer):
    assert len(buf) == len(ob)
    for s in range(len(ob)):
        t = ob.buf[s]
        np.testing.assert_array_equal(buf._h_obs[2 * s], np.asarray(t.observation).reshape(-1))
        np.testing.assert_array_equal(buf._h_obs[2 * s + 1],
                                      np.asarray(t.next_observation).reshape(-1))
        np.testing.assert_array_equal(buf._h_act[2 * s], t.action)
        assert buf._h_rew[2 * s] == np.float32(t.reward)
        assert buf._h_term[s] == np.float32(t.terminal)
        # kernel chain table: slot s continues into slot s+1 iff the reference's
        # next_transition is the transition stored there
        cont = t.next is not None and ob.buf[(s + 1) % ob.maxlen] is t.next
        assert (buf._h_last[s] != s) == cont, s


@pytest.mark.parametrize("maxlen,n", [(5000, 700), (97, 700), (2, 50), (1, 50)])
def test_replay_host_mirror_matches_reference_buffer(maxlen, n):
    buf = ReplayBuffer(maxlen, env=ToyEnv())
    ob = OReplayBuffer(maxlen, (5,), 2)
    _fill([buf, ob], n)
    _check_host(buf, ob)


def test_replay_maxlen1_keeps_the_stored_transition():
    """maxlen 1: the newest transition must not link to itself (it replaced
    its predecessor); to_mdp_dataset traces stored transitions only (the
    reference also walks evicted objects it keeps reachable, module doc)."""
    buf = ReplayBuffer(1, env=ToyEnv())
    ob = OReplayBuffer(1, (5,), 2)
    _fill([buf, ob], 500)
    assert buf._h_last[0] == 0 and buf._next_id[0] == -1
    ds = buf.to_mdp_dataset()
    assert len(ds.observations) == 1
    np.testing.assert_array_equal(ds.observations[0], np.asarray(ob.buf[0].observation))


def test_replay_to_mdp_dataset_matches_reference():
    buf = ReplayBuffer(5000, env=ToyEnv())
    ob = OReplayBuffer(5000, (5,), 2)
    _fill([buf, ob], 500)
    ds = buf.to_mdp_dataset()
    o, a, r, t, e = ob.to_mdp_arrays()
    np.testing.assert_array_equal(ds.observations, o)
    np.testing.assert_array_equal(ds.actions, np.asarray(a, np.float32))
    np.testing.assert_array_equal(ds.rewards.reshape(-1), np.asarray(r, np.float32))
    np.testing.assert_array_equal(ds.terminals.reshape(-1), np.asarray(t, np.float32))
    np.testing.assert_array_equal(np.asarray(ds.episode_terminals).reshape(-1) > 0, e)


def test_replay_append_episode_and_validation():
    from d3rlpy_amd.dataset import MDPDataset
    obs = np.random.RandomState(0).randn(20, 5).astype(np.float32)
    act = np.random.RandomState(1).uniform(-1, 1, (20, 2)).astype(np.float32)
    rew = np.arange(20, dtype=np.float32)
    term = np.zeros(20, np.float32)
    term[9] = term[19] = 1.0
    ds = MDPDataset(obs, act, rew, term)
    buf = ReplayBuffer(100, episodes=ds.episodes)
    # terminal episodes keep every step (the last with a zero next observation)
    assert len(buf) == 20
    assert buf._h_term[9] == 1.0 and buf._h_last[9] == 9 and buf._h_last[8] == 9
    np.testing.assert_array_equal(buf._h_obs[2 * 9 + 1], np.zeros(5, np.float32))
    with pytest.raises(AssertionError):
        buf.append(np.zeros(4, np.float32), act[0], 0.0, False)
    with pytest.raises(ValueError):
        ReplayBuffer(10)


def test_explorers_follow_the_reference_formulas():
    class _Algo:
        action_size = 4

        def predict(self, x):
            return np.full(x.shape[0], 3)
    e = LinearDecayEpsilonGreedy(1.0, 0.1, 100)
    assert e.compute_epsilon(0) == 1.0 and e.compute_epsilon(100) == 0.1
    assert abs(e.compute_epsilon(50) - 0.55) < 1e-12
    np.random.seed(0)
    greedy = ConstantEpsilonGreedy(0.0).sample(_Algo(), np.zeros((8, 2)), 0)
    assert (greedy == 3).all()

    class _CAlgo:
        def predict(self, x):
            return np.full((x.shape[0], 2), 0.95, np.float32)
    np.random.seed(1)
    a = NormalNoise(0.0, 0.1).sample(_CAlgo(), np.zeros((3, 2)), 0)
    np.random.seed(1)
    n = np.random.normal(0.0, 0.1)
    np.testing.assert_array_equal(a, np.clip(0.95 + n, -1.0, 1.0))


# ------------------------------------------------------------------- GPU
def _compare(batch, ref, image=False):
    B = batch.batch_size
    np.testing.assert_array_equal(batch.obs.cpu().numpy().reshape(B, -1),
                                  ref["observations"].reshape(B, -1))
    np.testing.assert_array_equal(batch.next_obs.cpu().numpy().reshape(B, -1),
                                  ref["next_observations"].reshape(B, -1))
    np.testing.assert_array_equal(batch.act.cpu().numpy().reshape(ref["actions"].shape),
                                  ref["actions"])
    np.testing.assert_array_equal(batch.rew.cpu().numpy(), ref["rewards"].reshape(-1))
    np.testing.assert_array_equal(batch.term.cpu().numpy(), ref["terminals"].reshape(-1))
    np.testing.assert_array_equal(batch.n_steps.cpu().numpy(), ref["n_steps"].reshape(-1))


@pytest.mark.gpu
@pytest.mark.parametrize("maxlen,n_steps", [(4000, 1), (4000, 3), (97, 1), (97, 3)])
def test_gpu_replay_sample_matches_reference(maxlen, n_steps):
    buf = ReplayBuffer(maxlen, env=ToyEnv())
    ob = OReplayBuffer(maxlen, (5,), 2)
    _fill([buf, ob], 900)
    B = 256
    np.random.seed(3)
    idx = ob.sample_indices(B)
    ref = ob.gather(idx, n_steps=n_steps, gamma=0.99)
    if n_steps == 1:
        np.random.seed(3)
        batch = buf.sample(B, n_steps=1, gamma=0.99)   # same np.random.choice stream
    else:
        batch = buf.sample(B, n_steps=n_steps, gamma=0.99, indices=idx)
    torch.cuda.synchronize()
    _compare(batch, ref)
    # appends after a sample reach the device copy on the next sample
    _fill([buf, ob], 150, seed=7)
    np.random.seed(4)
    idx = ob.sample_indices(128)
    _compare(buf.sample(128, indices=idx), ob.gather(idx))


@pytest.mark.gpu
def test_gpu_replay_sample_pixels_discrete():
    buf = ReplayBuffer(300, env=ToyEnv((1, 12, 12), 4, discrete=True))
    ob = OReplayBuffer(300, (1, 12, 12), 4)
    _fill([buf, ob], 400, obs_shape=(1, 12, 12), action_size=4, discrete=True)
    np.random.seed(5)
    idx = ob.sample_indices(64)
    _compare(buf.sample(64, indices=idx), ob.gather(idx))
    with pytest.raises(NotImplementedError):
        buf.sample(8, n_frames=4)


@pytest.mark.gpu
def test_gpu_fit_online_sac(tmp_path):
    from d3rlpy_amd.algos import SAC
    np.random.seed(0)
    torch.manual_seed(0)
    env = ToyEnv((5,), 2, seed=11)
    algo = SAC(batch_size=32)
    buf = ReplayBuffer(2000, env=env)
    hist = algo.fit_online(env, buf, n_steps=300, n_steps_per_epoch=100,
                           update_start_step=50, random_steps=50, logdir=str(tmp_path),
                           save_metrics=False, verbose=False, eval_env=ToyEnv(seed=12))
    assert len(hist) == 3
    for m in hist[1:]:
        for k in ("critic_loss", "actor_loss", "temp", "evaluation"):
            assert np.isfinite(m[k]), (k, m)
    assert len(buf) > 250


@pytest.mark.gpu
def test_gpu_fit_online_dqn_pixels(tmp_path):
    from d3rlpy_amd.algos import DQN
    np.random.seed(0)
    torch.manual_seed(0)
    env = ToyEnv((1, 84, 84), 4, discrete=True, seed=13)
    algo = DQN(batch_size=32, scaler="pixel", target_update_interval=50)
    hist = algo.fit_online(env, ReplayBuffer(1000, env=env),
                           LinearDecayEpsilonGreedy(1.0, 0.1, 200), n_steps=200,
                           n_steps_per_epoch=100, update_start_step=40,
                           logdir=str(tmp_path), save_metrics=False, verbose=False)
    assert len(hist) == 2 and np.isfinite(hist[-1]["loss"])


@pytest.mark.gpu
def test_gpu_collect_then_offline_fit(tmp_path):
    """collect (iterators.py:288-380) into the ring, to_mdp_dataset, then the
    offline fitter on the collected episodes."""
    from d3rlpy_amd.algos import SAC
    np.random.seed(0)
    torch.manual_seed(0)
    env = ToyEnv((5,), 2, seed=21)
    algo = SAC(batch_size=32)
    buf = algo.collect(env, n_steps=400)
    assert len(buf) >= 380
    g = algo.collect(ToyEnv((5,), 2, seed=22), deterministic=True, n_steps=50)
    a = g._h_act[0:2 * len(g):2]
    assert np.all(np.abs(a) <= 1.0)
    ds = buf.to_mdp_dataset()
    res = algo.fit(ds, n_steps=100, n_steps_per_epoch=100, save_metrics=False,
                   verbose=False, logdir=str(tmp_path))
    assert np.isfinite(res[-1][1]["critic_loss"])
