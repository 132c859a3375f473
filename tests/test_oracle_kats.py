"""Pin the oracle against the reference test-suite's known-answer tests (CPU).

Each test restates one KAT from /root/reference/tests (cited) and applies it
to the oracle's restated function.  The reference cannot be imported here
(SURVEY §8c), so these formula-level KATs are what pins the oracle.
"""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F
from torch.distributions import Normal

from oracle import gather as og
from oracle import models as om


def ref_huber_loss(a, b):
    """tests/models/torch/model_test.py:31-38."""
    abs_diff = np.abs(a - b).reshape((-1,))
    l2_diff = ((a - b) ** 2).reshape((-1,))
    huber_diff = np.zeros_like(abs_diff)
    huber_diff[abs_diff < 1.0] = 0.5 * l2_diff[abs_diff < 1.0]
    huber_diff[abs_diff >= 1.0] = abs_diff[abs_diff >= 1.0] - 0.5
    return np.mean(huber_diff)


def ref_quantile_huber_loss(a, b, taus, n_quantiles):
    """tests/models/torch/model_test.py:41-49."""
    abs_diff = np.abs(a - b).reshape((-1,))
    l2_diff = ((a - b) ** 2).reshape((-1,))
    huber_diff = np.zeros_like(abs_diff)
    huber_diff[abs_diff < 1.0] = 0.5 * l2_diff[abs_diff < 1.0]
    huber_diff[abs_diff >= 1.0] = abs_diff[abs_diff >= 1.0] - 0.5
    huber_diff = huber_diff.reshape(-1, n_quantiles, n_quantiles)
    delta = np.array((b - a) < 0.0, dtype=np.float32)
    element_wise_loss = np.abs(taus - delta) * huber_diff
    return element_wise_loss.sum(axis=2).mean(axis=1)


def test_huber_kat():
    """q_functions/test_mean_q_function.py:38-57 uses ref_huber_loss on TD errors."""
    rs = np.random.RandomState(0)
    a = rs.randn(64, 1) * 2
    b = rs.randn(64, 1) * 2
    loss = om.huber_loss(torch.tensor(a), torch.tensor(b)).mean()
    assert np.allclose(loss.numpy(), ref_huber_loss(a, b))


def test_quantile_huber_kat():
    """q_functions/test_utility.py:57-69."""
    rs = np.random.RandomState(1)
    y = rs.random_sample((32, 200, 1))
    target = rs.random_sample((32, 1, 200))
    taus = rs.random_sample((1, 1, 200))
    ref = ref_quantile_huber_loss(y, target, taus, 200)
    loss = om.quantile_huber_loss(torch.tensor(y), torch.tensor(target), torch.tensor(taus))
    assert np.allclose(loss.numpy(), ref)


@pytest.mark.parametrize("reduction", ["min", "max", "mean", "none"])
def test_reduce_ensemble_kat(reduction):
    """q_functions/test_ensemble_q_function.py:24-41."""
    y = torch.rand(2, 32, 1)
    ret = om.reduce_ensemble(y, reduction)
    ref = {"min": y.min(dim=0).values, "max": y.max(dim=0).values, "mean": y.mean(dim=0),
           "none": y}[reduction]
    assert torch.equal(ret, ref)


def test_continuous_mean_q_td_kat():
    """q_functions/test_mean_q_function.py:84-100: continuous TD error is MSE."""
    torch.manual_seed(0)
    enc = om.VectorEncoderWithAction(100, 2, [16])
    qf = om.ContinuousMeanQFunction(enc)
    rs = np.random.RandomState(2)
    gamma = 0.99
    q_tp1 = rs.random_sample((32, 1))
    rew_tp1 = rs.random_sample((32, 1))
    ter_tp1 = rs.randint(2, size=(32, 1))
    target = rew_tp1 + gamma * q_tp1 * (1 - ter_tp1)
    obs_t = torch.rand(32, 100)
    act_t = torch.rand(32, 2)
    q_t = qf(obs_t, act_t).detach().numpy()
    ref_loss = ((q_t - target) ** 2).mean()
    loss = qf.compute_error(obs_t, act_t, torch.tensor(rew_tp1, dtype=torch.float32),
                            torch.tensor(q_tp1, dtype=torch.float32),
                            torch.tensor(ter_tp1, dtype=torch.float32), gamma)
    assert np.allclose(loss.detach().numpy(), ref_loss)


def _ref_squashed_log_prob(dist, y):
    """tests/models/torch/test_distributions.py:51-55."""
    clipped_y = y.clamp(-0.999999, 0.999999)
    raw_y = torch.atanh(clipped_y)
    jacob = 2 * (math.log(2) - raw_y - F.softplus(-2 * raw_y))
    return (dist.log_prob(raw_y) - jacob).sum(dim=-1, keepdims=True)


def test_squashed_gaussian_kat():
    """test_distributions.py:58-102 (atol=1e-2 as in the reference)."""
    torch.manual_seed(3)
    mean = torch.rand(32, 2)
    std = torch.rand(32, 2).exp()
    dist = om.SquashedGaussian(mean, std)
    ref_dist = Normal(mean, std)
    ok = False
    for _ in range(10):
        eps = torch.randn(32, 2)
        y, log_prob = dist.sample_with_log_prob(eps)
        ref = _ref_squashed_log_prob(ref_dist, y)
        if y.shape == (32, 2) and log_prob.shape == (32, 1) and \
                torch.allclose(log_prob, ref, atol=1e-2):
            ok = True
            break
    assert ok
    # sample_n: (n, batch, action) / (n, batch, 1)
    y, lp = dist.sample_n_with_log_prob(torch.randn(10, 32, 2))
    assert y.shape == (10, 32, 2) and lp.shape == (10, 32, 1)
    assert torch.allclose(dist.mean_with_log_prob()[0], torch.tanh(mean))


def test_soft_hard_sync_kat():
    """tests/test_torch_utility.py:33-56."""
    torch.manual_seed(4)
    module = torch.nn.Linear(32, 32)
    targ = torch.nn.Linear(32, 32)
    original = torch.nn.Linear(32, 32)
    original.load_state_dict(targ.state_dict())
    tau = 0.05
    om.soft_sync(targ, module, tau)
    for p, tp, op in zip(module.parameters(), targ.parameters(), original.parameters()):
        assert torch.allclose(p * tau + op * (1.0 - tau), tp)
    om.hard_sync(targ, module)
    for p, tp in zip(module.parameters(), targ.parameters()):
        assert torch.allclose(tp, p)


@pytest.mark.parametrize("observation_shape", [(100,), (4, 84, 84)])
@pytest.mark.parametrize("n_frames", [1, 4])
@pytest.mark.parametrize("n_steps", [1, 3])
@pytest.mark.parametrize("discrete_action", [False, True])
def test_transition_minibatch_kat(observation_shape, n_frames, n_steps, discrete_action):
    """tests/test_dataset.py:321-420 (test_transition_minibatch), data_size 100."""
    data_size, action_size, gamma = 100, 2, 0.99
    rs = np.random.RandomState(5)
    if len(observation_shape) == 3:
        observations = rs.randint(256, size=(data_size, *observation_shape), dtype=np.uint8)
    else:
        observations = rs.random_sample((data_size,) + observation_shape).astype("f4")
    if discrete_action:
        actions = rs.randint(action_size, size=data_size)
    else:
        actions = rs.random_sample((data_size, action_size)).astype("f4")
    rewards = rs.random_sample((data_size, 1)).astype("f4")
    transitions = og.to_transitions(observations, actions, rewards, 1.0)
    batch = og.gather(transitions, n_frames, n_steps, gamma)
    if len(observation_shape) == 3:
        shape = (data_size, n_frames * observation_shape[0], *observation_shape[1:])
        if n_frames == 1:
            shape = (data_size, *observation_shape)
    else:
        shape = (data_size, *observation_shape)
    assert batch["observations"].shape == shape
    assert batch["next_observations"].shape == shape
    for i, t in enumerate(transitions):
        observation = batch["observations"][i]
        next_observation = batch["next_observations"][i]
        n = int(batch["n_steps"][i][0])
        assert n == min(data_size - i, n_steps)
        if n_frames > 1 and len(observation_shape) == 3:
            pad = ((n_frames - 1, 1), (0, 0), (0, 0), (0, 0))
            padded = np.pad(observations, pad, "edge")
            window = padded[i:i + n_frames]
            next_window = padded[i + n:i + n_frames + n]
            assert np.all(observation == np.vstack(window))
            if i >= data_size - n_steps:
                assert np.all(next_observation == 0)
            else:
                assert np.all(next_observation == np.vstack(next_window))
        else:
            next_t = t
            for _ in range(n - 1):
                next_t = next_t.next
            assert np.allclose(observation, t.observation)
            assert np.allclose(next_observation, next_t.next_observation)
        n_step_reward = 0.0
        terminal = 0.0
        next_t = t
        for j in range(n):
            n_step_reward += rewards[i + j] * gamma ** j
            terminal = next_t.terminal
            next_t = next_t.next
        assert np.all(batch["actions"][i] == t.action)
        assert np.allclose(batch["rewards"][i][0], n_step_reward)
        assert np.all(batch["terminals"][i][0] == terminal)


def test_random_iterator_stream():
    """iterators/random_iterator.py:38-41: one global-RNG randint per sample."""
    np.random.seed(7)
    a = og.random_indices(1000, 16)
    np.random.seed(7)
    b = np.array([np.random.randint(1000) for _ in range(16)])
    assert np.array_equal(a, b)
