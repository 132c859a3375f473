"""More reference KATs restated against the oracle (CPU): the QR / ensemble /
discrete-mean / pixel-encoder / residual-policy / VAE / TorchMiniBatch tests
of /root/reference/tests, each cited, plus closed-form checks where the
reference test checks shapes only, and the squashed-Gaussian log-prob from
injected noise against the explicit formula (no retry loop)."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F
from torch.distributions import Normal

from oracle import bcq as ob
from oracle import discrete_cql as od
from oracle import models as om
from oracle.cql import Batch

from test_oracle_kats import ref_huber_loss, ref_quantile_huber_loss


def test_qr_taus_kat():
    """q_functions/test_qr_q_function.py:97-102: tau_i = i*step + step/2."""
    taus = ob.make_taus(200)
    step = 1 / 200
    for i in range(200):
        assert np.allclose(taus[0][i].numpy(), i * step + step / 2.0)


def test_qr_compute_error_kat():
    """q_functions/test_qr_q_function.py:104-131 (reduction none / mean)."""
    torch.manual_seed(0)
    B, F_, A, K, gamma = 32, 100, 2, 200, 0.99
    q = ob.ContinuousQRQFunction(om.VectorEncoderWithAction(F_, A, [16]), K)
    obs_t, act_t = torch.rand(B, F_), torch.rand(B, A)
    rew, q_tp1 = torch.rand(B, 1), torch.rand(B, K)
    ter = torch.randint(2, size=(B, 1))
    assert q.compute_error(obs_t, act_t, rew, q_tp1, ter, reduction="none").shape == (B, 1)
    loss = q.compute_error(obs_t, act_t, rew, q_tp1, ter)
    target = rew.numpy() + gamma * q_tp1.numpy() * (1 - ter.numpy())
    y = q.compute_target(obs_t, act_t).detach().numpy()
    ref = ref_quantile_huber_loss(y.reshape(B, 1, -1), target.reshape(B, -1, 1),
                                  ob.make_taus(K).numpy().reshape(1, 1, -1), K)
    assert np.allclose(loss.detach().numpy(), ref.mean())
    assert q.compute_target(obs_t, act_t).shape == (B, K)
    assert q(obs_t, act_t).shape == (B, 1)


@pytest.mark.parametrize("reduction", ["min", "max"])
def test_reduce_quantile_ensemble_kat(reduction):
    """q_functions/test_ensemble_q_function.py:44-61."""
    y = torch.rand(2, 32, 200)
    ret = ob.reduce_quantile_ensemble(y, reduction)
    mean = y.mean(dim=2)
    idx = (mean.min(dim=0) if reduction == "min" else mean.max(dim=0)).indices
    assert ret.shape == (32, 200)
    assert torch.allclose(ret, y[idx, torch.arange(32)])


def test_reduce_quantile_ensemble_mix():
    y = torch.rand(2, 8, 16)
    mix = ob.reduce_quantile_ensemble(y, "mix", lam=0.75)
    mn, mx = ob.reduce_quantile_ensemble(y, "min"), ob.reduce_quantile_ensemble(y, "max")
    assert torch.allclose(mix, 0.75 * mn + 0.25 * mx)


@pytest.mark.parametrize("kind", ["mean", "qr"])
def test_ensemble_compute_error_is_sum_kat(kind):
    """q_functions/test_ensemble_q_function.py:206-231: the ensemble TD loss
    is the sum of its members' compute_error."""
    torch.manual_seed(1)
    B, F_, A, K, E, gamma = 32, 100, 2, 200, 5, 0.99
    if kind == "mean":
        ens = om.EnsembleContinuousQFunction(
            [om.ContinuousMeanQFunction(om.VectorEncoderWithAction(F_, A, [16]))
             for _ in range(E)])
        q_tp1 = torch.rand(B, 1)
    else:
        ens = ob.EnsembleQRQFunction([ob.ContinuousQRQFunction(
            om.VectorEncoderWithAction(F_, A, [16]), K) for _ in range(E)])
        q_tp1 = torch.rand(B, K)
    obs_t, act_t, rew = torch.rand(B, F_), torch.rand(B, A), torch.rand(B, 1)
    ter = torch.randint(2, size=(B, 1))
    ref = 0.0
    for f in ens.q_funcs:
        ref += f.compute_error(obs_t, act_t, rew, q_tp1, ter, gamma)
    assert torch.allclose(ref, ens.compute_error(obs_t, act_t, rew, q_tp1, ter, gamma))
    if kind == "mean":  # test_ensemble_q_function.py:185-200
        values = ens(obs_t, act_t, "none")
        assert torch.equal(ens.compute_target(obs_t, act_t), values.min(dim=0).values)
        assert torch.allclose(values.mean(dim=0), ens(obs_t, act_t, "mean"))


def test_discrete_mean_q_huber_td_kat():
    """q_functions/test_mean_q_function.py:19-57 (ref_huber_loss of the
    picked Q against r + gamma * q' * (1 - terminal))."""
    torch.manual_seed(2)
    rs = np.random.RandomState(2)
    B, A, gamma = 32, 2, 0.99
    q = od.DiscreteMeanQFunction(od.PixelEncoder((1, 36, 36), feature_size=100), A)
    x = torch.rand(B, 1, 36, 36)
    assert q(x).shape == (B, A)
    act = torch.randint(high=A, size=(B,))
    assert torch.allclose(q(x)[torch.arange(B), act], q.compute_target(x, act).view(-1))
    q_tp1 = rs.random_sample((B, 1))
    rew = rs.random_sample((B, 1))
    ter = rs.randint(2, size=(B, 1))
    target = rew + gamma * q_tp1 * (1 - ter)
    act_t = rs.randint(A, size=(B, 1))
    q_t = q(x).detach().numpy()[np.arange(B), act_t.reshape(-1)]
    ref = ref_huber_loss(q_t.reshape(-1, 1), target)
    loss = q.compute_error(x, torch.tensor(act_t, dtype=torch.int64),
                           torch.tensor(rew, dtype=torch.float32),
                           torch.tensor(q_tp1, dtype=torch.float32),
                           torch.tensor(ter, dtype=torch.float32), gamma=gamma)
    assert np.allclose(loss.detach().numpy(), ref)


def test_pixel_encoder_geometry_kat():
    """models/torch/test_encoders.py:14-44: 4x84x84 -> 3136 -> 512."""
    enc = od.PixelEncoder((4, 84, 84), feature_size=512)
    assert enc._fc.in_features == 3136
    assert enc(torch.rand(32, 4, 84, 84)).shape == (32, 512)


def test_residual_policy_bound_kat():
    """models/torch/test_policies.py:43-61: a' != a and |a' - a| <= scale."""
    torch.manual_seed(3)
    pol = ob.DeterministicResidualPolicy(om.VectorEncoderWithAction(100, 2, [16]), 2, 0.05)
    x, a = torch.rand(32, 100), torch.rand(32, 2)
    y = pol(x, a)
    assert y.shape == (32, 2)
    assert not (y == a).any()
    assert ((y - a).abs() <= 0.05).all()


def test_conditional_vae_kat_and_loss():
    """models/torch/test_imitators.py:22-66 (shapes) + the loss of
    imitators.py:80-86 against its closed form: MSE(decode(x, mu + eps*sigma),
    a) + beta * mean KL(N(mu, sigma) || N(0, 1))."""
    torch.manual_seed(4)
    B, F_, A, L, beta = 32, 100, 2, 32, 0.5
    vae = ob.ConditionalVAE(om.VectorEncoderWithAction(F_, A, [16]),
                            om.VectorEncoderWithAction(F_, L, [16]), A, L, beta,
                            min_logstd=-4.0, max_logstd=15.0)
    x, a = torch.rand(B, F_), torch.rand(B, A)
    dist = vae.encode(x, a)
    assert isinstance(dist, Normal) and dist.mean.shape == (B, L)
    assert vae.decode(x, torch.rand(B, L)).shape == (B, A)
    eps = torch.randn(B, L)
    loss = vae.compute_error(x, a, eps)
    mu, sd = dist.loc.double(), dist.scale.double()
    kl = (torch.log(1.0 / sd) + (sd ** 2 + mu ** 2) / 2 - 0.5).mean()
    y = vae.decode(x, (dist.loc + eps * dist.scale)).double()
    ref = ((y - a.double()) ** 2).mean() + beta * kl
    assert abs(float(loss.detach()) - float(ref)) <= 1e-5 * max(1.0, abs(float(ref)))


def test_torch_mini_batch_scaler_kat():
    """test_torch_utility.py:282-369: the observation scaler transforms
    observations and next_observations only (actions / rewards / terminals /
    n_steps untouched) — the oracle's TorchMiniBatch stage (TD3PlusBCOracle
    ._scaled)."""
    from oracle.td3bc import TD3PlusBCOracle

    class DummyScaler:
        def transform(self, x):
            return x + 0.1

    rs = np.random.RandomState(5)
    B = 32
    b = Batch.from_numpy(rs.random_sample((B, 3)), rs.random_sample((B, 1)),
                         rs.random_sample(B), rs.random_sample((B, 3)), np.zeros(B),
                         np.ones(B))
    orc = TD3PlusBCOracle(3, 1, hidden_units=[8], scaler=DummyScaler())
    s = orc._scaled(b)
    assert torch.equal(s.observations, b.observations + 0.1)
    assert torch.equal(s.next_observations, b.next_observations + 0.1)
    for f in ("actions", "rewards", "terminals", "n_steps"):
        assert torch.equal(getattr(s, f), getattr(b, f))


def test_compute_max_with_n_actions_brute_force():
    """tests/models/torch/test_q_functions.py:21-45 checks the shape
    (batch, n_quantiles); the selection itself against a loop restating
    q_functions/__init__.py:8-63: per (row, sample) the member with the
    max / min mean quantile, mix = (1-lam) max + lam min of the means, the
    argmax sample, and the mixed quantile vectors of that sample."""
    torch.manual_seed(6)
    B, N, A, K, lam = 100, 10, 2, 32, 0.75
    ens = ob.EnsembleQRQFunction([ob.ContinuousQRQFunction(
        om.VectorEncoderWithAction(6, A, [16]), K) for _ in range(2)])
    x, acts = torch.rand(B, 6), torch.rand(B, N, A)
    got = ob.compute_max_with_n_actions(x, acts, ens, lam)
    assert got.shape == (B, K)
    with torch.no_grad():
        for b in range(0, B, 7):
            qs = torch.stack([torch.stack([f.compute_target(x[b:b + 1], acts[b, n:n + 1])[0]
                                           for n in range(N)]) for f in ens.q_funcs])  # C,N,K
            means = qs.mean(-1)  # C, N
            mx, mn = means.max(0), means.min(0)
            pick = ((1 - lam) * mx.values + lam * mn.values).argmax()
            ref = (1 - lam) * qs[mx.indices[pick], pick] + lam * qs[mn.indices[pick], pick]
            assert torch.allclose(got[b], ref, atol=1e-6)


def test_squashed_gaussian_log_prob_formula():
    """distributions.py:133-135 with the rsample draw injected: the oracle's
    log-prob equals sum_a [log N(u; mu, sigma) - 2 (log 2 - u - softplus(-2u))],
    u = mu + sigma * eps, evaluated in fp64 (no atanh round trip, so no retry
    loop or 1e-2 tolerance as in test_distributions.py:58-102)."""
    torch.manual_seed(7)
    mu = torch.rand(32, 3) * 2 - 1
    sd = torch.rand(32, 3).exp()
    eps = torch.randn(32, 3)
    y, lp = om.SquashedGaussian(mu, sd).sample_with_log_prob(eps)
    u = mu.double() + sd.double() * eps.double()
    lnorm = -((u - mu.double()) ** 2) / (2 * sd.double() ** 2) - torch.log(sd.double()) \
        - 0.5 * math.log(2 * math.pi)
    ref = (lnorm - 2 * (math.log(2) - u - F.softplus(-2 * u))).sum(-1, keepdim=True)
    assert torch.allclose(lp.double(), ref, rtol=2e-6, atol=2e-6)
    assert torch.allclose(y.double(), torch.tanh(u), atol=1e-6)
    # sample_n: (n, batch, action) / (n, batch, 1)
    yn, lpn = om.SquashedGaussian(mu, sd).sample_n_with_log_prob(torch.randn(10, 32, 3))
    assert yn.shape == (10, 32, 3) and lpn.shape == (10, 32, 1)
