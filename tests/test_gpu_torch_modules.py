"""Reference-shaped torch modules running forward AND backward on the HIP custom
ops (torch.ops.d3rlpy_amd.* through the autograd functions of
d3rlpy_amd/torch_ops.py), checked against the CPU oracle's loss and
gradients (GPU only).

  * CQL critic loss (cql_impl.py:110-125 + 196-223: TD error of the mean-Q
    ensemble + conservative logsumexp term, with the policy's importance
    samples drawn by squashed_gaussian_sample) -> the critic's gradients
  * SAC / CQL actor loss (sac_impl.py:114-121) -> the policy's gradients
  * QR quantile loss (q_functions/utility.py:49-64) -> dL/dquantiles
  * IQN embedding + quantile Huber (iqn_q_function.py:33-47) -> the embed
    layer's gradients

Bars: losses within 1e-5 (relative), gradients within 2e-5 of the largest
entry (fp32 on both sides, different summation orders) — the bars of the
pipeline parity tests.
"""
import math

import numpy as np
import pytest
import torch

from d3rlpy_amd import torch_ops as T
from oracle.cql import Batch, CQLNoise, CQLOracle

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(got, exp, tol=2e-5, what=""):
    got, exp = got.detach().double().cpu(), exp.detach().double().cpu()
    scale = exp.abs().max().clamp_min(1e-12)
    err = float((got - exp).abs().max() / scale)
    assert err <= tol, f"{what}: {err:.3g}"


def _param(t):
    return t.detach().to(DEV).clone().requires_grad_(True)


class HipQ:
    """EnsembleContinuousQFunction of mean-Q members on the HIP ops: member
    weights stacked [C][out][in], every layer one launch for all members."""

    def __init__(self, q_funcs):
        fcs = [[*q._encoder._fcs, q._fc] for q in q_funcs]
        self.W = [_param(torch.stack([f[l].weight for f in fcs])) for l in range(len(fcs[0]))]
        self.b = [_param(torch.stack([f[l].bias for f in fcs])) for l in range(len(fcs[0]))]

    def __call__(self, x, a):  # -> [C, R, 1]
        h = torch.cat([x, a], dim=1)
        for l in range(len(self.W)):
            h = T.linear(h, self.W[l], self.b[l], relu=l + 1 < len(self.W))
        return h

    def params(self):
        return [p for pair in zip(self.W, self.b) for p in pair]


class HipPolicy:
    """SquashedNormalPolicy on the HIP ops (mu / logstd heads, clamp inside the
    sampling op)."""

    def __init__(self, pol):
        self.W = [_param(fc.weight) for fc in pol._encoder._fcs]
        self.b = [_param(fc.bias) for fc in pol._encoder._fcs]
        self.Wm, self.bm = _param(pol._mu.weight), _param(pol._mu.bias)
        self.Ws, self.bs = _param(pol._logstd.weight), _param(pol._logstd.bias)
        self.lo, self.hi = pol._min_logstd, pol._max_logstd

    def heads(self, x):
        h = x
        for W, b in zip(self.W, self.b):
            h = T.linear(h, W, b, relu=True)
        return T.linear(h, self.Wm, self.bm), T.linear(h, self.Ws, self.bs)

    def sample_with_log_prob(self, x, eps):
        mu, ls = self.heads(x)
        return T.squashed_gaussian_sample(mu, ls, eps, self.lo, self.hi)

    def sample_n_with_log_prob(self, x, eps_n):  # eps_n [n, B, A] -> ([B, n, A], [B, n, 1])
        n, B, A = eps_n.shape
        mu, ls = self.heads(x)
        act, lp = T.squashed_gaussian_sample(mu.expand(n, B, A).reshape(-1, A),
                                             ls.expand(n, B, A).reshape(-1, A),
                                             eps_n.reshape(-1, A), self.lo, self.hi)
        return act.view(n, B, A).transpose(0, 1), lp.view(n, B, 1).transpose(0, 1)

    def params(self):
        ps = [p for pair in zip(self.W, self.b) for p in pair]
        return ps + [self.Wm, self.bm, self.Ws, self.bs]


def _setup(B=32, D=11, A=3, N=10, seed=0):
    orc = CQLOracle(D, A, n_critics=2, n_action_samples=N, seed=seed)
    rs = np.random.RandomState(seed)
    batch = Batch.from_numpy(rs.randn(B, D), np.tanh(rs.randn(B, A)), rs.randn(B),
                             rs.randn(B, D), (rs.rand(B) < 0.1).astype(np.float32),
                             rs.randint(1, 3, size=B))
    noise = CQLNoise.draw(torch.Generator().manual_seed(seed + 1), B, A, N)
    return orc, batch, noise


def test_cql_critic_loss_and_grads_through_hip_ops():
    orc, batch, noise = _setup()
    B, A, N, C = batch.observations.shape[0], 3, 10, 2
    q_tpn = orc.compute_target(batch, noise)  # the target network's value (no grad)
    for p in orc._q_func.parameters():
        p.grad = None
    ref_loss = orc.compute_critic_loss(batch, q_tpn, noise)
    ref_loss.backward()
    ref_grads = [p.grad.clone() for q in orc._q_func.q_funcs
                 for p in [*sum([[fc.weight, fc.bias] for fc in q._encoder._fcs], []),
                           q._fc.weight, q._fc.bias]]

    q, pol = HipQ(orc._q_func.q_funcs), HipPolicy(orc._policy)
    g = lambda t: t.to(DEV)  # noqa: E731
    obs, act, obs1 = g(batch.observations), g(batch.actions), g(batch.next_observations)

    def policy_is_values(policy_obs, value_obs, eps_n):  # cql_impl.py:143-171
        with torch.no_grad():
            pa, lp = pol.sample_n_with_log_prob(policy_obs, g(eps_n))
        flat_obs = value_obs.expand(N, *value_obs.shape).transpose(0, 1).reshape(-1, 11)
        vals = q(flat_obs, pa.reshape(-1, A)).view(C, B, N)
        return vals - lp.reshape(1, B, N)

    def random_is_values(o, rand):  # cql_impl.py:173-194
        flat_obs = o.expand(N, *o.shape).transpose(0, 1).reshape(-1, 11)
        return q(flat_obs, g(rand)).view(C, B, N) - math.log(0.5 ** A)

    tv = torch.cat([policy_is_values(obs, obs, noise.critic_pi_t),
                    policy_is_values(obs1, obs, noise.critic_pi_tp1),
                    random_is_values(obs, noise.critic_rand)], dim=2)
    lse = T.logsumexp(tv, keepdim=True)  # the conservative logsumexp op
    data = q(obs, act)  # [C, B, 1]
    cons = lse.mean(dim=0).mean() - data.mean(dim=0).mean()
    alpha = orc._log_alpha().exp().clamp(0, 1e6)[0][0].to(DEV)
    cons = alpha * (orc._conservative_weight * cons - orc._alpha_threshold)
    gamma = g(orc._gamma ** batch.n_steps).view(-1)
    td = T.td_mse_loss(data.view(C, B), g(batch.rewards).view(-1),
                       g(q_tpn).view(1, B).expand(C, B).contiguous(), g(batch.terminals).view(-1),
                       gamma)
    loss = td.sum() + cons
    loss.backward()
    assert abs(float(loss.detach()) - float(ref_loss)) <= 1e-5 * max(1.0, abs(float(ref_loss)))
    for l in range(3):  # reference order per member: fcs..., _fc
        for c in range(C):
            per = 6
            _close(q.W[l].grad[c], ref_grads[c * per + 2 * l], what=f"W{l}[{c}]")
            _close(q.b[l].grad[c], ref_grads[c * per + 2 * l + 1], what=f"b{l}[{c}]")


def test_sac_actor_loss_and_grads_through_hip_ops():
    orc, batch, noise = _setup(seed=3)
    for p in orc._policy.parameters():
        p.grad = None
    ref = orc.compute_actor_loss(batch, noise.eps_actor)
    ref.backward()
    q, pol = HipQ(orc._q_func.q_funcs), HipPolicy(orc._policy)
    obs = batch.observations.to(DEV)
    act, lp = pol.sample_with_log_prob(obs, noise.eps_actor.to(DEV))
    temp = orc._log_temp().exp().to(DEV)[0][0]
    q_t = q(obs, act).min(dim=0).values  # reduce_ensemble "min"
    loss = (temp * lp - q_t).mean()
    loss.backward()
    assert abs(float(loss) - float(ref)) <= 1e-5 * max(1.0, abs(float(ref)))
    refp = [*sum([[fc.weight, fc.bias] for fc in orc._policy._encoder._fcs], []),
            orc._policy._mu.weight, orc._policy._mu.bias, orc._policy._logstd.weight,
            orc._policy._logstd.bias]
    for got, exp, name in zip(pol.params(), refp, ["W0", "b0", "W1", "b1", "mu.W", "mu.b",
                                                   "ls.W", "ls.b"]):
        _close(got.grad, exp.grad, what=name)


def test_qr_quantile_loss_through_hip_op():
    from oracle.bcq import compute_quantile_loss, make_taus
    gen = torch.Generator().manual_seed(5)
    B, K, gamma = 64, 200, 0.99
    qt = torch.randn(B, K, generator=gen).requires_grad_(True)
    rew = torch.randn(B, 1, generator=gen)
    targ = torch.randn(B, K, generator=gen)
    term = (torch.rand(B, 1, generator=gen) < 0.2).float()
    taus = make_taus(K)
    ref = compute_quantile_loss(qt, rew, targ, term, taus, gamma).mean()
    ref.backward()
    qh = qt.detach().to(DEV).requires_grad_(True)
    y = (rew + gamma * targ * (1 - term)).to(DEV)  # utility.py:58
    loss = T.quantile_huber_loss(qh, y, taus.view(1, K).expand(B, K).contiguous().to(DEV)).mean()
    loss.backward()
    assert abs(float(loss) - float(ref)) <= 1e-5 * abs(float(ref))
    _close(qh.grad, qt.grad, what="dq")


def test_iqn_embedding_and_quantile_loss_through_hip_ops():
    from oracle.discrete_cql import compute_iqn_feature
    gen = torch.Generator().manual_seed(7)
    B, K, E, F = 16, 64, 64, 128
    h = torch.randn(B, F, generator=gen)
    taus = torch.rand(B, K, generator=gen)
    embed = torch.nn.Linear(E, F)
    with torch.no_grad():
        embed.weight.copy_(torch.randn(F, E, generator=gen) * 0.1)
        embed.bias.copy_(torch.randn(F, generator=gen) * 0.1)
    y = torch.randn(B, K, generator=gen)
    feat = compute_iqn_feature(h, taus, embed, E)  # [B, K, F]
    quant = feat.sum(dim=2)  # a linear read-out of the feature
    from oracle.bcq import compute_quantile_huber_loss
    ref = compute_quantile_huber_loss(quant.view(B, 1, K), y.view(B, K, 1),
                                      taus.view(B, 1, K)).mean()
    ref.backward()
    W, b = _param(embed.weight), _param(embed.bias)
    phi = T.iqn_cos_embed(taus.to(DEV), W, b).view(B, K, F)
    hq = (h.to(DEV).view(B, 1, F) * phi).sum(dim=2)
    loss = T.quantile_huber_loss(hq, y.to(DEV), taus.to(DEV)).mean()
    loss.backward()
    assert abs(float(loss) - float(ref)) <= 1e-5 * abs(float(ref))
    _close(W.grad, embed.weight.grad, what="embed.W")
    _close(b.grad, embed.bias.grad, what="embed.b")


def test_op_gradients_match_torch_autograd():
    """Each forward / backward pair against torch's own autograd of the
    reference expression (logsumexp: fp64; the squashed Gaussian: fp32, the
    reference's precision), including clamp-active logstd entries."""
    gen = torch.Generator(device=DEV).manual_seed(11)
    x = torch.randn(2, 40, 30, device=DEV, generator=gen)
    xd = x.double().requires_grad_(True)
    gx = torch.randn(2, 40, device=DEV, generator=gen)
    xh = x.clone().requires_grad_(True)
    T.logsumexp(xh).backward(gx)
    torch.logsumexp(xd, dim=-1).backward(gx.double())
    _close(xh.grad, xd.grad, tol=1e-6, what="logsumexp")
    mu = torch.randn(64, 6, device=DEV, generator=gen)
    ls = torch.randn(64, 6, device=DEV, generator=gen)
    ls[0, 0], ls[1, 1] = 2.5, -25.0  # clamp active
    eps = torch.randn(64, 6, device=DEV, generator=gen)
    mh, lh = mu.clone().requires_grad_(True), ls.clone().requires_grad_(True)
    a, lp = T.squashed_gaussian_sample(mh, lh, eps)
    ga = torch.randn_like(a)
    gl = torch.randn_like(lp)
    (a * ga).sum().backward(retain_graph=True)
    (lp * gl).sum().backward()
    # the reference's own precision: torch fp32 autograd of policies.py /
    # distributions.py (at the clamp floor std = e^-20 the fp32 raw - mu
    # cancels, in the reference as here, so fp64 is not the yardstick)
    md, ld = mu.clone().requires_grad_(True), ls.clone().requires_grad_(True)
    std = ld.clamp(-20.0, 2.0).exp()
    raw = md + eps * std
    dist = torch.distributions.Normal(md, std)
    jac = 2 * (math.log(2) - raw - torch.nn.functional.softplus(-2 * raw))
    lpd = (dist.log_prob(raw) - jac).sum(dim=-1, keepdim=True)
    ((torch.tanh(raw) * ga).sum() + (lpd * gl).sum()).backward()
    _close(a, torch.tanh(raw), tol=1e-6, what="action")
    _close(lp, lpd, tol=1e-5, what="log_prob")
    _close(mh.grad, md.grad, tol=1e-5, what="dmu")
    _close(lh.grad, ld.grad, tol=1e-5, what="dlogstd")
    assert float(lh.grad[0, 0]) == 0.0 and float(lh.grad[1, 1]) == 0.0
