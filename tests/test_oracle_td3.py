"""Known-answer checks of the TD3+BC oracle restatement (CPU).

The reference's own TD3+BC tests (tests/algos/test_td3_plus_bc.py,
tests/algos/torch/test_td3_plus_bc_impl.py) only exercise the update loop
and carry no vectors, so these pin the restated formulas against closed-form
values of td3_impl.py:61-78 and td3_plus_bc_impl.py:64-70.
"""
import numpy as np
import torch

from oracle.cql import Batch
from oracle.td3bc import StandardScalerT, TD3PlusBCOracle, fit_standard_scaler


def _batch(rs, B, D, A):
    return Batch.from_numpy(rs.randn(B, D).astype(np.float32),
                            rs.uniform(-1, 1, (B, A)).astype(np.float32),
                            rs.randn(B).astype(np.float32), rs.randn(B, D).astype(np.float32),
                            (rs.rand(B) < 0.3).astype(np.float32), np.ones(B, np.float32))


def test_target_without_noise_is_min_of_target_critics():
    rs = np.random.RandomState(0)
    orc = TD3PlusBCOracle(4, 2, hidden_units=[16, 16], seed=1)
    b = _batch(rs, 8, 4, 2)
    y = orc.compute_target(b, torch.zeros(8, 2))
    a = orc._targ_policy(b.next_observations)
    qs = torch.stack([q(b.next_observations, a) for q in orc._targ_q_func.q_funcs])
    assert torch.allclose(y, qs.min(0).values)


def test_target_noise_is_clipped_then_action_clamped():
    rs = np.random.RandomState(1)
    orc = TD3PlusBCOracle(3, 2, hidden_units=[8], seed=2, target_smoothing_sigma=0.2,
                          target_smoothing_clip=0.5)
    b = _batch(rs, 5, 3, 2)
    big = torch.full((5, 2), 100.0)
    a = orc._targ_policy(b.next_observations)
    expect = (a + 0.5).clamp(-1, 1)  # sigma*100 clipped to +0.5, then into [-1, 1]
    y = orc.compute_target(b, big)
    qs = torch.stack([q(b.next_observations, expect) for q in orc._targ_q_func.q_funcs])
    assert torch.allclose(y, qs.min(0).values)


def test_actor_loss_closed_form_and_detached_lambda():
    rs = np.random.RandomState(2)
    orc = TD3PlusBCOracle(4, 3, hidden_units=[16, 16], alpha=2.5, seed=3)
    b = _batch(rs, 12, 4, 3)
    a = orc._policy(b.observations)
    q0 = orc._q_func.q_funcs[0](b.observations, a)
    lam = 2.5 / q0.abs().mean()
    expect = -lam * q0.mean() + ((b.actions - a) ** 2).mean()
    got = orc.compute_actor_loss(b)
    assert torch.allclose(got, expect)
    # lambda is detached: dL/dq0 is -lam / B for every row (what the HIP seed
    # kernel writes), not the derivative of alpha * q / mean|q|
    q_leaf = q0.detach().clone().requires_grad_(True)
    lam_d = 2.5 / q_leaf.abs().mean().detach()
    (lam_d * -q_leaf.mean()).backward()
    assert torch.allclose(q_leaf.grad, torch.full_like(q_leaf, -float(lam_d) / 12))


def test_standard_scaler_transform_and_fit():
    rs = np.random.RandomState(3)
    obs = rs.randn(1000, 5) * 3 + 1
    mean, std = fit_standard_scaler(obs)
    assert np.allclose(mean, obs.mean(0)) and np.allclose(std, obs.std(0))
    sc = StandardScalerT(mean, std, eps=1e-3)
    x = torch.from_numpy(obs[:7].astype(np.float32))
    m32 = torch.tensor(mean.reshape(1, -1), dtype=torch.float32)
    s32 = torch.tensor(std.reshape(1, -1), dtype=torch.float32)
    assert torch.equal(sc.transform(x), (x - m32) / (s32 + 1e-3))


def test_delayed_actor_schedule():
    rs = np.random.RandomState(4)
    orc = TD3PlusBCOracle(3, 1, hidden_units=[8], seed=5)
    b = _batch(rs, 4, 3, 1)
    n = torch.zeros(4, 1)
    p0 = [p.clone() for p in orc._policy.parameters()]
    t0 = [p.clone() for p in orc._targ_q_func.parameters()]
    m = orc.update(b, n, grad_step=1)
    assert set(m) == {"critic_loss"}
    assert all(torch.equal(a, b_) for a, b_ in zip(p0, orc._policy.parameters()))
    assert all(torch.equal(a, b_) for a, b_ in zip(t0, orc._targ_q_func.parameters()))
    m = orc.update(b, n, grad_step=2)
    assert set(m) == {"critic_loss", "actor_loss"}
    assert not all(torch.equal(a, b_) for a, b_ in zip(t0, orc._targ_q_func.parameters()))


def test_td3_ddpg_oracle_parents():
    """TD3Oracle / DDPGOracle restate the parents of TD3PlusBCImpl:
    the DDPG actor loss is -mean Q_0(s, pi(s)) (ddpg_impl.py:244-249), and
    DDPG's unsmoothed target (ddpg_impl.py:251-260) equals TD3's target with
    sigma = clip = 0 (what the HIP DDPGImpl runs) bit for bit."""
    import torch
    from oracle.cql import Batch
    from oracle.td3bc import DDPGOracle, TD3Oracle
    rs = np.random.RandomState(3)
    B, D, A = 16, 4, 2
    arrs = (rs.randn(B, D).astype(np.float32), rs.uniform(-1, 1, (B, A)).astype(np.float32),
            rs.randn(B).astype(np.float32), rs.randn(B, D).astype(np.float32),
            np.zeros(B, np.float32), np.ones(B, np.float32))
    tb = Batch.from_numpy(*arrs)
    td3 = TD3Oracle(D, A, hidden_units=(32, 32), seed=1)
    with torch.no_grad():
        act = td3._policy(tb.observations)
        q0 = td3._q_func(tb.observations, act, "none")[0]
        assert torch.equal(td3.compute_actor_loss(tb), -q0.mean())
    ddpg = DDPGOracle(D, A, hidden_units=(32, 32), seed=1)
    assert len(ddpg._q_func.q_funcs) == 1
    ref = TD3Oracle(D, A, n_critics=1, hidden_units=(32, 32), seed=1,
                    target_smoothing_sigma=0.0, target_smoothing_clip=0.0)
    noise = torch.randn(B, A, generator=torch.Generator().manual_seed(0))
    assert torch.equal(ddpg.compute_target(tb), ref.compute_target(tb, noise))
