"""TD3 and DDPG update parity: HIP TD3Impl / DDPGImpl (d3rlpy_amd.algos.td3)
vs the CPU oracle restatements (oracle.td3bc.TD3Oracle / DDPGOracle), GPU only.

Same protocol and tolerances as tests/test_gpu_td3_parity.py: every step starts
from the oracle's exact state (reference checkpoint layout), both run one
``_update`` of the reference schedule (TD3: actor + targets every 2nd step;
DDPG: every step) on the same batch and target-smoothing noise.
  losses      |a-b| <= 1e-5 * max(1, |b|)
  gradients   max|a-b| / max|b| <= 2e-5 per tensor
  parameters  |a-b| <= 1e-5 absolute (targets included)
"""
import numpy as np
import pytest
import torch

from cql_helpers import HostBatch, max_rel
from oracle.cql import Batch
from td3_helpers import (make_family_impl, make_scaler_stats, make_td3_batch, make_td3_oracle,
                         td3_oracle_state)

pytestmark = pytest.mark.gpu

CASES = {
    "td3_hopper": dict(kind="td3", D=11, A=3, hidden=[256, 256], B=256, C=2, scaler=False),
    "td3_scaled_small": dict(kind="td3", D=5, A=2, hidden=[64, 64], B=32, C=2, scaler=True),
    "ddpg_pendulum": dict(kind="ddpg", D=3, A=1, hidden=[256, 256], B=100, C=1, scaler=False),
    "ddpg_two_critics": dict(kind="ddpg", D=7, A=2, hidden=[128, 128], B=64, C=2, scaler=True),
}


def _critic_grads(orc):
    return [[(fc.weight.grad.clone(), fc.bias.grad.clone())
             for fc in list(qf._encoder._fcs) + [qf._fc]] for qf in orc._q_func.q_funcs]


def _policy_grads(orc):
    pol = orc._policy
    return ([(fc.weight.grad.clone(), fc.bias.grad.clone()) for fc in pol._encoder._fcs]
            + [(pol._fc.weight.grad.clone(), pol._fc.bias.grad.clone())])


@pytest.mark.parametrize("case", list(CASES))
def test_td3_family_update_parity(case):
    cfg = CASES[case]
    kind, D, A, H, B, C = cfg["kind"], cfg["D"], cfg["A"], cfg["hidden"], cfg["B"], cfg["C"]
    rs = np.random.RandomState(12)
    stats = make_scaler_stats(rs, D) if cfg["scaler"] else None
    orc = make_td3_oracle(D, A, H, C=C, seed=4, scaler_stats=stats, kind=kind)
    impl = make_family_impl(kind, D, A, H, C, scaler_stats=stats)
    gen = torch.Generator().manual_seed(8)
    for step in range(4):
        impl.set_state_dict(td3_oracle_state(orc))
        arrs = make_td3_batch(rs, B, D, A)
        noise = torch.randn(B, A, generator=gen)
        actor = kind == "ddpg" or step % 2 == 0
        tb = Batch.from_numpy(*arrs)
        m_orc = {"critic_loss": float(orc.update_critic(tb, noise))}
        cg = _critic_grads(orc)
        if actor:
            m_orc["actor_loss"] = float(orc.update_actor(tb))
            pg = _policy_grads(orc)
            orc.update_critic_target()
            orc.update_actor_target()
        # DDPG draws no smoothing noise: run it on its own path (noise=None)
        m_hip = impl.update_step(HostBatch(*arrs), update_actor=actor,
                                 noise=None if kind == "ddpg" else noise.numpy())
        torch.cuda.synchronize()
        for k, v in m_orc.items():
            assert abs(m_hip[k] - v) <= 1e-5 * max(1.0, abs(v)), (step, k, m_hip[k], v)
        ge = 0.0
        for c in range(C):
            for l in range(impl.critic.n_layers):
                ge = max(ge, max_rel(impl.critic_grad(impl.critic.wname(l))[c], cg[c][l][0]),
                         max_rel(impl.critic_grad(impl.critic.bname(l))[c], cg[c][l][1]))
        pe = 0.0
        if actor:
            for l in range(impl.policy.n_layers):
                pe = max(pe, max_rel(impl.policy_grad(impl.policy.wname(l))[0], pg[l][0]),
                         max_rel(impl.policy_grad(impl.policy.bname(l))[0], pg[l][1]))
        sd, ref = impl.get_state_dict(), td3_oracle_state(orc)
        worst = max(float((sd[k][n] - t).abs().max())
                    for k in ("_q_func", "_targ_q_func", "_policy", "_targ_policy")
                    for n, t in ref[k].items())
        print(f"[{case}] step {step} actor={actor}: critic grad rel {ge:.2e}, policy grad rel "
              f"{pe:.2e}, param abs {worst:.2e}")
        assert ge <= 2e-5 and pe <= 2e-5, (ge, pe)
        assert worst <= 1e-5, worst


@pytest.mark.parametrize("algo_name", ["td3", "ddpg"])
def test_td3_family_fit_and_predict(algo_name):
    """Algo surface: fit() on a small synthetic dataset (device sampler,
    graph-replayed steps), reference metric keys, finite losses, predict /
    sample_action / predict_value shapes, checkpoint round trip."""
    from d3rlpy_amd.algos import get_algo
    from d3rlpy_amd.datasets import get_synthetic_d4rl
    ds = get_synthetic_d4rl("hopper-medium-v0", n=5000, seed=0)
    algo = get_algo(algo_name, discrete=False)(batch_size=64)
    hist = list(algo.fitter(ds, n_steps=40, n_steps_per_epoch=20, save_metrics=False))
    assert len(hist) == 2
    keys = set(hist[-1][1])
    assert {"critic_loss", "actor_loss"} <= keys, keys
    assert all(np.isfinite(v) for v in hist[-1][1].values())
    x = ds.observations[:7]
    a = algo.predict(x)
    assert a.shape == (7, 3) and np.all(np.abs(a) <= 1.0)
    assert np.array_equal(algo.sample_action(x), a)   # deterministic policy
    v = algo.predict_value(x, a)
    assert v.shape == (7,) and np.all(np.isfinite(v))
