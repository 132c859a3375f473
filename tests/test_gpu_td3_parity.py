"""TD3+BC update parity: HIP TD3PlusBCImpl vs the CPU oracle restatement (GPU only).

Same initial state (loaded through the reference checkpoint layout), same
minibatch, same injected target-smoothing noise; consecutive TD3PlusBC._update
steps with the delayed actor (update_actor_interval=2: actor + soft targets at
grad_step 0, 2, ...).  Compared after every step: critic_loss / actor_loss,
the reduced critic and policy gradients, post-Adam parameters and targets.

Tolerances (fp32, 1e-5 target of BASELINE.json north_star):
  losses      |a-b| <= 1e-5 * max(1, |b|)
  gradients   max|a-b| / max|b| <= 2e-5 per tensor (two fp32 summation orders)
  parameters  |a-b| <= 1e-5 absolute (targets included)
"""
import copy
import numpy as np
import pytest
import torch

from cql_helpers import HostBatch, max_rel
from oracle.cql import Batch
from td3_helpers import (make_scaler_stats, make_td3_batch, make_td3_impl, make_td3_oracle,
                         td3_oracle_state)

pytestmark = pytest.mark.gpu

CASES = {
    # K1 = configs[0]: pendulum-random shapes, batch 100, standard scaler
    # (td3_plus_bc.py:101-119); steps 0 and 2 include the delayed actor
    "k1_pendulum": dict(D=3, A=1, hidden=[256, 256], B=100, scaler=True, n_steps=1),
    "small_scaled": dict(D=5, A=2, hidden=[64, 64], B=32, scaler=True, n_steps=1),
    "hopper_scaled": dict(D=11, A=3, hidden=[256, 256], B=256, scaler=True, n_steps=1),
    "halfcheetah_nstep": dict(D=17, A=6, hidden=[256, 256], B=256, scaler=True, n_steps=3),
    "deep_unscaled": dict(D=7, A=2, hidden=[128, 128, 128], B=64, scaler=False, n_steps=1),
}


def _critic_grads(orc):
    return [[(fc.weight.grad.clone(), fc.bias.grad.clone())
             for fc in list(qf._encoder._fcs) + [qf._fc]] for qf in orc._q_func.q_funcs]


def _policy_grads(orc):
    pol = orc._policy
    return ([(fc.weight.grad.clone(), fc.bias.grad.clone()) for fc in pol._encoder._fcs]
            + [(pol._fc.weight.grad.clone(), pol._fc.bias.grad.clone())])


def _check_state(impl, orc, tol=1e-5):
    sd = impl.get_state_dict()
    ref = td3_oracle_state(orc)
    worst = 0.0
    for key in ("_q_func", "_targ_q_func", "_policy", "_targ_policy"):
        for name, t in ref[key].items():
            worst = max(worst, float((sd[key][name] - t).abs().max()))
    assert worst <= tol, worst
    return worst


@pytest.mark.parametrize("case", list(CASES))
def test_td3bc_update_parity(case):
    cfg = CASES[case]
    D, A, H, B = cfg["D"], cfg["A"], cfg["hidden"], cfg["B"]
    rs = np.random.RandomState(2)
    stats = make_scaler_stats(rs, D) if cfg["scaler"] else None
    orc = make_td3_oracle(D, A, H, seed=7, scaler_stats=stats)
    impl = make_td3_impl(D, A, H, scaler_stats=stats)
    gen = torch.Generator().manual_seed(3)
    for step in range(4):
        impl.set_state_dict(td3_oracle_state(orc))
        arrs = make_td3_batch(rs, B, D, A, cfg["n_steps"])
        noise = torch.randn(B, A, generator=gen)
        actor = step % 2 == 0
        tb = Batch.from_numpy(*arrs)
        m_orc = {"critic_loss": float(orc.update_critic(tb, noise))}
        cg = _critic_grads(orc)
        if actor:
            m_orc["actor_loss"] = float(orc.update_actor(tb))
            pg = _policy_grads(orc)
            orc.update_critic_target()
            orc.update_actor_target()
        m_hip = impl.update_step(HostBatch(*arrs), update_actor=actor, noise=noise.numpy())
        torch.cuda.synchronize()
        for k, v in m_orc.items():
            assert abs(m_hip[k] - v) <= 1e-5 * max(1.0, abs(v)), (step, k, m_hip[k], v)
        if not actor:
            assert np.isnan(m_hip["actor_loss"])
        ge = 0.0
        for c in range(impl._n_critics):
            for l in range(impl.critic.n_layers):
                ge = max(ge, max_rel(impl.critic_grad(impl.critic.wname(l))[c], cg[c][l][0]),
                         max_rel(impl.critic_grad(impl.critic.bname(l))[c], cg[c][l][1]))
        pe = 0.0
        if actor:
            for l in range(impl.policy.n_layers):
                pe = max(pe, max_rel(impl.policy_grad(impl.policy.wname(l))[0], pg[l][0]),
                         max_rel(impl.policy_grad(impl.policy.bname(l))[0], pg[l][1]))
        worst = _check_state(impl, orc)
        print(f"[{case}] step {step} actor={actor}: critic grad rel {ge:.2e}, "
              f"policy grad rel {pe:.2e}, param abs {worst:.2e}")
        assert ge <= 2e-5 and pe <= 2e-5, (ge, pe)


def test_td3bc_trajectory_drift():
    """Eight consecutive updates without re-synchronisation (K1 shapes)."""
    D, A, H, B = 17, 6, [256, 256], 256
    rs = np.random.RandomState(4)
    stats = make_scaler_stats(rs, D)
    orc = make_td3_oracle(D, A, H, seed=1, scaler_stats=stats)
    impl = make_td3_impl(D, A, H, scaler_stats=stats)
    impl.set_state_dict(td3_oracle_state(orc))
    gen = torch.Generator().manual_seed(5)
    for step in range(8):
        arrs = make_td3_batch(rs, B, D, A)
        noise = torch.randn(B, A, generator=gen)
        m_orc = orc.update(Batch.from_numpy(*arrs), noise, grad_step=step)
        m_hip = impl.update_step(HostBatch(*arrs), update_actor=step % 2 == 0,
                                 noise=noise.numpy())
        for k, v in m_orc.items():
            assert abs(m_hip[k] - v) <= 1e-4 * max(1.0, abs(v)), (step, k, m_hip[k], v)
    w = _check_state(impl, orc, tol=1e-4)
    print(f"td3bc trajectory drift after 8 steps: {w:.2e}")


def test_td3bc_graph_replay_matches_eager():
    D, A, H, B = 17, 6, [256, 256], 256
    rs = np.random.RandomState(6)
    stats = make_scaler_stats(rs, D)
    impl_a = make_td3_impl(D, A, H, scaler_stats=stats)
    impl_b = make_td3_impl(D, A, H, scaler_stats=stats)
    impl_b.store.data.copy_(impl_a.store.data)
    impl_b.targ.data.copy_(impl_a.targ.data)
    arrs = make_td3_batch(rs, B, D, A)
    for impl in (impl_a, impl_b):
        impl._workspace(B).seed = 99
    for it in range(6):
        actor = it % 2 == 0
        ma = impl_a.update_step(HostBatch(*arrs), update_actor=actor, use_graph=False)
        mb = impl_b.update_step(HostBatch(*arrs), update_actor=actor, use_graph=True)
        assert np.array_equal(np.array(list(ma.values())), np.array(list(mb.values())),
                              equal_nan=True), (it, ma, mb)
    torch.cuda.synchronize()
    assert torch.equal(impl_a.store.data, impl_b.store.data)
    assert torch.equal(impl_a.targ.data, impl_b.targ.data)
    assert len(impl_b._workspace(B)._graphs) == 2


def test_td3bc_checkpoint_roundtrip(tmp_path):
    D, A, H = 11, 3, [64, 64]
    orc = make_td3_oracle(D, A, H, seed=3)
    impl = make_td3_impl(D, A, H)
    rs = np.random.RandomState(1)
    impl.update_step(HostBatch(*make_td3_batch(rs, 32, D, A)), noise=np.zeros((32, A), np.float32))
    f = tmp_path / "td3.pt"
    impl.save_model(str(f))
    sd = torch.load(str(f), weights_only=True)
    assert set(sd) == set(td3_oracle_state(orc))
    for k in sd:
        getattr(orc, k).load_state_dict(copy.deepcopy(sd[k]))
    impl2 = make_td3_impl(D, A, H)
    impl2.load_model(str(f))
    assert torch.equal(impl2.store.data, impl.store.data)
    assert torch.equal(impl2.targ.data, impl.targ.data)
