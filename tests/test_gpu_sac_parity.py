"""SAC and CQL(soft_q_backup=True) update parity: HIP vs the CPU oracle (GPU only).

SAC._update (algos/sac.py:195-214) and the soft target of SACImpl.compute_target
(sac_impl.py:148-162), which CQL also uses with soft_q_backup=True
(cql_impl.py:225-230).  Same protocol and tolerances as test_gpu_cql_parity:
each step starts HIP from the oracle's exact state loaded through the
reference checkpoint layout; same batch, same injected noise (eps_targ is the
soft target's policy-sample noise).
"""
import numpy as np
import pytest
import torch

from cql_helpers import (HostBatch, make_batch, make_impl, make_oracle, make_sac_impl,
                         noise_dict, oracle_policy_grads, oracle_state)
from oracle.cql import Batch, CQLNoise, SACOracle
from test_gpu_cql_parity import _compare_step, _oracle_step

pytestmark = pytest.mark.gpu

CASES = {
    "small": dict(D=5, A=2, hidden=[64, 64], B=32),
    "hopper": dict(D=11, A=3, hidden=[256, 256], B=256),
}


def _sac_oracle_step(orc, tb, nz, A):
    m = {}
    tl, t = orc.update_temp(tb, nz.eps_temp)
    m.update(temp_loss=float(tl), temp=float(t))
    m["critic_loss"] = float(orc.update_critic(tb, nz))
    cgrads = [[(fc.weight.grad.clone(), fc.bias.grad.clone())
               for fc in list(qf._encoder._fcs) + [qf._fc]] for qf in orc._q_func.q_funcs]
    m["actor_loss"] = float(orc.update_actor(tb, nz.eps_actor))
    pgrads = oracle_policy_grads(orc._policy, A)
    orc.update_critic_target()
    orc.update_actor_target()
    return m, cgrads, pgrads


@pytest.mark.parametrize("case", list(CASES))
def test_sac_update_parity(case):
    cfg = CASES[case]
    D, A, H, B = cfg["D"], cfg["A"], cfg["hidden"], cfg["B"]
    orc = SACOracle(D, A, hidden_units=H, seed=13)
    impl = make_sac_impl(D, A, H)
    rs = np.random.RandomState(3)
    gen = torch.Generator().manual_seed(3)
    for step in range(3):
        impl.set_state_dict(oracle_state(orc))
        arrs = make_batch(rs, B, D, A)
        nz = CQLNoise.draw(gen, B, A, 0, soft_target=True)
        m_orc, cgrads, pgrads = _sac_oracle_step(orc, Batch.from_numpy(*arrs), nz, A)
        m_hip = impl.update_step(HostBatch(*arrs), noise=noise_dict(nz))
        torch.cuda.synchronize()
        assert set(impl.active_metric_names()) == set(m_orc)
        _compare_step("sac-" + case, step, impl, orc, m_hip, m_orc, cgrads, pgrads, A,
                      grad_tol=2e-5)


@pytest.mark.parametrize("case", list(CASES))
def test_cql_soft_q_backup_parity(case):
    cfg = CASES[case]
    D, A, H, B, N = cfg["D"], cfg["A"], cfg["hidden"], cfg["B"], 4
    orc = make_oracle(D, A, H, N, seed=17, soft_q_backup=True)
    impl = make_impl(D, A, H, N, soft_q_backup=True)
    rs = np.random.RandomState(4)
    gen = torch.Generator().manual_seed(4)
    for step in range(3):
        impl.set_state_dict(oracle_state(orc))
        arrs = make_batch(rs, B, D, A)
        nz = CQLNoise.draw(gen, B, A, N, soft_target=True)
        m_orc, cgrads, pgrads = _oracle_step(orc, Batch.from_numpy(*arrs), nz, A)
        m_hip = impl.update_step(HostBatch(*arrs), noise=noise_dict(nz))
        torch.cuda.synchronize()
        _compare_step("cql-soft-" + case, step, impl, orc, m_hip, m_orc, cgrads, pgrads, A,
                      grad_tol=2e-5)


def test_sac_fit_and_predict():
    """SAC.fit on a synthetic dataset runs the graph-replayed pipeline: the
    reference's metric keys, finite values; predict / predict_value shapes."""
    from d3rlpy_amd.algos import get_algo
    from d3rlpy_amd.datasets import get_synthetic_d4rl
    ds = get_synthetic_d4rl("hopper-medium-v0", n=5000, seed=0)
    sac = get_algo("sac", discrete=False)(batch_size=64)
    hist = list(sac.fitter(ds, n_steps=40, n_steps_per_epoch=20, save_metrics=False))
    assert len(hist) == 2
    for _, m in hist:
        assert set(m) == {"temp_loss", "temp", "critic_loss", "actor_loss"}, set(m)
        assert all(np.isfinite(v) for v in m.values())
    x = ds.observations[:7]
    a = sac.predict(x)
    assert a.shape == (7, 3) and np.all(np.abs(a) <= 1.0)
    v = sac.predict_value(x, a)
    assert v.shape == (7,) and np.all(np.isfinite(v))
