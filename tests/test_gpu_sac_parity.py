"""SAC and CQL(soft_q_backup=True) update parity: HIP vs the CPU oracle (GPU only).

SAC._update (algos/sac.py:195-214) and the soft target of SACImpl.compute_target
(sac_impl.py:148-162), which CQL also uses with soft_q_backup=True
(cql_impl.py:225-230).  Same protocol and tolerances as test_gpu_cql_parity:
each step starts HIP from the oracle's exact state loaded through the
reference checkpoint layout; same batch, same injected noise (eps_targ is the
soft target's policy-sample noise).
"""
import copy

import numpy as np
import pytest
import torch

from cql_helpers import (HostBatch, make_batch, make_impl, make_oracle, make_sac_impl, max_rel,
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
        sd0 = copy.deepcopy(oracle_state(orc))
        impl.set_state_dict(sd0)
        arrs = make_batch(rs, B, D, A)
        nz = CQLNoise.draw(gen, B, A, 0, soft_target=True)
        m_orc, cgrads, pgrads = _sac_oracle_step(orc, Batch.from_numpy(*arrs), nz, A)
        m_hip = impl.update_step(HostBatch(*arrs), noise=noise_dict(nz))
        torch.cuda.synchronize()
        assert set(impl.active_metric_names()) == set(m_orc)
        _compare_step("sac-" + case, step, impl, orc, m_hip, m_orc, cgrads, pgrads, A,
                      grad_tol=2e-5, sd0=sd0)


@pytest.mark.parametrize("case", list(CASES))
def test_cql_soft_q_backup_parity(case):
    cfg = CASES[case]
    D, A, H, B, N = cfg["D"], cfg["A"], cfg["hidden"], cfg["B"], 4
    orc = make_oracle(D, A, H, N, seed=17, soft_q_backup=True)
    impl = make_impl(D, A, H, N, soft_q_backup=True)
    rs = np.random.RandomState(4)
    gen = torch.Generator().manual_seed(4)
    for step in range(3):
        sd0 = copy.deepcopy(oracle_state(orc))
        impl.set_state_dict(sd0)
        arrs = make_batch(rs, B, D, A)
        nz = CQLNoise.draw(gen, B, A, N, soft_target=True)
        m_orc, cgrads, pgrads = _oracle_step(orc, Batch.from_numpy(*arrs), nz, A)
        m_hip = impl.update_step(HostBatch(*arrs), noise=noise_dict(nz))
        torch.cuda.synchronize()
        _compare_step("cql-soft-" + case, step, impl, orc, m_hip, m_orc, cgrads, pgrads, A,
                      grad_tol=2e-5, sd0=sd0)


def test_cql_standard_scaler_parity():
    """CQL with scaler='standard': the HIP pipeline standardises the staged
    batch on device (d3a_standardize_f32); the oracle receives the batch
    transformed as TorchMiniBatch does (torch_utility.py:179-181).  Metrics
    within 1e-5 of the fp32 oracle; each gradient tensor within 1e-5 (max-
    normalised) of an fp64 evaluation of the same update, or no further from it
    than 3x the fp32 oracle's own distance (a critic's head-bias gradient is
    one sum of ~8k cancelling row terms: both fp32 paths land ~2-5e-5 from
    exact on it here, at an absolute error of ~1e-9)."""
    from d3rlpy_amd.preprocessing import StandardScaler
    from oracle.td3bc import StandardScalerT
    from cql_helpers import copy_oracle_to_impl, oracle_critic_params
    D, A, H, B, N = 11, 3, [256, 256], 256, 10
    rs = np.random.RandomState(8)
    # statistics of the data below (obs ~ 3 N(0,1) + 1), slightly off as a
    # fitted scaler's would be
    mean = (1.0 + 0.1 * rs.randn(D)).astype(np.float32)
    std = (3.0 * (1.0 + 0.1 * rs.rand(D))).astype(np.float32)
    orc = make_oracle(D, A, H, N, seed=19)
    o64 = make_oracle(D, A, H, N, seed=19)
    for m in (o64._q_func, o64._policy, o64._targ_q_func, o64._targ_policy, o64._log_temp,
              o64._log_alpha):
        m.double()
    impl = make_impl(D, A, H, N, scaler=StandardScaler(mean=mean, std=std))
    copy_oracle_to_impl(orc, impl)
    sc = StandardScalerT(mean, std)
    obs, act, rew, nobs, term, nst = make_batch(rs, B, D, A)
    obs, nobs = obs * 3 + 1, nobs * 3 + 1
    nz = CQLNoise.draw(torch.Generator().manual_seed(8), B, A, N)
    tb = Batch.from_numpy(sc.transform(torch.from_numpy(obs)).numpy(), act, rew,
                          sc.transform(torch.from_numpy(nobs)).numpy(), term, nst)
    tb64 = Batch(*(getattr(tb, f).double() for f in tb.__dataclass_fields__))
    nz64 = CQLNoise(**{k: v.double() for k, v in noise_dict(nz).items()})
    m32 = None
    grads = []
    for o, b, n in ((orc, tb, nz), (o64, tb64, nz64)):
        tl, t = o.update_temp(b, n.eps_temp)
        al, a = o.update_alpha(b, n)
        cl = o.update_critic(b, n)
        grads.append([[(fc.weight.grad.clone(), fc.bias.grad.clone())
                       for fc in list(qf._encoder._fcs) + [qf._fc]] for qf in o._q_func.q_funcs])
        actl = o.update_actor(b, n.eps_actor)
        grads[-1].append(oracle_policy_grads(o._policy, A))
        if m32 is None:
            m32 = dict(temp_loss=float(tl), temp=float(t), alpha_loss=float(al), alpha=float(a),
                       critic_loss=float(cl), actor_loss=float(actl))
    m_hip = impl.update_step(HostBatch(obs, act, rew, nobs, term, nst), noise=noise_dict(nz))
    torch.cuda.synchronize()
    for k, v in m32.items():
        assert abs(m_hip[k] - v) <= 1e-5 * max(1.0, abs(v)), (k, m_hip[k], v)
    for c in range(3):
        net = impl.critic if c < 2 else impl.policy
        for l in range(net.n_layers):
            for k, nm in enumerate((net.wname(l), net.bname(l))):
                g = impl.critic_grad(nm)[c] if c < 2 else impl.policy_grad(nm)[0]
                e_hip = max_rel(g, grads[1][c][l][k])
                e_orc = max_rel(grads[0][c][l][k], grads[1][c][l][k])
                print(f"[cql-scaler] {c} {nm}: hip-vs-fp64 {e_hip:.1e} oracle32-vs-fp64 "
                      f"{e_orc:.1e}")
                assert e_hip <= max(1e-5, 3 * e_orc), (c, nm, e_hip, e_orc)
    # post-Adam parameters against the fp32 oracle
    perr = 0.0
    for c in range(2):
        for (W, b), (Wo, bo) in zip([impl.critic.export_linear(l, c) for l in
                                     range(impl.critic.n_layers)], oracle_critic_params(orc, c)):
            perr = max(perr, float((W.cpu() - Wo).abs().max()), float((b.cpu() - bo).abs().max()))
    assert perr <= 1e-5, perr


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
