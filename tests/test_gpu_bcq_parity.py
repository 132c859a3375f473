"""BCQ update parity (K3: QR critics): HIP BCQImpl vs the CPU oracle (GPU only).

Same initial state (loaded through the reference checkpoint layout), same
minibatch, same injected draws (VAE rsample noise, the B*N target latents,
the actor latents).  Compared per stage: imitator / critic / actor losses,
the reduced gradients of the three optimisers, post-Adam parameters and
targets.  Tolerances: losses 1e-5 relative, gradients 2e-5 max-normalised
between the two fp32 implementations (HIP itself is within 1e-5 of fp64:
tests/test_gpu_arbiters.py), parameters 1e-5 absolute or proven Adam
amplification of a near-zero gradient entry (tests/arbiter_helpers.py).
"""
import copy
import numpy as np
import pytest
import torch

from cql_helpers import HostBatch, max_rel
from oracle.bcq import BCQNoise, BCQOracle
from oracle.cql import Batch

pytestmark = pytest.mark.gpu

STATE_KEYS = ("_q_func", "_targ_q_func", "_policy", "_targ_policy", "_imitator",
              "_critic_optim", "_actor_optim", "_imitator_optim")

CASES = {
    "small": dict(D=5, A=2, hidden=[64, 64], N=10, K=16, B=32),
    "k3": dict(D=17, A=6, hidden=[256, 256], N=100, K=200, B=256),  # halfcheetah shapes
}


def make_bcq_impl(D, A, hidden, N, K, C=2, scaler=None):
    from d3rlpy_amd.algos.bcq_impl import BCQImpl
    from d3rlpy_amd.factories import AdamFactory, QRQFunctionFactory, VectorEncoderFactory
    impl = BCQImpl(
        observation_shape=(D,), action_size=A, actor_learning_rate=1e-3,
        critic_learning_rate=1e-3, imitator_learning_rate=1e-3,
        actor_optim_factory=AdamFactory(), critic_optim_factory=AdamFactory(),
        imitator_optim_factory=AdamFactory(), actor_encoder_factory=VectorEncoderFactory(hidden),
        critic_encoder_factory=VectorEncoderFactory(hidden),
        imitator_encoder_factory=VectorEncoderFactory(hidden),
        q_func_factory=QRQFunctionFactory(n_quantiles=K), gamma=0.99, tau=0.005, n_critics=C,
        lam=0.75, n_action_samples=N, action_flexibility=0.05, beta=0.5, use_gpu=0,
        scaler=scaler, action_scaler=None, reward_scaler=None)
    impl.build()
    return impl


def oracle_state(orc):
    return {k: getattr(orc, k).state_dict() for k in STATE_KEYS}


def _batch(rs, B, D, A):
    return (rs.randn(B, D).astype(np.float32), rs.uniform(-1, 1, (B, A)).astype(np.float32),
            rs.randn(B).astype(np.float32), rs.randn(B, D).astype(np.float32),
            (rs.rand(B) < 0.1).astype(np.float32), np.ones(B, np.float32))


def _grads(modules):
    return [p.grad.clone() for m in modules for p in m.parameters()]


def _grad_err(impl, refs, ref_g, getter, name):
    e = 0.0
    for (key, seg, member, sl), g in zip(refs, ref_g):
        hip = getter(seg)[member]
        hip = hip if sl is None else hip[sl]
        ek = max_rel(hip, g)
        if ek > 2e-5:
            print(f"  {name} {key}: rel {ek:.2e}")
        e = max(e, ek)
    return e


def _param_check(label, impl, orc, key, optim_key, sd0, refs, getter):
    """Parameters of ``key`` after its stage: 1e-5 of the oracle, or proven
    Adam amplification of a near-zero gradient entry (arbiter_helpers)."""
    from arbiter_helpers import adam_state_by_key, check_params_adam, hip_grads
    sd = impl.get_state_dict()
    keys = [r[0] for r in refs]
    states = adam_state_by_key(sd0[optim_key], keys)
    w, n = check_params_adam(label, sd0[key], sd[key], oracle_state(orc)[key],
                             hip_grads(refs, getter), lr=1e-3, states=states or None)
    return w, n


@pytest.mark.parametrize("case", list(CASES))
def test_bcq_update_parity(case):
    """Stage by stage (update_imitator, update_critic, update_actor + targets),
    each HIP stage started from the oracle's exact state.  Adam's first steps
    move every parameter by ~lr whatever the gradient's size, so fp32
    rounding in near-zero gradient entries shows up as ~1e-5 parameter
    differences after a stage; re-synchronising between stages keeps each
    stage's comparison at the rounding level of that stage alone."""
    cfg = CASES[case]
    D, A, H, N, K, B = cfg["D"], cfg["A"], cfg["hidden"], cfg["N"], cfg["K"], cfg["B"]
    orc = BCQOracle(D, A, n_action_samples=N, n_quantiles=K, hidden_units=H, seed=3)
    impl = make_bcq_impl(D, A, H, N, K)
    rs = np.random.RandomState(0)
    gen = torch.Generator().manual_seed(1)
    from oracle.models import soft_sync
    for step in range(2):
        arrs = _batch(rs, B, D, A)
        nz = BCQNoise.draw(gen, B, A, N)
        noise = {k: getattr(nz, k).numpy() for k in ("eps_vae", "z_target", "z_actor")}
        tb = Batch.from_numpy(*arrs)
        hb = HostBatch(*arrs)
        # imitator
        impl.set_state_dict(oracle_state(orc))
        sd0 = impl.get_state_dict()
        lo = float(orc.update_imitator(tb, nz.eps_vae))
        ig = [p.grad.clone() for p in orc._imitator.parameters()]
        lh = impl._run(hb, (True, False, False, False), noise, True, False)["imitator_loss"]
        assert abs(lh - lo) <= 1e-5 * max(1.0, abs(lo)), (step, lh, lo)
        e_i = _grad_err(impl, impl._imitator_refs(), ig, impl.imitator_grad, "imitator")
        p_i, a_i = _param_check("imitator", impl, orc, "_imitator", "_imitator_optim", sd0,
                                impl._imitator_refs(), impl.imitator_grad)
        # critic
        impl.set_state_dict(oracle_state(orc))
        sd0 = impl.get_state_dict()
        lo = float(orc.update_critic(tb, nz.z_target))
        cg = [p.grad.clone() for p in orc._q_func.parameters()]
        lh = impl._run(hb, (False, True, False, False), noise, True, False)["critic_loss"]
        assert abs(lh - lo) <= 1e-5 * max(1.0, abs(lo)), (step, lh, lo)
        e_c = _grad_err(impl, impl._critic_refs(), cg, impl.critic_grad, "critic")
        p_c, a_c = _param_check("critic", impl, orc, "_q_func", "_critic_optim", sd0,
                                impl._critic_refs(), impl.critic_grad)
        # actor + targets
        impl.set_state_dict(oracle_state(orc))
        sd0 = impl.get_state_dict()
        lo = float(orc.update_actor(tb, nz.z_actor))
        pg = [p.grad.clone() for p in orc._policy.parameters()]
        soft_sync(orc._targ_policy, orc._policy, orc._tau)
        soft_sync(orc._targ_q_func, orc._q_func, orc._tau)
        m = impl._run(hb, (False, False, True, True), noise, True, False)
        assert abs(m["actor_loss"] - lo) <= 1e-5 * max(1.0, abs(lo)), (step, m, lo)
        e_p = _grad_err(impl, impl._policy_refs(), pg, impl.policy_grad, "policy")
        p_p, a_p = _param_check("policy", impl, orc, "_policy", "_actor_optim", sd0,
                                impl._policy_refs(), impl.policy_grad)
        sd = impl.get_state_dict()
        ref = oracle_state(orc)
        p_t = max(float((sd[k][n] - t).abs().max()) for k in ("_targ_policy", "_targ_q_func")
                  for n, t in ref[k].items())
        print(f"[{case}] step {step}: grad rel imitator {e_i:.1e} critic {e_c:.1e} policy "
              f"{e_p:.1e}; param abs {max(p_i, p_c, p_p):.1e} ({a_i + a_c + a_p} entries "
              f"proven Adam amplification), targets {p_t:.1e}")
        assert max(e_i, e_c, e_p) <= 2e-5
        # parameters: 1e-5 absolute, except entries where Adam amplifies a
        # near-zero gradient (lr * g / (|g| + eps) at BCQ's lr = 1e-3), each of
        # which is proven to be Adam applied to HIP's 2e-5-checked gradient
        assert p_t <= 1e-5


def test_bcq_full_step_equals_stages():
    """update_step (one pipeline / graph) == the three stages run one by one
    on the same state and draws (bit-identical: same kernels, same order)."""
    D, A, H, N, K, B = 17, 6, [256, 256], 100, 200, 256
    a = make_bcq_impl(D, A, H, N, K)
    b = make_bcq_impl(D, A, H, N, K)
    b.set_state_dict(a.get_state_dict())
    rs = np.random.RandomState(4)
    for step in range(2):
        arrs = _batch(rs, B, D, A)
        nz = BCQNoise.draw(torch.Generator().manual_seed(step), B, A, N)
        noise = {k: getattr(nz, k).numpy() for k in ("eps_vae", "z_target", "z_actor")}
        ma = a.update_step(HostBatch(*arrs), noise=noise)
        mi = b._run(HostBatch(*arrs), (True, False, False, False), noise, True, False)
        mc = b._run(HostBatch(*arrs), (False, True, False, False), noise, True, False)
        mp = b._run(HostBatch(*arrs), (False, False, True, True), noise, True, False)
        assert ma["imitator_loss"] == mi["imitator_loss"]
        assert ma["critic_loss"] == mp["critic_loss"] and ma["actor_loss"] == mp["actor_loss"]
        torch.cuda.synchronize()
        assert torch.equal(a.store.data, b.store.data)
        s0, s1 = a.soft_span
        assert torch.equal(a.targ.data[s0:s1], b.targ.data[s0:s1])
        # the full step's bookkeeping rides in its Adam launches (no step_end):
        # the same optimiser step counters as the staged runs' step_end
        assert torch.equal(a.counters[:3], b.counters[:3]), (a.counters, b.counters)


def test_bcq_standard_scaler_matches_prescaled_batch():
    """scaler='standard': the on-device transform (d3a_standardize_f32) of a
    raw batch gives bit-identical updates to an unscaled Impl fed the batch
    transformed by torch as TorchMiniBatch does (torch_utility.py:179-181):
    sub, add and div are correctly rounded either way."""
    from d3rlpy_amd.preprocessing import StandardScaler
    from oracle.td3bc import StandardScalerT
    D, A, H, N, K, B = 17, 6, [256, 256], 100, 200, 256
    rs = np.random.RandomState(6)
    mean = (1.0 + 0.1 * rs.randn(D)).astype(np.float32)
    std = (3.0 * (1.0 + 0.1 * rs.rand(D))).astype(np.float32)
    a = make_bcq_impl(D, A, H, N, K, scaler=StandardScaler(mean=mean, std=std))
    b = make_bcq_impl(D, A, H, N, K)
    b.set_state_dict(a.get_state_dict())
    sc = StandardScalerT(mean, std)
    for step in range(2):
        obs, act, rew, nobs, term, nst = _batch(rs, B, D, A)
        obs, nobs = obs * 3 + 1, nobs * 3 + 1
        nz = BCQNoise.draw(torch.Generator().manual_seed(step), B, A, N)
        noise = {k: getattr(nz, k).numpy() for k in ("eps_vae", "z_target", "z_actor")}
        ma = a.update_step(HostBatch(obs, act, rew, nobs, term, nst), noise=noise)
        mb = b.update_step(HostBatch(sc.transform(torch.from_numpy(obs)).numpy(), act, rew,
                                     sc.transform(torch.from_numpy(nobs)).numpy(), term, nst),
                           noise=noise)
        assert ma == mb, (step, ma, mb)
    torch.cuda.synchronize()
    assert torch.equal(a.store.data, b.store.data)


def test_bcq_graph_replay_matches_eager():
    D, A, H, N, K, B = 17, 6, [256, 256], 100, 200, 256
    a = make_bcq_impl(D, A, H, N, K)
    b = make_bcq_impl(D, A, H, N, K)
    b.set_state_dict(a.get_state_dict())
    for impl in (a, b):
        impl._workspace(B).seed = 5
    arrs = _batch(np.random.RandomState(2), B, D, A)
    for it in range(3):
        ma = a.update_step(HostBatch(*arrs), use_graph=False)
        mb = b.update_step(HostBatch(*arrs), use_graph=True)
        assert ma == mb, (it, ma, mb)
    torch.cuda.synchronize()
    assert torch.equal(a.store.data, b.store.data)
    s0, s1 = a.soft_span  # targets exist for the critic and policy only
    assert torch.equal(a.targ.data[s0:s1], b.targ.data[s0:s1])


def test_bcq_checkpoint_roundtrip(tmp_path):
    D, A, H, N, K = 5, 2, [64, 64], 10, 16
    orc = BCQOracle(D, A, n_action_samples=N, n_quantiles=K, hidden_units=H, seed=4)
    impl = make_bcq_impl(D, A, H, N, K)
    impl.update_step(HostBatch(*_batch(np.random.RandomState(3), 32, D, A)))
    f = tmp_path / "bcq.pt"
    impl.save_model(str(f))
    sd = torch.load(str(f), weights_only=True)
    assert set(sd) == set(STATE_KEYS)
    for k in sd:
        getattr(orc, k).load_state_dict(copy.deepcopy(sd[k]))
    impl2 = make_bcq_impl(D, A, H, N, K)
    impl2.load_model(str(f))
    assert torch.equal(impl2.store.data, impl.store.data)


def test_bcq_predict_best_action_shape():
    D, A, H, N, K = 5, 2, [64, 64], 10, 16
    impl = make_bcq_impl(D, A, H, N, K)
    a = impl.predict_best_action(np.random.RandomState(0).randn(7, D).astype(np.float32))
    assert a.shape == (7, A) and np.all(np.abs(a) <= 1.0)


@pytest.mark.parametrize("N,K", [(10, 200), (3, 7)])
def test_qr_loss_in_launch_target_is_bitwise_the_target_launch(N, K):
    """d3a_bcq_qr_loss with tg_* (the target rows formed in the loss launch
    from the target pass's quantiles and means) writes dq and loss_cb bitwise
    as d3a_bcq_target + d3a_bcq_qr_loss (bcq_impl.py:215-226 +
    qr_q_function.py:130-150), ties in the means included."""
    from d3rlpy_amd import _native as N_
    from d3rlpy_amd import ops
    dev = torch.device("cuda")
    B, C, lam, gamma = 64, 2, 0.75, 0.99
    g = torch.Generator().manual_seed(N * 100 + K)
    tq = torch.randn(C, B * N, K, generator=g).to(dev)
    tq[:, ::5] = tq[:, 1::5][:, : tq[:, ::5].shape[1]]  # repeated rows: tied means
    means = tq.mean(dim=2).contiguous()
    q = torch.randn(C, B, K, generator=g).to(dev)
    rew = torch.randn(B, generator=g).to(dev)
    term = (torch.rand(B, generator=g) < 0.2).float().to(dev)
    nst = torch.ones(B, device=dev)
    target = torch.zeros(B, K, device=dev)
    res = []
    for fused in (False, True):
        dq = torch.full((C, B, K), float("nan"), device=dev)
        loss = torch.full((C, B), float("nan"), device=dev)
        d = N_.BcqQrDesc()
        d.q, d.rew, d.term, d.n_steps = q.data_ptr(), rew.data_ptr(), term.data_ptr(), nst.data_ptr()
        d.dq, d.loss_cb, d.B, d.K, d.C, d.gamma = dq.data_ptr(), loss.data_ptr(), B, K, C, gamma
        if fused:
            d.target = None
            d.tg_q, d.tg_means, d.tg_N, d.tg_C, d.tg_lam = tq.data_ptr(), means.data_ptr(), N, C, lam
        else:
            t = N_.BcqTargetDesc()
            t.q, t.target, t.B, t.N, t.K, t.C, t.lam = tq.data_ptr(), target.data_ptr(), B, N, K, C, lam
            t.means = means.data_ptr()
            ops.call_desc("d3a_bcq_target", t)
            d.target = target.data_ptr()
        ops.call_desc("d3a_bcq_qr_loss", d)
        torch.cuda.synchronize()
        res.append((dq, loss))
    assert not torch.isnan(res[0][0]).any() and not torch.isnan(res[1][1]).any()
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1])


def test_bcq_philox_in_encoder_launch_is_bitwise_the_fill_launch(monkeypatch):
    """The step's Philox noise formed by extra workgroups of the VAE encoder's
    parts-path launch (d3a_mlp_fwd_desc.philox, round 6) against its own
    d3a_philox_fill launch: three graph-replayed K3 updates from one state and
    seed leave every parameter, target and the noise counter bitwise equal."""
    from d3rlpy_amd.algos import bcq_impl
    D, A, H, N, K, B = 17, 6, [256, 256], 100, 200, 256
    a = make_bcq_impl(D, A, H, N, K)
    b = make_bcq_impl(D, A, H, N, K)
    b.set_state_dict(a.get_state_dict())
    for impl, fused in ((a, True), (b, False)):
        monkeypatch.setattr(bcq_impl, "_PHILOX_IN_ENC", fused)
        impl._workspace(B).seed = 11
        rs = np.random.RandomState(6)
        for _ in range(3):
            impl.update_step(HostBatch(*_batch(rs, B, D, A)), use_graph=True)
        torch.cuda.synchronize()
    assert torch.equal(a.store.data, b.store.data)
    s0, s1 = a.soft_span
    assert torch.equal(a.targ.data[s0:s1], b.targ.data[s0:s1])
    wa, wb = a._workspace(B), b._workspace(B)
    assert torch.equal(wa.noise, wb.noise) and torch.equal(wa.rng_ctr, wb.rng_ctr)
    assert int(wa.rng_ctr.item()) == 3
