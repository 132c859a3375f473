"""fp64 arbiters for TD3+BC (K1), BCQ (K3) and DiscreteCQL-IQN (K5), and the
BCQ full step without re-synchronisation (GPU only).

Each stage of an update (TD3+BC: critic, actor + targets; BCQ: imitator,
critic, actor + targets; DiscreteCQL: the single loss) starts the fp64 oracle
from the exact state HIP starts it from (HIP's get_state_dict, reference
layout), so the comparison isolates the arithmetic of that stage.  Bars and
the Adam first-step argument: tests/arbiter_helpers.py.  The fp32 oracle's
own distance from fp64 is printed next to HIP's for every gradient tensor.

Reference: algos/td3_plus_bc.py:101-119 + td3_plus_bc_impl.py:64-70 (K1 at
pendulum shapes, obs 3 / act 1 / B 100, standard scaler), algos/bcq.py:261-279
+ bcq_impl.py:101-226 (K3), algos/torch/cql_impl.py:279-302 +
dqn_impl.py:97-171 (K5 IQN).
"""
import numpy as np
import pytest
import torch

from arbiter_helpers import (adam_state_by_key, batch64, check_grads, check_params_adam,
                             check_params_adam1, hip_grads, load_state, module_grads, to_double)
from cql_helpers import HostBatch
from oracle.cql import Batch

pytestmark = pytest.mark.gpu


def _sd_params(sd, key, prefix=""):
    return {k[len(prefix):] if prefix else k: v for k, v in sd[key].items()}


# ---------------------------------------------------------------- TD3+BC (K1)
def test_td3bc_k1_stages_vs_fp64():
    from td3_helpers import (make_scaler_stats, make_td3_batch, make_td3_impl, make_td3_oracle,
                             td3_oracle_state)
    D, A, H, B = 3, 1, [256, 256], 100
    rs = np.random.RandomState(12)
    stats = make_scaler_stats(rs, D)
    o32 = make_td3_oracle(D, A, H, seed=21, scaler_stats=stats)
    o64 = make_td3_oracle(D, A, H, seed=21, scaler_stats=stats)
    to_double(o64, ("_q_func", "_targ_q_func", "_policy", "_targ_policy"))
    impl = make_td3_impl(D, A, H, scaler_stats=stats)
    impl.set_state_dict(td3_oracle_state(o32))
    arrs = make_td3_batch(rs, B, D, A)
    tb = Batch.from_numpy(*arrs)
    noise = torch.randn(B, A, generator=torch.Generator().manual_seed(4))
    # critic stage
    sd0 = impl.get_state_dict()
    for o in (o32, o64):
        load_state(o, sd0)
    o32.update_critic(tb, noise)
    o64.update_critic(batch64(tb), noise.double())
    m = impl.update_critic(HostBatch(*arrs), noise=noise.numpy())
    torch.cuda.synchronize()
    g_hip = hip_grads(impl._critic_refs(), impl.critic_grad)
    g64 = module_grads(o64._q_func)
    ge = check_grads("critic", g_hip, g64, module_grads(o32._q_func))
    sd1 = impl.get_state_dict()
    pw, namp = check_params_adam1("critic", _sd_params(sd0, "_q_func"), _sd_params(sd1, "_q_func"),
                                  dict(o64._q_func.state_dict()), g_hip, lr=3e-4)
    print(f"K1 critic: grad {ge:.1e}, param {pw:.1e} ({namp} amplified), loss {m}")
    # actor + targets stage, from HIP's post-critic state
    for o in (o32, o64):
        load_state(o, sd1)
    o32.update_actor(tb)
    o64.update_actor(batch64(tb))
    for o in (o32, o64):
        o.update_critic_target()
        o.update_actor_target()
    impl._run(HostBatch(*arrs), (False, True, True), None, True, False)
    torch.cuda.synchronize()
    g_hip = hip_grads(impl._policy_refs(), impl.policy_grad)
    ge = check_grads("policy", g_hip, module_grads(o64._policy), module_grads(o32._policy))
    sd2 = impl.get_state_dict()
    pw, namp = check_params_adam1("policy", _sd_params(sd1, "_policy"), _sd_params(sd2, "_policy"),
                                  dict(o64._policy.state_dict()), g_hip, lr=3e-4)
    # soft targets: three rounded ops, within fp32 rounding of fp64
    tw = max(float((sd2[k][n].double() - t.double()).abs().max())
             for k in ("_targ_q_func", "_targ_policy")
             for n, t in getattr(o64, k).state_dict().items())
    print(f"K1 actor: grad {ge:.1e}, param {pw:.1e} ({namp} amplified), targets {tw:.1e}")
    assert tw <= 1e-6


# ------------------------------------------------------------------- BCQ (K3)
def _bcq(seed=3):
    from oracle.bcq import BCQOracle
    from test_gpu_bcq_parity import make_bcq_impl, oracle_state
    D, A, H, N, K = 17, 6, [256, 256], 100, 200
    o32 = BCQOracle(D, A, n_action_samples=N, n_quantiles=K, hidden_units=H, seed=seed)
    o64 = BCQOracle(D, A, n_action_samples=N, n_quantiles=K, hidden_units=H, seed=seed)
    to_double(o64, ("_imitator", "_q_func", "_policy", "_targ_q_func", "_targ_policy"))
    impl = make_bcq_impl(D, A, H, N, K)
    impl.set_state_dict(oracle_state(o32))
    return impl, o32, o64, (D, A, N)


def _bcq_draws(B, A, N, seed):
    from oracle.bcq import BCQNoise
    nz = BCQNoise.draw(torch.Generator().manual_seed(seed), B, A, N)
    nz64 = BCQNoise(*(getattr(nz, f).double() for f in ("eps_vae", "z_target", "z_actor")))
    host = {k: getattr(nz, k).numpy() for k in ("eps_vae", "z_target", "z_actor")}
    return nz, nz64, host


def test_bcq_k3_stages_vs_fp64():
    from test_gpu_bcq_parity import _batch
    from oracle.models import soft_sync
    B = 256
    impl, o32, o64, (D, A, N) = _bcq()
    arrs = _batch(np.random.RandomState(7), B, D, A)
    tb, hb = Batch.from_numpy(*arrs), HostBatch(*arrs)
    nz, nz64, host = _bcq_draws(B, A, N, 8)
    stages = [
        ("imitator", (True, False, False, False), "_imitator", impl._imitator_refs,
         impl.imitator_grad, lambda o, b, n: o.update_imitator(b, n.eps_vae)),
        ("critic", (False, True, False, False), "_q_func", impl._critic_refs, impl.critic_grad,
         lambda o, b, n: o.update_critic(b, n.z_target)),
        ("actor", (False, False, True, True), "_policy", impl._policy_refs, impl.policy_grad,
         lambda o, b, n: (o.update_actor(b, n.z_actor),
                          soft_sync(o._targ_policy, o._policy, o._tau),
                          soft_sync(o._targ_q_func, o._q_func, o._tau))),
    ]
    for name, flags, key, refs, getter, run in stages:
        sd0 = impl.get_state_dict()
        for o in (o32, o64):
            load_state(o, sd0)
        run(o32, tb, nz)
        run(o64, batch64(tb), nz64)
        impl._run(hb, flags, host, True, False)
        torch.cuda.synchronize()
        g_hip = hip_grads(refs(), getter)
        ge = check_grads(name, g_hip, module_grads(getattr(o64, key)),
                         module_grads(getattr(o32, key)))
        sd1 = impl.get_state_dict()
        pw, namp = check_params_adam1(name, _sd_params(sd0, key), _sd_params(sd1, key),
                                      dict(getattr(o64, key).state_dict()), g_hip, lr=1e-3)
        print(f"K3 {name}: grad {ge:.1e}, param {pw:.1e} ({namp} amplified)")


def test_bcq_k3_full_step_vs_oracle():
    """One whole BCQ._update (update_step: one pipeline, no re-sync between
    stages) against the fp32 oracle's whole update from the same state.
    Later stages see parameters that differ by the earlier stages' Adam
    amplification (arbiter_helpers), so the stage gradients are compared at
    the bar the K3 arbiter measures for fp32-vs-fp32 (2e-5) and the
    parameters entry by entry through the Adam first-step argument."""
    from test_gpu_bcq_parity import _batch
    B = 256
    impl, o32, _, (D, A, N) = _bcq(seed=9)
    arrs = _batch(np.random.RandomState(10), B, D, A)
    nz, _, host = _bcq_draws(B, A, N, 11)
    sd0 = impl.get_state_dict()
    # the oracle's whole update (BCQOracle.update) with each stage's gradients
    # captured when its optimiser steps: the reference's later stages add
    # their backward into earlier modules' .grad (update_actor backpropagates
    # into the critic and the VAE decoder without zeroing them), so .grad
    # after the whole update is not what each optimiser consumed
    from oracle.models import soft_sync
    tb = Batch.from_numpy(*arrs)
    m_orc = {"imitator_loss": float(o32.update_imitator(tb, nz.eps_vae))}
    g_orc = {"_imitator": module_grads(o32._imitator)}
    m_orc["critic_loss"] = float(o32.update_critic(tb, nz.z_target))
    g_orc["_q_func"] = module_grads(o32._q_func)
    m_orc["actor_loss"] = float(o32.update_actor(tb, nz.z_actor))
    g_orc["_policy"] = module_grads(o32._policy)
    soft_sync(o32._targ_policy, o32._policy, o32._tau)
    soft_sync(o32._targ_q_func, o32._q_func, o32._tau)
    m_hip = impl.update_step(HostBatch(*arrs), noise=host)
    torch.cuda.synchronize()
    for k, v in m_orc.items():
        assert abs(m_hip[k] - v) <= 1e-5 * max(1.0, abs(v)), (k, m_hip[k], v)
    sd1 = impl.get_state_dict()
    for key, refs, getter in (("_imitator", impl._imitator_refs, impl.imitator_grad),
                              ("_q_func", impl._critic_refs, impl.critic_grad),
                              ("_policy", impl._policy_refs, impl.policy_grad)):
        g_hip = hip_grads(refs(), getter)
        ge = check_grads(key, g_hip, g_orc[key], tol=2e-5)
        pw, namp = check_params_adam1(key, _sd_params(sd0, key), _sd_params(sd1, key),
                                      dict(getattr(o32, key).state_dict()), g_hip, lr=1e-3)
        print(f"K3 full step {key}: grad {ge:.1e}, param {pw:.1e} ({namp} amplified)")
    tw = max(float((sd1[k][n] - t).abs().max()) for k in ("_targ_q_func", "_targ_policy")
             for n, t in getattr(o32, k).state_dict().items())
    print(f"K3 full step targets {tw:.1e}; metrics {m_hip}")
    assert tw <= 1e-5


# ---------------------------------------------------- DiscreteCQL-IQN (K5)
def _dcql_batch(rs, B, A):
    from oracle.discrete_cql import PixelBatch
    from test_gpu_discrete_cql import _HB, _batch
    obs, act, rew, nobs, term, nst = _batch(rs, B, A)
    pb = PixelBatch(torch.from_numpy(obs), torch.from_numpy(act).long(),
                    torch.from_numpy(rew).view(-1, 1), torch.from_numpy(nobs),
                    torch.from_numpy(term).view(-1, 1), torch.from_numpy(nst).view(-1, 1))
    return pb, _HB(obs, act, rew, nobs, term, nst)


def _force_conv_masks(o64, obs64, masks):
    """Make o64's online PixelEncoder use HIP's ReLU decisions (masks[l],
    (B, co, oh, ow)) on the batch's observations ``obs64`` — the pass whose
    gradients the update takes — and record each layer's fp64 pre-activation
    z and its rounding scale sum_k |w_k x_k| + |b| for the tie check."""
    import types
    enc = o64._q_func._encoder
    enc._ties = []

    def conv_encode(self, x):
        forced = x.shape == obs64.shape and torch.equal(x, obs64)
        h = x
        for l, conv in enumerate(self._convs):
            z = conv(h)
            if forced:
                with torch.no_grad():
                    scale = torch.nn.functional.conv2d(h.abs(), conv.weight.abs(),
                                                       conv.bias.abs(), stride=conv.stride)
                self._ties.append((z.detach(), scale))
                h = z * masks[l]
            else:
                h = torch.relu(z)
        return h
    enc._conv_encode = types.MethodType(conv_encode, enc)
    return enc


def _hip_conv_masks(impl, B):
    """HIP's ReLU decisions of the online encoder over the batch's
    observations (the first B samples of its [obs; next_obs] pass; NHWC)."""
    ws = impl._workspace(B)
    out = []
    for (ci, h, w, co, k, s, oh, ow), y in zip(impl.geom, ws.enc.ys):
        m = y[:B * oh * ow].view(B, oh, ow, co).permute(0, 3, 1, 2) > 0
        out.append(m.double().cpu())
    return out


def test_dcql_k5_b512_parity(monkeypatch):
    """The full K5 batch (B = 512 selects other conv / GEMM variants than the
    B = 16 / 64 cases): two consecutive updates, each started from the fp32
    oracle's state, against the fp32 oracle and against an fp64 arbiter.

    At B = 512 the online encoder makes 6.5 M conv0 ReLU decisions per
    update; a few pre-activations lie within fp32 rounding of zero, and where
    HIP and an oracle round such a tie differently the whole position's
    contribution moves into or out of the conv weight gradient (measured:
    one step at 4e-3 max-normalised on conv0).  So the arbiter evaluates the
    update in fp64 with HIP's own ReLU decisions on the observation pass and
    requires (1) HIP's gradients within 1e-5 of that, and (2) every decision
    where HIP differs from the exact fp64 sign to be a tie: |z| <= 2e-5 of
    the rounding scale sum_k |w_k x_k| + |b|."""
    import oracle.discrete_cql as odc
    from oracle.discrete_cql import DiscreteCQLIQNOracle, IQNTaus
    from test_gpu_discrete_cql import OBS, TAU_KEYS, make_impl, oracle_state
    monkeypatch.setattr(odc, "compute_iqn_feature", _prior_fp32_feature(odc.compute_iqn_feature))
    A, K, B = 4, 64, 512
    torch.set_num_threads(16)
    orc = DiscreteCQLIQNOracle(OBS, A, seed=6)
    impl = make_impl(A)
    rs = np.random.RandomState(13)
    gen = torch.Generator().manual_seed(14)
    pre = "_q_funcs.0."
    for step in range(2):
        sd = {k: {n: t.clone() for n, t in v.items()} if k != "_optim" else v
              for k, v in oracle_state(orc).items()}
        impl.set_state_dict(sd)
        sd0 = impl.get_state_dict()
        (pb, hb), taus = _dcql_batch(rs, B, A), IQNTaus.draw(gen, B, K)
        o64 = DiscreteCQLIQNOracle(OBS, A, seed=6)
        to_double(o64, ("_q_func", "_targ_q_func"))
        o64._scale = lambda x: x.double() / 255.0
        o64._q_func.load_state_dict({k[len(pre):]: v for k, v in sd["_q_func"].items()})
        o64._targ_q_func.load_state_dict({k[len(pre):]: v for k, v in sd["_targ_q_func"].items()})
        lo = orc.update(pb, taus)
        g32 = {pre + k: v for k, v in module_grads(orc._q_func).items()}
        m = impl.update_step(hb, taus={k: getattr(taus, k).numpy() for k in TAU_KEYS})
        torch.cuda.synchronize()
        assert abs(m["loss"] - lo) <= 1e-5 * max(1.0, abs(lo)), (step, m, lo)
        g_hip = hip_grads(impl._refs(), impl.grad)
        masks = _hip_conv_masks(impl, B)
        enc = _force_conv_masks(o64, pb.observations.double() / 255.0, masks)
        taus64 = IQNTaus(*(getattr(taus, f).double() for f in taus.__dataclass_fields__))
        pb64 = type(pb)(pb.observations, pb.actions, pb.rewards.double(), pb.next_observations,
                        pb.terminals.double(), pb.n_steps.double())
        l64 = o64.update(pb64, taus64)
        assert abs(m["loss"] - l64) <= 1e-5 * max(1.0, abs(l64)), (step, m, l64)
        g64 = {pre + k: v for k, v in module_grads(o64._q_func).items()}
        ge = check_grads(f"step {step}", g_hip, g64, g32)
        # the ReLU decisions where HIP differs from the exact sign are ties
        flips, worst = 0, 0.0
        for l, (z, scale) in enumerate(enc._ties[:len(masks)]):
            diff = (z > 0).double() != masks[l]
            if bool(diff.any()):
                r = float((z.abs() / scale)[diff].max())
                flips += int(diff.sum())
                worst = max(worst, r)
                print(f"  step {step} conv{l}: {int(diff.sum())} of {z.numel()} ReLU decisions "
                      f"differ from fp64, max |z| / scale {r:.1e}")
        assert worst <= 2e-5, worst
        sd1 = impl.get_state_dict()
        ref = oracle_state(orc)["_q_func"]
        if step == 0:  # Adam's first step: amplified entries are proven, not bounded
            pw, namp = check_params_adam1("dcql", sd0["_q_func"], sd1["_q_func"], ref, g_hip,
                                          lr=6.25e-5)
        else:
            # later steps: 1e-5 of the oracle, or -- entry by entry -- Adam from
            # the loaded optimiser state applied to HIP's own checked gradient
            states = adam_state_by_key(sd0["_optim"], [r[0] for r in impl._refs()])
            assert states, "step 1 must start from a non-empty Adam state"
            pw, namp = check_params_adam("dcql", sd0["_q_func"], sd1["_q_func"], ref, g_hip,
                                         lr=6.25e-5, states=states)
        print(f"K5 B=512 step {step}: loss {m['loss']:.6f} vs {lo:.6f} (fp64 {l64:.6f}), grad "
              f"vs fp64-with-HIP-masks {ge:.1e}, {flips} tie flips, param vs oracle {pw:.1e} "
              f"({namp} amplified)")


def _prior_fp32_feature(orig):
    """compute_iqn_feature (iqn_q_function.py:33-47) whose cosine prior is
    evaluated in fp32 — the reference's own precision for that elementwise
    input (arange().float(), math.pi * steps * taus, cos) — also when the
    network runs in fp64.  With an fp64 prior, cos(pi * i * tau) at
    arguments up to ~200 differs from the fp32 prior by ~1e-5 absolute, a
    difference both fp32 implementations share bit for bit (it is the
    reference's definition, not evaluation error)."""
    import math

    def feat(h, taus, embed, embed_size):
        if h.dtype != torch.float64:
            return orig(h, taus, embed, embed_size)
        steps = torch.arange(embed_size, device=h.device).float() + 1
        prior = torch.cos(math.pi * steps.view(1, 1, -1) * taus.float().view(h.shape[0], -1, 1))
        phi = torch.relu(embed(prior.double()))
        return h.view(h.shape[0], 1, -1) * phi
    return feat


def test_dcql_k5_vs_fp64(monkeypatch):
    import oracle.discrete_cql as odc
    from oracle.discrete_cql import DiscreteCQLIQNOracle, IQNTaus
    monkeypatch.setattr(odc, "compute_iqn_feature", _prior_fp32_feature(odc.compute_iqn_feature))
    from test_gpu_discrete_cql import OBS, TAU_KEYS, make_impl, oracle_state
    A, K, B = 4, 64, 128
    torch.set_num_threads(16)
    o32 = DiscreteCQLIQNOracle(OBS, A, seed=15)
    o64 = DiscreteCQLIQNOracle(OBS, A, seed=15)
    to_double(o64, ("_q_func", "_targ_q_func"))
    o64._scale = lambda x: x.double() / 255.0  # PixelScaler.transform in fp64
    impl = make_impl(A)
    impl.set_state_dict(oracle_state(o32))
    sd0 = impl.get_state_dict()
    pb, hb = _dcql_batch(np.random.RandomState(16), B, A)
    taus = IQNTaus.draw(torch.Generator().manual_seed(17), B, K)
    taus64 = IQNTaus(*(getattr(taus, f).double() for f in taus.__dataclass_fields__))
    pb64 = type(pb)(pb.observations, pb.actions, pb.rewards.double(), pb.next_observations,
                    pb.terminals.double(), pb.n_steps.double())
    o32.update(pb, taus)
    l64 = o64.update(pb64, taus64)
    m = impl.update_step(hb, taus={k: getattr(taus, k).numpy() for k in TAU_KEYS})
    torch.cuda.synchronize()
    assert abs(m["loss"] - l64) <= 1e-5 * max(1.0, abs(l64)), (m, l64)
    pre = "_q_funcs.0."
    g_hip = hip_grads(impl._refs(), impl.grad)
    ge = check_grads("dcql", g_hip, {pre + k: v for k, v in module_grads(o64._q_func).items()},
                     {pre + k: v for k, v in module_grads(o32._q_func).items()})
    sd1 = impl.get_state_dict()
    pw, namp = check_params_adam1("dcql", sd0["_q_func"], sd1["_q_func"],
                                  {pre + k: v for k, v in o64._q_func.state_dict().items()},
                                  g_hip, lr=6.25e-5)
    print(f"K5 vs fp64: loss {m['loss']:.8f} vs {l64:.8f}, grad {ge:.1e}, param {pw:.1e} "
          f"({namp} amplified)")
