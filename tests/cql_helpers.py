"""Shared helpers for CQL parity tests: build oracle + HIP impl with equal weights."""
import numpy as np
import torch

from oracle.cql import Batch, CQLNoise, CQLOracle


def make_impl(D, A, hidden, N, C=2, **kw):
    from d3rlpy_amd.algos.cql_impl import CQLImpl
    from d3rlpy_amd.factories import AdamFactory, MeanQFunctionFactory, VectorEncoderFactory
    args = dict(actor_learning_rate=1e-4, critic_learning_rate=3e-4, temp_learning_rate=1e-4,
                alpha_learning_rate=1e-4, gamma=0.99, tau=0.005, initial_temperature=1.0,
                initial_alpha=1.0, alpha_threshold=10.0, conservative_weight=5.0,
                soft_q_backup=False, scaler=None)
    args.update(kw)
    impl = CQLImpl(
        observation_shape=(D,), action_size=A,
        actor_optim_factory=AdamFactory(), critic_optim_factory=AdamFactory(),
        temp_optim_factory=AdamFactory(), alpha_optim_factory=AdamFactory(),
        actor_encoder_factory=VectorEncoderFactory(hidden),
        critic_encoder_factory=VectorEncoderFactory(hidden),
        q_func_factory=MeanQFunctionFactory(), n_critics=C, n_action_samples=N,
        use_gpu=0, action_scaler=None, reward_scaler=None,
        **args)
    impl.build()
    return impl


def make_sac_impl(D, A, hidden, C=2, **kw):
    from d3rlpy_amd.algos.sac import SACImpl
    from d3rlpy_amd.factories import AdamFactory, MeanQFunctionFactory, VectorEncoderFactory
    args = dict(actor_learning_rate=3e-4, critic_learning_rate=3e-4, temp_learning_rate=3e-4,
                gamma=0.99, tau=0.005, initial_temperature=1.0)
    args.update(kw)
    impl = SACImpl(
        observation_shape=(D,), action_size=A,
        actor_optim_factory=AdamFactory(), critic_optim_factory=AdamFactory(),
        temp_optim_factory=AdamFactory(),
        actor_encoder_factory=VectorEncoderFactory(hidden),
        critic_encoder_factory=VectorEncoderFactory(hidden),
        q_func_factory=MeanQFunctionFactory(), n_critics=C, use_gpu=0, scaler=None,
        action_scaler=None, reward_scaler=None, **args)
    impl.build()
    return impl


def make_oracle(D, A, hidden, N, C=2, seed=0, **kw):
    return CQLOracle(D, A, n_critics=C, n_action_samples=N, hidden_units=hidden, seed=seed, **kw)


def copy_oracle_to_impl(orc: CQLOracle, impl) -> None:
    A = impl._action_size
    for c, qf in enumerate(orc._q_func.q_funcs):
        for l, fc in enumerate(qf._encoder._fcs):
            impl.critic.load_linear(l, c, fc)
        impl.critic.load_linear(len(qf._encoder._fcs), c, qf._fc)
    pol = orc._policy
    for l, fc in enumerate(pol._encoder._fcs):
        impl.policy.load_linear(l, 0, fc)
    L = len(pol._encoder._fcs)
    Wh, bh = impl.policy.export_linear(L, 0)
    with torch.no_grad():
        Wh[:A].copy_(pol._mu.weight)
        Wh[A:].copy_(pol._logstd.weight)
        bh[:A].copy_(pol._mu.bias)
        bh[A:].copy_(pol._logstd.bias)
        impl.targ.data.copy_(impl.store.data)
    # targets of the oracle equal the online nets at build (deepcopy)


def impl_critic_params(impl, c):
    """List of (W, b) per layer of critic c, in reference module order."""
    out = []
    for l in range(impl.critic.n_layers):
        W, b = impl.critic.export_linear(l, c)
        out.append((W.detach().cpu(), b.detach().cpu()))
    return out


def oracle_critic_params(orc, c, target=False):
    qf = (orc._targ_q_func if target else orc._q_func).q_funcs[c]
    layers = list(qf._encoder._fcs) + [qf._fc]
    return [(fc.weight.detach(), fc.bias.detach()) for fc in layers]


def oracle_policy_head(pol, A):
    layers = [(fc.weight.detach(), fc.bias.detach()) for fc in pol._encoder._fcs]
    W = torch.cat([pol._mu.weight.detach(), pol._logstd.weight.detach()], 0)
    b = torch.cat([pol._mu.bias.detach(), pol._logstd.bias.detach()], 0)
    return layers + [(W, b)]


def oracle_policy_grads(pol, A):
    layers = [(fc.weight.grad, fc.bias.grad) for fc in pol._encoder._fcs]
    W = torch.cat([pol._mu.weight.grad, pol._logstd.weight.grad], 0)
    b = torch.cat([pol._mu.bias.grad, pol._logstd.bias.grad], 0)
    return layers + [(W, b)]


def make_batch(rs: np.random.RandomState, B, D, A):
    obs = rs.randn(B, D).astype(np.float32)
    act = rs.uniform(-1, 1, size=(B, A)).astype(np.float32)
    rew = rs.randn(B).astype(np.float32)
    nobs = rs.randn(B, D).astype(np.float32)
    term = (rs.rand(B) < 0.1).astype(np.float32)
    nst = np.ones(B, dtype=np.float32)
    return obs, act, rew, nobs, term, nst


class HostBatch:
    """TransitionMiniBatch-like numpy container."""

    def __init__(self, obs, act, rew, nobs, term, nst):
        self.observations = obs
        self.actions = act
        self.rewards = rew.reshape(-1, 1)
        self.next_observations = nobs
        self.terminals = term.reshape(-1, 1)
        self.n_steps = nst.reshape(-1, 1)


def noise_dict(nz: CQLNoise):
    return nz.tensors()


def max_rel(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float((a - b).abs().max()) / max(1e-30, float(b.abs().max()))


ORACLE_STATE_KEYS = ("_q_func", "_targ_q_func", "_policy", "_targ_policy", "_log_temp",
                     "_log_alpha", "_critic_optim", "_actor_optim", "_temp_optim",
                     "_alpha_optim")


def oracle_state(orc):
    """torch_utility.get_state_dict(impl) of the oracle (reference attribute names)."""
    return {k: getattr(orc, k).state_dict() for k in ORACLE_STATE_KEYS}
