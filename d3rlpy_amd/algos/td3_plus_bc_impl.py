"""TD3PlusBCImpl on HIP kernels — drop-in for d3rlpy/algos/torch/td3_plus_bc_impl.py:19-70
(and what it inherits: TD3Impl td3_impl.py:18-78, DDPGBaseImpl ddpg_impl.py:30-227).

Same constructor arguments, same ``update_critic / update_actor /
update_critic_target / update_actor_target`` methods; plus ``update_step``
which runs one ``TD3PlusBC._update`` (algos/td3_plus_bc.py:177-192) — a critic
update every step, the actor and both soft target updates every
``update_actor_interval``-th step — as one device pipeline (a HIP-graph replay
after the first call).

Pipeline of one update_step (current stream, no host sync):
  1  d3a_td3_prep: standard-scale obs / next_obs (the reference's
     TorchMiniBatch scaler) straight into the Q-input rows
     x_q = (s, a) and x_targ = (s', .)
  2  target policy on x_targ[:, :D]; d3a_td3_target writes the smoothed,
     clipped target action into x_targ[:, D:]
  3  critic ensemble on x_q, target ensemble on x_targ; d3a_td3_critic_loss
  4  critic backward over the B rows, Adam (critic)
  -- actor steps only --
  5  policy on x_q[:, :D]; d3a_td3bc_actor_input builds x_actor = (s, pi(s))
  6  critic member 0 (the updated critic) on x_actor; d3a_td3bc_actor_seed
     (lam = alpha / mean|Q0|, dL/dQ0 = -lam/B); input gradient dQ0/dx
  7  d3a_td3bc_actor_head (adds the BC gradient, tanh backward); policy
     backward, Adam (actor)
  8  d3a_step_end: soft update of both targets + metric ring + step counters
"""
from __future__ import annotations

from typing import Dict, Optional, Sequence

import numpy as np
import torch
from torch import nn

from .. import _native as NAT
from .. import checkpoint as ckpt
from .. import mlp, ops
from ..nets import AdamGroup, EnsembleMLP, GradSpace, OptimState, ParamStore
from .impl_base import DeviceBatch, ImplBase, as_device_batch

METRIC_NAMES = ("critic_loss", "actor_loss")


class TD3PlusBCImpl(ImplBase):
    # behaviour-cloning actor loss (td3_plus_bc_impl.py:64-70); TD3Impl /
    # DDPGImpl (algos/td3.py) clear it for -mean Q_0 (ddpg_impl.py:244-249)
    _BC = True

    def __init__(
        self,
        observation_shape: Sequence[int],
        action_size: int,
        actor_learning_rate: float,
        critic_learning_rate: float,
        actor_optim_factory,
        critic_optim_factory,
        actor_encoder_factory,
        critic_encoder_factory,
        q_func_factory,
        gamma: float,
        tau: float,
        n_critics: int,
        target_smoothing_sigma: float,
        target_smoothing_clip: float,
        alpha: float,
        use_gpu,
        scaler,
        action_scaler,
        reward_scaler,
    ):
        super().__init__(observation_shape, action_size, scaler, action_scaler, reward_scaler,
                         use_gpu)
        if q_func_factory.get_type() != "mean":
            raise NotImplementedError(f"{self._name()} on HIP supports the 'mean' Q function")
        if len(observation_shape) != 1:
            raise NotImplementedError(f"{self._name()} on HIP supports vector observations")
        if scaler is not None and scaler.get_type() != "standard":
            raise NotImplementedError(f"{self._name()} on HIP supports the 'standard' scaler")
        if action_scaler is not None or reward_scaler is not None:
            raise NotImplementedError("action/reward scalers are out of scope (SURVEY §2 #4)")
        self._actor_learning_rate = actor_learning_rate
        self._critic_learning_rate = critic_learning_rate
        self._actor_optim_factory = actor_optim_factory
        self._critic_optim_factory = critic_optim_factory
        self._actor_encoder_factory = actor_encoder_factory
        self._critic_encoder_factory = critic_encoder_factory
        self._q_func_factory = q_func_factory
        self._gamma = gamma
        self._tau = tau
        self._n_critics = n_critics
        self._target_smoothing_sigma = target_smoothing_sigma
        self._target_smoothing_clip = target_smoothing_clip
        self._alpha = alpha
        self._ws: Dict[int, "_Workspace"] = {}

    @classmethod
    def _name(cls) -> str:
        return cls.__name__.replace("Impl", "")

    # ------------------------------------------------------------------ build
    def build(self) -> None:
        dev = self.torch_device
        D, A, C = self._observation_shape[0], self._action_size, self._n_critics
        hq = list(self._critic_encoder_factory.hidden_units)
        hp = list(self._actor_encoder_factory.hidden_units)
        store = ParamStore()
        # DDPGBaseImpl.build (ddpg_impl.py:95-111): critic, then actor
        self.critic = EnsembleMLP(store, "q", C, [D + A] + hq + [1])
        self.policy = EnsembleMLP(store, "pi", 1, [D] + hp + [A])
        store.allocate(dev)
        self.store = store
        self._init_like_reference()
        self.targ = store.like()
        self.targ.data.copy_(store.data)
        self.counters = torch.zeros(8, dtype=torch.int64, device=dev)  # [0] critic [1] actor
        f = self._critic_optim_factory
        self.critic_state = OptimState(store, self.critic.names(), self._critic_learning_rate,
                                       f.betas, f.eps, step=self.counters[0:1])
        f = self._actor_optim_factory
        self.actor_state = OptimState(store, self.policy.names(), self._actor_learning_rate,
                                      f.betas, f.eps, step=self.counters[1:2])
        if self._scaler is not None:
            if self._scaler.mean is None:
                raise ValueError("the standard scaler is not fitted (fit_dataset / fit)")
            D_ = self._observation_shape[0]
            self.scaler_mean = torch.as_tensor(np.asarray(self._scaler.mean).reshape(D_),
                                               dtype=torch.float32).to(dev)
            self.scaler_std = torch.as_tensor(np.asarray(self._scaler.std).reshape(D_),
                                              dtype=torch.float32).to(dev)
        else:
            self.scaler_mean = self.scaler_std = None

    def _init_like_reference(self) -> None:
        """nn.Linear default init in the reference construction order
        (create_continuous_q_function, then create_deterministic_policy)."""
        D, A, C = self._observation_shape[0], self._action_size, self._n_critics
        hq = list(self._critic_encoder_factory.hidden_units)
        hp = list(self._actor_encoder_factory.hidden_units)
        for c in range(C):
            sizes = [D + A] + hq
            for l in range(len(hq)):
                self.critic.load_linear(l, c, nn.Linear(sizes[l], sizes[l + 1]))
            self.critic.load_linear(len(hq), c, nn.Linear(hq[-1], 1))
        sizes = [D] + hp
        for l in range(len(hp)):
            self.policy.load_linear(l, 0, nn.Linear(sizes[l], sizes[l + 1]))
        self.policy.load_linear(len(hp), 0, nn.Linear(hp[-1], A))

    # ---------------------------------------------------------- checkpoints
    def _critic_refs(self):
        refs, L = [], self.critic.n_layers
        for c in range(self._n_critics):
            for l in range(L - 1):
                refs.append((f"_q_funcs.{c}._encoder._fcs.{l}.weight", self.critic.wname(l), c, None))
                refs.append((f"_q_funcs.{c}._encoder._fcs.{l}.bias", self.critic.bname(l), c, None))
            refs.append((f"_q_funcs.{c}._fc.weight", self.critic.wname(L - 1), c, None))
            refs.append((f"_q_funcs.{c}._fc.bias", self.critic.bname(L - 1), c, None))
        return refs

    def _policy_refs(self):
        """DeterministicPolicy.parameters() order: encoder fcs, _fc."""
        refs, L = [], self.policy.n_layers
        for l in range(L - 1):
            refs.append((f"_encoder._fcs.{l}.weight", self.policy.wname(l), 0, None))
            refs.append((f"_encoder._fcs.{l}.bias", self.policy.bname(l), 0, None))
        refs.append(("_fc.weight", self.policy.wname(L - 1), 0, None))
        refs.append(("_fc.bias", self.policy.bname(L - 1), 0, None))
        return refs

    def get_state_dict(self) -> Dict[str, dict]:
        """torch_utility.get_state_dict layout of the reference TD3PlusBCImpl."""
        torch.cuda.synchronize()
        cr, pr = self._critic_refs(), self._policy_refs()
        return {
            "_q_func": ckpt.module_state(self.store, cr),
            "_targ_q_func": ckpt.module_state(self.targ, cr),
            "_policy": ckpt.module_state(self.store, pr),
            "_targ_policy": ckpt.module_state(self.targ, pr),
            "_critic_optim": ckpt.adam_state(self.critic_state, cr),
            "_actor_optim": ckpt.adam_state(self.actor_state, pr),
        }

    def set_state_dict(self, sd: Dict[str, dict]) -> None:
        cr, pr = self._critic_refs(), self._policy_refs()
        ckpt.load_module_state(self.store, cr, sd["_q_func"])
        ckpt.load_module_state(self.targ, cr, sd["_targ_q_func"])
        ckpt.load_module_state(self.store, pr, sd["_policy"])
        ckpt.load_module_state(self.targ, pr, sd["_targ_policy"])
        ckpt.load_adam_state(self.critic_state, cr, sd["_critic_optim"])
        ckpt.load_adam_state(self.actor_state, pr, sd["_actor_optim"])
        torch.cuda.synchronize()

    def save_model(self, fname: str) -> None:
        torch.save(self.get_state_dict(), fname)

    def load_model(self, fname: str) -> None:
        self.set_state_dict(torch.load(fname, map_location="cpu", weights_only=True))

    # --------------------------------------------------------------- updates
    def _workspace(self, B: int) -> "_Workspace":
        ws = self._ws.get(B)
        if ws is None:
            if self._ws:
                raise NotImplementedError("one batch size per TD3PlusBCImpl is supported")
            ws = _Workspace(self, B)
            self._ws[B] = ws
        return ws

    def update_step(self, batch, update_actor: bool = True,
                    noise: Optional[np.ndarray] = None, sync: bool = True,
                    use_graph: bool = True):
        """One TD3PlusBC._update: critic; actor + both targets when update_actor."""
        return self._run(batch, (True, update_actor, update_actor), noise, sync, use_graph)

    def update_critic(self, batch, noise: Optional[np.ndarray] = None) -> np.ndarray:
        m = self._run(batch, (True, False, False), noise, True, False)
        return np.float32(m["critic_loss"])

    def update_actor(self, batch) -> np.ndarray:
        m = self._run(batch, (False, True, False), None, True, False)
        return np.float32(m["actor_loss"])

    def update_critic_target(self) -> None:
        s, e = self.store.span(self.critic.names())
        ops.soft_update(self.targ.data[s:e], self.store.data[s:e], self._tau)

    def update_actor_target(self) -> None:
        s, e = self.store.span(self.policy.names())
        ops.soft_update(self.targ.data[s:e], self.store.data[s:e], self._tau)

    def _run(self, batch, flags, noise, sync, use_graph):
        db = as_device_batch(batch, self.torch_device)
        ws = self._workspace(db.batch_size)
        ws.stage(db, noise)
        ws.execute(flags, use_graph=use_graph and noise is None)
        if not sync:
            return None
        vals = ws.metrics.cpu().numpy()
        return {k: float(v) for k, v in zip(METRIC_NAMES, vals)}

    # ------------------------------------------------- device-side batches
    def staging_batch(self, batch_size: int) -> DeviceBatch:
        ws = self._workspace(batch_size)
        B = batch_size
        return DeviceBatch(ws.obs2[:B], ws.act, ws.rew, ws.obs2[B:], ws.term, ws.nsteps)

    def active_metric_names(self):
        return list(METRIC_NAMES)

    def metrics_ring(self, n_steps: int):
        for ws in self._ws.values():
            ws.ring_ctr.zero_()
        return n_steps

    def read_metrics_ring(self, handle):
        names = self.active_metric_names()
        if not self._ws:
            return names, np.zeros((0, len(names)), dtype=np.float32)
        ws = next(iter(self._ws.values()))
        k = min(int(ws.ring_ctr.item()), ws.ring.shape[0])
        return names, ws.ring[:k].cpu().numpy()

    # ------------------------------------------------------------- inference
    def _policy_module(self) -> nn.Module:
        from ..export import DeterministicPolicy, mlp_module
        return DeterministicPolicy(mlp_module(self.policy, self.store))

    def _predict_best_action(self, x: torch.Tensor) -> torch.Tensor:
        acts = mlp.Acts.alloc(self.policy, x.shape[0], self.torch_device)
        x = x.contiguous().float()
        mlp.forward(self.policy, self.store, x.data_ptr(), True, x.shape[1], acts)
        return torch.tanh(acts.out[0])

    def _sample_action(self, x: torch.Tensor) -> torch.Tensor:
        # DDPGImpl._sample_action (ddpg_impl.py:262-263): the greedy action
        return self._predict_best_action(x)

    def _predict_value(self, x: torch.Tensor, action: torch.Tensor) -> torch.Tensor:
        xa = torch.cat([x.float(), action.float()], dim=1).contiguous()
        acts = mlp.Acts.alloc(self.critic, xa.shape[0], self.torch_device)
        mlp.forward(self.critic, self.store, xa.data_ptr(), True, xa.shape[1], acts)
        return acts.out

    # ------------------------------------------------------------ inspection
    def critic_grad(self, name: str) -> torch.Tensor:
        return next(iter(self._ws.values())).critic_opt.grad(name)

    def policy_grad(self, name: str) -> torch.Tensor:
        return next(iter(self._ws.values())).actor_opt.grad(name)


class _Workspace:
    """Every device buffer of one TD3+BC update at batch size B."""

    def __init__(self, impl: TD3PlusBCImpl, B: int):
        dev = impl.torch_device
        self.impl = impl
        D, A, C = impl._observation_shape[0], impl._action_size, impl._n_critics
        self.B, self.D, self.A, self.C = B, D, A, C
        self.LDX = LDX = (D + A + 3) // 4 * 4  # 16-byte aligned Q-input rows
        z = lambda *s: torch.zeros(*s, dtype=torch.float32, device=dev)  # noqa: E731
        self.obs2 = z(2 * B, D)
        self.act = z(B, A)
        self.rew = z(B)
        self.term = z(B)
        self.nsteps = z(B)
        self.noise = z(B * A)
        self.rng_ctr = torch.zeros(1, dtype=torch.int64, device=dev)
        self.rng_ticket = torch.zeros(1, dtype=torch.int32, device=dev)
        self.seed = int(torch.randint(0, 2**62, (1,)).item())
        self.x_q = z(B, LDX)
        self.x_targ = z(B, LDX)
        self.x_actor = z(B, LDX)
        self.tpacts = mlp.Acts.alloc(impl.policy, B, dev)
        self.pacts = mlp.Acts.alloc(impl.policy, B, dev)
        self.qacts = mlp.Acts.alloc(impl.critic, B, dev)
        self.tacts = mlp.Acts.alloc(impl.critic, B, dev)
        self.aacts = mlp.Acts.alloc(impl.critic, B, dev)
        self.dq = z(C, B)
        self.ag = z(B)
        self.adx = z(B, D + A)
        self.pi_act = z(B, A)
        self.dhead = z(B, A)
        self.metrics = z(len(METRIC_NAMES))
        self.scalars = z(4)
        self.ring = z(1 << 16, len(METRIC_NAMES))
        self.ring_ctr = torch.zeros(1, dtype=torch.int64, device=dev)
        self.cgrads = GradSpace(dev)
        self.cbwd = mlp.BackwardSpace(impl.critic, B, self.cgrads, dev)
        self.abwd = mlp.BackwardSpace(impl.critic, B, None, dev)
        self.pgrads = GradSpace(dev)
        self.pbwd = mlp.BackwardSpace(impl.policy, B, self.pgrads, dev)
        self.critic_opt = AdamGroup(impl.critic_state, self.cgrads)
        self.actor_opt = AdamGroup(impl.actor_state, self.pgrads)
        self._graphs: Dict[tuple, torch.cuda.CUDAGraph] = {}
        self._op_state = None  # tensors the update-step op declares mutated
        self._ran_eager = set()
        self._external_noise = False
        self._build_descs()

    def _build_descs(self):
        impl = self.impl
        B, D, A, C, LDX = self.B, self.D, self.A, self.C, self.LDX
        p = NAT.Td3PrepDesc()
        p.obs, p.next_obs, p.act = (self.obs2.data_ptr(), self.obs2.data_ptr() + 4 * B * D,
                                    self.act.data_ptr())
        if impl.scaler_mean is not None:
            p.mean, p.std = impl.scaler_mean.data_ptr(), impl.scaler_std.data_ptr()
            p.eps = impl._scaler.eps
        p.x_q, p.x_targ = self.x_q.data_ptr(), self.x_targ.data_ptr()
        p.B, p.D, p.A, p.ldx = B, D, A, LDX
        self.prep_desc = p

        t = NAT.Td3TargetDesc()
        t.head, t.noise = self.tpacts.out.data_ptr(), self.noise.data_ptr()
        t.sigma, t.clip = impl._target_smoothing_sigma, impl._target_smoothing_clip
        t.x_targ, t.ldx, t.D, t.B, t.A = self.x_targ.data_ptr(), LDX, D, B, A
        self.target_desc = t

        l = NAT.Td3CriticLossDesc()
        l.q, l.q_targ = self.qacts.out.data_ptr(), self.tacts.out.data_ptr()
        l.rew, l.term, l.n_steps = self.rew.data_ptr(), self.term.data_ptr(), self.nsteps.data_ptr()
        l.dq, l.metrics = self.dq.data_ptr(), self.metrics.data_ptr()
        l.B, l.C, l.gamma = B, C, impl._gamma
        self.loss_desc = l

        a = NAT.Td3bcActorDesc()
        a.head, a.x_q, a.x_actor, a.pi_act = (self.pacts.out.data_ptr(), self.x_q.data_ptr(),
                                              self.x_actor.data_ptr(), self.pi_act.data_ptr())
        a.q0, a.g, a.scalars = self.aacts.out.data_ptr(), self.ag.data_ptr(), self.scalars.data_ptr()
        a.dq_da, a.ld_da, a.da_off = self.adx.data_ptr(), D + A, D
        a.act, a.dhead, a.metrics = self.act.data_ptr(), self.dhead.data_ptr(), self.metrics.data_ptr()
        a.alpha = impl._alpha
        a.B, a.D, a.A, a.ldx = B, D, A, LDX
        a.bc = int(impl._BC)
        self.actor_desc = a

    def stage(self, db: DeviceBatch, noise) -> None:
        B, D = self.B, self.D
        if db.obs.data_ptr() != self.obs2.data_ptr():
            self.obs2[:B].copy_(db.obs.view(B, D), non_blocking=True)
            self.obs2[B:].copy_(db.next_obs.view(B, D), non_blocking=True)
            self.act.copy_(db.act.view(B, self.A), non_blocking=True)
            self.rew.copy_(db.rew.view(B), non_blocking=True)
            self.term.copy_(db.term.view(B), non_blocking=True)
            self.nsteps.copy_(db.n_steps.view(B), non_blocking=True)
        self._external_noise = noise is not None
        if noise is not None:
            self.noise.copy_(torch.as_tensor(np.asarray(noise), dtype=torch.float32).view(-1))

    def dominant_kernel(self):
        """The critic-ensemble forward over the B data rows (one d3a_mlp_fwd
        launch, or the hidden-layer GEMM on the per-layer path)."""
        impl = self.impl
        net, st = impl.critic, impl.store
        s = net.sizes
        B, C = self.B, self.C
        if mlp.fused_ok(net, B):
            def launch():
                mlp.forward(net, st, self.x_q.data_ptr(), True, self.LDX, self.qacts)
            flops = 2 * C * B * sum(s[l] * s[l + 1] for l in range(len(s) - 1))
            return launch, flops, (f"d3a_mlp_fwd critic ensemble: C={C} x {B} rows x "
                                   f"{'-'.join(map(str, s))}")
        Hin, H = s[1], s[2]
        h0, h1 = self.qacts.h[0], self.qacts.h[1]

        def launch():
            ops.linear_fwd(h0.data_ptr(), False, Hin, net.W(1, st), net.b(1, st), h1.data_ptr(),
                           C, B, Hin, H, relu=True, ldy=H, sxb=B * Hin, syb=B * H)
        return launch, 2 * C * B * Hin * H, f"gemm_f32 critic layer-2 fwd: C={C} x [{B}x{Hin}]@[{Hin}x{H}]"

    def execute(self, flags, use_graph: bool) -> None:
        key = tuple(bool(f) for f in flags) + (self._external_noise,)
        if not use_graph:
            self._enqueue(*flags)
            return
        g = self._graphs.get(key)
        if g is None:
            if key not in self._ran_eager:
                self._ran_eager.add(key)
                self._enqueue(*flags)
                return
            g = torch.cuda.CUDAGraph()
            torch.cuda.synchronize()
            with ops.graph_capture(g):
                self._enqueue(*flags)
            self._graphs[key] = g
        # the replay through the torch custom op (TORCH_LIBRARY d3rlpy_amd)
        if self._op_state is None:
            self._op_state = ops.update_state(self.impl, self)
        ops.replay_update(g, self._op_state)

    def _enqueue(self, critic: bool, actor: bool, targets: bool) -> None:
        impl = self.impl
        B, D, A, LDX = self.B, self.D, self.A, self.LDX
        st, tg = impl.store, impl.targ
        ops.call_desc("d3a_td3_prep", self.prep_desc)
        if critic:
            # DDPG (sigma = 0) draws no smoothing noise: the zero buffer leaves
            # clamp(tanh(mu') + 0, -1, 1) = tanh(mu') (ddpg_impl.py:251-260)
            if not self._external_noise and impl._target_smoothing_sigma != 0.0:
                ops.philox_fill(self.noise, B * A, 0, -1.0, 1.0, self.seed, self.rng_ctr,
                                self.rng_ticket)
            # target action: targ_policy(s') + clipped noise (td3_impl.py:61-78)
            mlp.forward(impl.policy, tg, self.x_targ.data_ptr(), True, LDX, self.tpacts,
                        keep_h=False)
            ops.call_desc("d3a_td3_target", self.target_desc)
            # critic ensemble on (s, a) and, in the same launches, the target
            # ensemble on (s', a') (aux pass)
            mlp.forward(impl.critic, st, self.x_q.data_ptr(), True, LDX, self.qacts,
                        aux=(tg, self.x_targ.data_ptr(), LDX, self.tacts))
            self.loss_desc.actor_step = int(actor)
            ops.call_desc("d3a_td3_critic_loss", self.loss_desc)
            mlp.backward(self.cbwd, st, self.x_q.data_ptr(), True, LDX, self.qacts,
                         self.dq.data_ptr(), 1, B, 0, B)
            self.critic_opt.launch()
        if actor:
            mlp.forward(impl.policy, st, self.x_q.data_ptr(), True, LDX, self.pacts)
            ad = self.actor_desc
            ops.call_desc("d3a_td3bc_actor_input", ad)
            # q_t = q_func(s, pi(s), "none")[0]: only member 0 enters the loss
            mlp.forward(impl.critic, st, self.x_actor.data_ptr(), True, LDX, self.aacts,
                        members=1)
            ops.call_desc("d3a_td3bc_actor_seed", ad)
            mlp.backward(self.abwd, st, self.x_actor.data_ptr(), True, LDX, self.aacts,
                         self.ag.data_ptr(), 1, B, 0, B, weight_grads=False, dx=self.adx,
                         members=1)
            ops.call_desc("d3a_td3bc_actor_head", ad)
            mlp.backward(self.pbwd, st, self.x_q.data_ptr(), True, LDX, self.pacts,
                         self.dhead.data_ptr(), A, B * A, 0, B)
            self.actor_opt.launch()
        ops.step_end(impl.counters, (1 if critic else 0) | (2 if actor else 0), self.metrics,
                     self.ring, self.ring_ctr, impl.targ.data if targets else None,
                     impl.store.data if targets else None, impl._tau)
