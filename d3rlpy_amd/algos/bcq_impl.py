"""BCQImpl on HIP kernels — drop-in for d3rlpy/algos/torch/bcq_impl.py:25-226
(continuous BCQ; quantile-regression critics as in K3).

Same constructor arguments and ``update_imitator / update_critic /
update_actor / update_critic_target / update_actor_target`` methods; plus
``update_step`` = one ``BCQ._update`` (algos/bcq.py:261-279 with the
defaults rl_start_step 0, update_actor_interval 1) as one device pipeline
(a HIP-graph replay after the first call).

Pipeline of one update_step:
  imitator  x = (s, a) -> VAE encoder -> d3a_bcq_vae_sample (z = mu + eps std,
            KL) -> VAE decoder -> d3a_bcq_vae_loss -> decoder backward (with
            dL/dz) -> d3a_bcq_vae_enc_grad -> encoder backward -> Adam
  critic    target over N sampled actions per next state (B*N rows):
            (s', clamp(z)) -> decoder -> (s', tanh) -> target residual policy
            -> (s', clamp(a + 0.05 tanh)) -> target QR critics -> d3a_bcq_target
            (compute_max_with_n_actions); critics on (s, a) ->
            d3a_bcq_qr_loss (quantile Huber) -> backward -> Adam
  actor     (s, clamp(z)) -> decoder -> residual policy -> critic 0 ->
            dQ0/da -> d3a_bcq_actor_head -> policy backward -> Adam
  targets   one soft update over the contiguous critic + policy parameters
The B*N-row target passes (25,600 rows at K3) run through the one-launch
fused MLP forward (d3a_mlp_fwd, MFMA quantile head).
"""
from __future__ import annotations

import math
import os
from typing import Dict, Optional, Sequence

import numpy as np
import torch
from torch import nn

from .. import _native as NAT
from .. import checkpoint as ckpt
from .. import mlp, ops
from ..nets import AdamGroup, EnsembleMLP, GradSpace, OptimState, ParamStore
from .impl_base import DeviceBatch, ImplBase, as_device_batch

METRIC_NAMES = ("imitator_loss", "critic_loss", "actor_loss")

# the B-row small-net passes on d3a_mlp_fwd's parts path (D3A_BCQ_PARTS=0: the
# one-workgroup-per-16-rows small kernel, A/B)
_PARTS = os.environ.get("D3A_BCQ_PARTS", "1") == "1"

# concurrent graph branches in the update (_Workspace._enqueue), off by
# default: measured slower at K3, round 5 -- forked at the step's start 1,758
# against 1,825 steps/s (every cross-stream edge costs ~4 us between the small
# launches of the imitator chain), forked behind the imitator (as now) 1,521
# against 1,829 (the side passes' workgroups delay the one-per-CU target pass
# and stretch its tail); D3A_BCQ_BRANCHES=1 turns them on
_BRANCHES = os.environ.get("D3A_BCQ_BRANCHES", "0") == "1"
# a full update (imitator, critic, actor and targets) carries the targets' soft
# update and the step bookkeeping in its three Adam launches instead of a
# d3a_step_end launch (as CQL's update does); D3A_BCQ_ADAM_TAIL=0 keeps
# step_end (A/B)
_ADAM_TAIL = os.environ.get("D3A_BCQ_ADAM_TAIL", "1") == "1"
# the step's Philox noise on extra workgroups of the VAE encoder's launch
# (round 6; D3A_BCQ_PHILOX_IN_ENC=0: its own d3a_philox_fill launch)
_PHILOX_IN_ENC = os.environ.get("D3A_BCQ_PHILOX_IN_ENC", "1") == "1"
# the target rows formed inside the QR-loss launch (from the target pass's
# quantile means) instead of a d3a_bcq_target launch; D3A_BCQ_FUSED_TARGET=0
# keeps the launch (A/B)
_FUSED_TARGET = os.environ.get("D3A_BCQ_FUSED_TARGET", "1") == "1"


def _pad4(n: int) -> int:
    return (n + 3) // 4 * 4


class BCQImpl(ImplBase):
    def __init__(
        self,
        observation_shape: Sequence[int],
        action_size: int,
        actor_learning_rate: float,
        critic_learning_rate: float,
        imitator_learning_rate: float,
        actor_optim_factory,
        critic_optim_factory,
        imitator_optim_factory,
        actor_encoder_factory,
        critic_encoder_factory,
        imitator_encoder_factory,
        q_func_factory,
        gamma: float,
        tau: float,
        n_critics: int,
        lam: float,
        n_action_samples: int,
        action_flexibility: float,
        beta: float,
        use_gpu,
        scaler,
        action_scaler,
        reward_scaler,
    ):
        super().__init__(observation_shape, action_size, scaler, action_scaler, reward_scaler,
                         use_gpu)
        if q_func_factory.get_type() != "qr":
            raise NotImplementedError("BCQ on HIP implements the quantile-regression critics of "
                                      "K3 (q_func_factory='qr')")
        if len(observation_shape) != 1:
            raise NotImplementedError("BCQ on HIP supports vector observations")
        if scaler is not None and scaler.get_type() != "standard":
            raise NotImplementedError("the HIP BCQImpl supports the 'standard' scaler")
        if action_scaler is not None or reward_scaler is not None:
            raise NotImplementedError("action/reward scalers are out of scope (SURVEY §2 #4)")
        self._actor_learning_rate = actor_learning_rate
        self._critic_learning_rate = critic_learning_rate
        self._imitator_learning_rate = imitator_learning_rate
        self._actor_optim_factory = actor_optim_factory
        self._critic_optim_factory = critic_optim_factory
        self._imitator_optim_factory = imitator_optim_factory
        self._actor_encoder_factory = actor_encoder_factory
        self._critic_encoder_factory = critic_encoder_factory
        self._imitator_encoder_factory = imitator_encoder_factory
        self._q_func_factory = q_func_factory
        self._gamma = gamma
        self._tau = tau
        self._n_critics = n_critics
        self._lam = lam
        self._n_action_samples = n_action_samples
        self._action_flexibility = action_flexibility
        self._beta = beta
        self._n_quantiles = q_func_factory.n_quantiles
        self._ws: Dict[int, "_Workspace"] = {}

    # ------------------------------------------------------------------ build
    def build(self) -> None:
        dev = self.torch_device
        D, A, C, K = self._observation_shape[0], self._action_size, self._n_critics, \
            self._n_quantiles
        L = 2 * A
        hi = list(self._imitator_encoder_factory.hidden_units)
        hq = list(self._critic_encoder_factory.hidden_units)
        hp = list(self._actor_encoder_factory.hidden_units)
        store = ParamStore()
        # imitator first (bcq_impl.py:101-105), then critic and actor: the
        # critic and policy segments are contiguous (one soft-update span)
        self.vae_enc = EnsembleMLP(store, "ve", 1, [D + A] + hi + [2 * L])
        self.vae_dec = EnsembleMLP(store, "vd", 1, [D + L] + hi + [A])
        self.critic = EnsembleMLP(store, "q", C, [D + A] + hq + [K])
        self.policy = EnsembleMLP(store, "pi", 1, [D + A] + hp + [A])
        store.allocate(dev)
        self.store = store
        self._init_like_reference()
        self.targ = store.like()
        self.targ.data.copy_(store.data)
        self.counters = torch.zeros(8, dtype=torch.int64, device=dev)  # critic, actor, imitator
        f = self._critic_optim_factory
        self.critic_state = OptimState(store, self.critic.names(), self._critic_learning_rate,
                                       f.betas, f.eps, step=self.counters[0:1])
        f = self._actor_optim_factory
        self.actor_state = OptimState(store, self.policy.names(), self._actor_learning_rate,
                                      f.betas, f.eps, step=self.counters[1:2])
        f = self._imitator_optim_factory
        self.imitator_state = OptimState(store, self.vae_enc.names() + self.vae_dec.names(),
                                         self._imitator_learning_rate, f.betas, f.eps,
                                         step=self.counters[2:3])
        s0, _ = store.span(self.critic.names())
        _, e1 = store.span(self.policy.names())
        self.soft_span = (s0, e1)

    def _init_like_reference(self) -> None:
        """nn.Linear default init in the reference construction order."""
        D, A, C, K = self._observation_shape[0], self._action_size, self._n_critics, \
            self._n_quantiles
        L = 2 * A
        hi = list(self._imitator_encoder_factory.hidden_units)
        hq = list(self._critic_encoder_factory.hidden_units)
        hp = list(self._actor_encoder_factory.hidden_units)
        for net, d_in in ((self.vae_enc, D + A), (self.vae_dec, D + L)):
            sizes = [d_in] + hi
            for l in range(len(hi)):
                net.load_linear(l, 0, nn.Linear(sizes[l], sizes[l + 1]))
        mu, ls, fc = nn.Linear(hi[-1], L), nn.Linear(hi[-1], L), nn.Linear(hi[-1], A)
        W, b = self.vae_enc.export_linear(len(hi), 0)
        with torch.no_grad():
            W[:L].copy_(mu.weight)
            W[L:].copy_(ls.weight)
            b[:L].copy_(mu.bias)
            b[L:].copy_(ls.bias)
        self.vae_dec.load_linear(len(hi), 0, fc)
        for c in range(C):
            sizes = [D + A] + hq
            for l in range(len(hq)):
                self.critic.load_linear(l, c, nn.Linear(sizes[l], sizes[l + 1]))
            self.critic.load_linear(len(hq), c, nn.Linear(hq[-1], K))
        sizes = [D + A] + hp
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
        """DeterministicResidualPolicy.parameters(): encoder fcs, _fc."""
        refs, L = [], self.policy.n_layers
        for l in range(L - 1):
            refs.append((f"_encoder._fcs.{l}.weight", self.policy.wname(l), 0, None))
            refs.append((f"_encoder._fcs.{l}.bias", self.policy.bname(l), 0, None))
        refs.append(("_fc.weight", self.policy.wname(L - 1), 0, None))
        refs.append(("_fc.bias", self.policy.bname(L - 1), 0, None))
        return refs

    def _imitator_refs(self):
        """ConditionalVAE.parameters(): encoder fcs, decoder fcs, _mu, _logstd, _fc."""
        refs = []
        for pre, net in (("_encoder_encoder", self.vae_enc), ("_decoder_encoder", self.vae_dec)):
            for l in range(net.n_layers - 1):
                refs.append((f"{pre}._fcs.{l}.weight", net.wname(l), 0, None))
                refs.append((f"{pre}._fcs.{l}.bias", net.bname(l), 0, None))
        L, Le = 2 * self._action_size, self.vae_enc.n_layers - 1
        mu, ls = slice(0, L), slice(L, 2 * L)
        refs += [("_mu.weight", self.vae_enc.wname(Le), 0, mu),
                 ("_mu.bias", self.vae_enc.bname(Le), 0, mu),
                 ("_logstd.weight", self.vae_enc.wname(Le), 0, ls),
                 ("_logstd.bias", self.vae_enc.bname(Le), 0, ls),
                 ("_fc.weight", self.vae_dec.wname(self.vae_dec.n_layers - 1), 0, None),
                 ("_fc.bias", self.vae_dec.bname(self.vae_dec.n_layers - 1), 0, None)]
        return refs

    def get_state_dict(self) -> Dict[str, dict]:
        """torch_utility.get_state_dict layout of the reference BCQImpl."""
        torch.cuda.synchronize()
        cr, pr, ir = self._critic_refs(), self._policy_refs(), self._imitator_refs()
        return {
            "_q_func": ckpt.module_state(self.store, cr),
            "_targ_q_func": ckpt.module_state(self.targ, cr),
            "_policy": ckpt.module_state(self.store, pr),
            "_targ_policy": ckpt.module_state(self.targ, pr),
            "_imitator": ckpt.module_state(self.store, ir),
            "_critic_optim": ckpt.adam_state(self.critic_state, cr),
            "_actor_optim": ckpt.adam_state(self.actor_state, pr),
            "_imitator_optim": ckpt.adam_state(self.imitator_state, ir),
        }

    def set_state_dict(self, sd: Dict[str, dict]) -> None:
        cr, pr, ir = self._critic_refs(), self._policy_refs(), self._imitator_refs()
        ckpt.load_module_state(self.store, cr, sd["_q_func"])
        ckpt.load_module_state(self.targ, cr, sd["_targ_q_func"])
        ckpt.load_module_state(self.store, pr, sd["_policy"])
        ckpt.load_module_state(self.targ, pr, sd["_targ_policy"])
        ckpt.load_module_state(self.store, ir, sd["_imitator"])
        ckpt.load_adam_state(self.critic_state, cr, sd["_critic_optim"])
        ckpt.load_adam_state(self.actor_state, pr, sd["_actor_optim"])
        ckpt.load_adam_state(self.imitator_state, ir, sd["_imitator_optim"])
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
                raise NotImplementedError("one batch size per BCQImpl is supported")
            ws = _Workspace(self, B)
            self._ws[B] = ws
        return ws

    def update_step(self, batch, noise: Optional[Dict[str, np.ndarray]] = None,
                    sync: bool = True, use_graph: bool = True):
        """One BCQ._update: imitator, critic, actor, both soft target updates."""
        return self._run(batch, (True, True, True, True), noise, sync, use_graph)

    def update_imitator(self, batch) -> np.ndarray:
        return np.float32(self._run(batch, (True, False, False, False), None, True,
                                    False)["imitator_loss"])

    def update_critic(self, batch) -> np.ndarray:
        return np.float32(self._run(batch, (False, True, False, False), None, True,
                                    False)["critic_loss"])

    def update_actor(self, batch) -> np.ndarray:
        return np.float32(self._run(batch, (False, False, True, False), None, True,
                                    False)["actor_loss"])

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
        out = {k: float(v) for k, v in zip(METRIC_NAMES, vals)}
        if flags[1] and not flags[2]:
            # the critic-loss reduction runs inside the actor stage; without
            # it, reduce the per-row losses here (method-level call only)
            out["critic_loss"] = float(ws.loss_cb.double().sum().item() / ws.B)
        return out

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
    def _mlp(self, net, x: torch.Tensor, store=None) -> torch.Tensor:
        x = x.contiguous().float()
        acts = mlp.Acts.alloc(net, x.shape[0], self.torch_device)
        mlp.forward(net, store or self.store, x.data_ptr(), True, x.shape[1], acts,
                    keep_h=False)
        return acts.out

    def _policy_module(self) -> nn.Module:
        from ..export import BCQGreedy, mlp_module
        return BCQGreedy(mlp_module(self.vae_dec, self.store), mlp_module(self.policy, self.store),
                         mlp_module(self.critic, self.store, 0), self._action_size,
                         self._n_action_samples, self._action_flexibility)

    def _predict_best_action(self, x: torch.Tensor) -> torch.Tensor:
        """bcq_impl.py:204-210: N sampled actions per state, argmax of Q_0."""
        N, A = self._n_action_samples, self._action_size
        B = x.shape[0]
        rx = x.repeat_interleave(N, dim=0)
        z = torch.randn(B * N, 2 * A, device=x.device).clamp(-0.5, 0.5)
        a_dec = torch.tanh(self._mlp(self.vae_dec, torch.cat([rx, z], 1))[0])
        res = self._mlp(self.policy, torch.cat([rx, a_dec], 1))[0]
        act = (a_dec + self._action_flexibility * torch.tanh(res)).clamp(-1.0, 1.0)
        q0 = self._mlp(self.critic, torch.cat([rx, act], 1))[0].mean(dim=1)
        idx = q0.view(B, N).argmax(dim=1)
        return act.view(B, N, A)[torch.arange(B, device=x.device), idx]

    def _sample_action(self, x: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError("BCQ does not support sampling action")

    def _predict_value(self, x: torch.Tensor, action: torch.Tensor) -> torch.Tensor:
        q = self._mlp(self.critic, torch.cat([x.float(), action.float()], 1))
        return q.mean(dim=2)  # [C][B] quantile means (ContinuousQRQFunction.forward)

    # ------------------------------------------------------------ inspection
    def critic_grad(self, name: str) -> torch.Tensor:
        return next(iter(self._ws.values())).critic_opt.grad(name)

    def policy_grad(self, name: str) -> torch.Tensor:
        return next(iter(self._ws.values())).actor_opt.grad(name)

    def imitator_grad(self, name: str) -> torch.Tensor:
        return next(iter(self._ws.values())).imitator_opt.grad(name)


class _Workspace:
    """Every device buffer of one BCQ update at batch size B."""

    def __init__(self, impl: BCQImpl, B: int):
        dev = impl.torch_device
        self.impl = impl
        D, A, C, K, N = (impl._observation_shape[0], impl._action_size, impl._n_critics,
                         impl._n_quantiles, impl._n_action_samples)
        L = 2 * A
        self.B, self.D, self.A, self.C, self.K, self.N, self.L = B, D, A, C, K, N, L
        BN = B * N
        self.LX1, self.LX2 = _pad4(D + A), _pad4(D + L)
        z = lambda *s: torch.zeros(*s, dtype=torch.float32, device=dev)  # noqa: E731
        self.obs2 = z(2 * B, D)
        self.act = z(B, A)
        self.rew = z(B)
        self.term = z(B)
        self.nsteps = z(B)
        # with a standard scaler every row builder reads the transform xobs2
        # (d3a_standardize_f32, TorchMiniBatch scaling, torch_utility.py:179-181)
        sc = impl._scaler
        if sc is not None:
            assert sc._mean is not None, "fit the scaler before the first update"
            self.sc_mean = torch.as_tensor(np.asarray(sc._mean, dtype=np.float32).reshape(-1),
                                           device=dev)
            self.sc_std = torch.as_tensor(np.asarray(sc._std, dtype=np.float32).reshape(-1),
                                          device=dev)
            self.sc_eps = float(sc._eps)
            self.xobs2 = z(2 * B, D)
        else:
            self.xobs2 = self.obs2
        self.obs, self.next_obs = self.xobs2[:B], self.xobs2[B:]
        # noise: [eps_vae (B L) | z_target (B N L) | z_actor (B L)]
        self.noise = z((B + BN + B) * L)
        self.eps_vae = self.noise[:B * L]
        self.z_target = self.noise[B * L:(B + BN) * L]
        self.z_actor = self.noise[(B + BN) * L:]
        self.rng_ctr = torch.zeros(1, dtype=torch.int64, device=dev)
        self.rng_ticket = torch.zeros(1, dtype=torch.int32, device=dev)
        self.seed = int(torch.randint(0, 2**62, (1,)).item())
        # imitator
        self.x_q = z(B, self.LX1)                       # (s, a): VAE encoder + critic rows
        self.ve_acts = mlp.Acts.alloc(impl.vae_enc, B, dev)
        self.std = z(B * L)
        self.x_vd = z(B, self.LX2)
        self.vd_acts = mlp.Acts.alloc(impl.vae_dec, B, dev)
        self.dhead_d = z(B, A)
        self.dx_vd = z(1, B, D + L)
        self.dhead_e = z(B, 2 * L)
        self.igrads = GradSpace(dev)
        self.ve_bwd = mlp.BackwardSpace(impl.vae_enc, B, self.igrads, dev, small=True)
        self.vd_bwd = mlp.BackwardSpace(impl.vae_dec, B, self.igrads, dev, small=True)
        # critic target over B*N sampled actions
        self.x_td = z(BN, self.LX2)
        self.td_acts = mlp.Acts.alloc(impl.vae_dec, BN, dev)
        self.x_tp = z(BN, self.LX1)
        self.tp_acts = mlp.Acts.alloc(impl.policy, BN, dev)
        self.x_tq = z(BN, self.LX1)
        self.tq_acts = mlp.Acts.alloc(impl.critic, BN, dev)
        self.target = z(B, K)
        self.q_acts = mlp.Acts.alloc(impl.critic, B, dev)
        self.dq = z(C, B, K)
        self.loss_cb = z(C, B)
        self.cgrads = GradSpace(dev)
        self.cbwd = mlp.BackwardSpace(impl.critic, B, self.cgrads, dev, small=True)
        # actor
        self.x_ad = z(B, self.LX2)
        self.ad_acts = mlp.Acts.alloc(impl.vae_dec, B, dev)
        self.a_dec_a = z(B, A)
        self.x_pa = z(B, self.LX1)
        self.pa_acts = mlp.Acts.alloc(impl.policy, B, dev)
        # the four B-row passes of the small nets (VAE encoder / decoder, the
        # actor's decoder and residual policy) on d3a_mlp_fwd's parts path: the
        # second layer split over D3A_MLP_PARTS workgroups, the head written as
        # partial sums the consumers add in order (d3a_bcq_* head_parts)
        P_ = NAT.MLP_PARTS
        pz = lambda net: (torch.zeros(P_, net.C, B, net.sizes[-1], device=dev)  # noqa: E731
                          if _PARTS and mlp.parts_ok(net) else None)
        self.pe, self.pd = pz(impl.vae_enc), pz(impl.vae_dec)  # (pe None where the
        # encoder's 2 L outputs exceed the parts path's 32: its head a matrix)
        self.pad, self.ppi = pz(impl.vae_dec), pz(impl.policy)
        self.x_qa = z(B, self.LX1)
        self.qa_acts = mlp.Acts.alloc(impl.critic, B, dev)
        # d(-mean_b mean_k q0)/dq0 is a constant
        self.dconst = torch.full((1, B, K), -1.0 / (B * K), dtype=torch.float32, device=dev)
        self.abwd = mlp.BackwardSpace(impl.critic, B, None, dev, small=True)
        self.adx = z(1, B, D + A)
        self.dhead_pi = z(B, A)
        self.pgrads = GradSpace(dev)
        self.pbwd = mlp.BackwardSpace(impl.policy, B, self.pgrads, dev, small=True)
        self.metrics = z(len(METRIC_NAMES))
        self.scalars = z(4)
        self.ring = z(1 << 16, len(METRIC_NAMES))
        self.ring_ctr = torch.zeros(1, dtype=torch.int64, device=dev)
        self.imitator_opt = AdamGroup(impl.imitator_state, self.igrads)
        self.critic_opt = AdamGroup(impl.critic_state, self.cgrads)
        self.actor_opt = AdamGroup(impl.actor_state, self.pgrads)
        self._graphs: Dict[tuple, torch.cuda.CUDAGraph] = {}
        self._op_state = None  # tensors the update-step op declares mutated
        self._ran_eager = set()
        self._external_noise = False
        self._build_descs()

    def _rows(self, obs, rep, a, E, lda, mode, x, ldx, rows, base=None, e_out=None, clip=0.0,
              scale=0.0, a_parts=None):
        d = NAT.BcqRowsDesc()
        d.obs, d.D, d.rep = obs.data_ptr(), self.D, rep
        d.a, d.E, d.lda = a, E, lda
        if a_parts is not None:  # a as head parts [P][1][rows][E]
            d.a, d.a_parts, d.s_a_part = a_parts.data_ptr(), a_parts.shape[0], a_parts[0].numel()
        d.base = base.data_ptr() if base is not None else None
        d.mode, d.clip, d.scale = mode, clip, scale
        d.x, d.ldx = x.data_ptr(), ldx
        d.e_out = e_out.data_ptr() if e_out is not None else None
        d.rows = rows
        return d

    def _build_descs(self):
        impl = self.impl
        B, D, A, C, K, N, L = self.B, self.D, self.A, self.C, self.K, self.N, self.L
        BN = B * N
        flex = impl._action_flexibility
        self.r_q = self._rows(self.obs, 1, self.act.data_ptr(), A, A, 0, self.x_q, self.LX1, B)
        # target: (s', clamp(z)) -> (s', tanh(dec)) -> (s', clamp(a_dec + flex tanh(pi)))
        self.r_td = self._rows(self.next_obs, N, self.z_target.data_ptr(), L, L, 1, self.x_td,
                               self.LX2, BN, clip=0.5)
        # (the x6 target passes build these rows while staging them: mlp.forward
        # xgen; the critic rows take the decoder's raw output as their base,
        # mode 4, so the policy pass need not store tanh of it)
        self.r_tp = self._rows(self.next_obs, N, self.td_acts.out.data_ptr(), A, A, 2, self.x_tp,
                               self.LX1, BN)
        self.r_tq = self._rows(self.next_obs, N, self.tp_acts.out.data_ptr(), A, A, 4, self.x_tq,
                               self.LX1, BN, base=self.td_acts.out, scale=flex)
        # actor: the same chain on (s, z_actor) with the online policy
        self.r_ad = self._rows(self.obs, 1, self.z_actor.data_ptr(), L, L, 1, self.x_ad,
                               self.LX2, B, clip=0.5)
        self.r_pa = self._rows(self.obs, 1, self.ad_acts.out.data_ptr(), A, A, 2, self.x_pa,
                               self.LX1, B, e_out=self.a_dec_a, a_parts=self.pad)
        self.r_qa = self._rows(self.obs, 1, self.pa_acts.out.data_ptr(), A, A, 3, self.x_qa,
                               self.LX1, B, base=self.a_dec_a, scale=flex, a_parts=self.ppi)

        v = NAT.BcqVaeDesc()
        v.obs, v.act, v.eps = self.obs.data_ptr(), self.act.data_ptr(), self.eps_vae.data_ptr()
        v.head_e, v.std_out = self.ve_acts.out.data_ptr(), self.std.data_ptr()
        v.x_dec, v.ldx = self.x_vd.data_ptr(), self.LX2
        v.head_d, v.dhead_d = self.vd_acts.out.data_ptr(), self.dhead_d.data_ptr()
        v.head_parts = NAT.MLP_PARTS
        # per-element KL terms: the sample kernel runs over many workgroups,
        # the loss kernel forms the logged KL mean
        self.kl_terms = torch.zeros(B * L, device=self.obs.device)
        v.kl = self.kl_terms.data_ptr()
        if self.pe is not None:
            v.head_e, v.s_e_part = self.pe.data_ptr(), self.pe[0].numel()
        if self.pd is not None:
            v.head_d, v.s_d_part = self.pd.data_ptr(), self.pd[0].numel()
        v.dx_dec, v.lddx, v.dhead_e = self.dx_vd.data_ptr(), D + L, self.dhead_e.data_ptr()
        v.scalars, v.metrics = self.scalars.data_ptr(), self.metrics.data_ptr()
        v.B, v.D, v.A, v.L = B, D, A, L
        v.beta, v.min_logstd, v.max_logstd = impl._beta, -4.0, 15.0
        self.vae_desc = v

        t = NAT.BcqTargetDesc()
        t.q, t.target = self.tq_acts.out.data_ptr(), self.target.data_ptr()
        # the quantile means, when the target pass's epilogue forms them
        self.tq_means = torch.zeros(C, BN, dtype=torch.float32, device=self.target.device)
        t.B, t.N, t.K, t.C, t.lam = B, N, K, C, impl._lam
        self.target_desc = t

        q = NAT.BcqQrDesc()
        q.q, q.target = self.q_acts.out.data_ptr(), self.target.data_ptr()
        q.rew, q.term, q.n_steps = self.rew.data_ptr(), self.term.data_ptr(), self.nsteps.data_ptr()
        q.dq, q.loss_cb = self.dq.data_ptr(), self.loss_cb.data_ptr()
        q.B, q.K, q.C, q.gamma = B, K, C, impl._gamma
        self.qr_desc = q

        a = NAT.BcqActorDesc()
        a.head, a.a_dec = self.pa_acts.out.data_ptr(), self.a_dec_a.data_ptr()
        if self.ppi is not None:
            a.head, a.head_parts, a.s_head_part = (self.ppi.data_ptr(), self.ppi.shape[0],
                                                   self.ppi[0].numel())
        a.dq_da, a.ld_da, a.da_off = self.adx.data_ptr(), D + A, D
        a.dhead, a.q0 = self.dhead_pi.data_ptr(), self.qa_acts.out.data_ptr()
        a.loss_cb, a.metrics = self.loss_cb.data_ptr(), self.metrics.data_ptr()
        a.B, a.A, a.K, a.C, a.scale = B, A, K, C, flex
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
            g = lambda k: torch.as_tensor(np.asarray(noise[k]), dtype=torch.float32).view(-1)  # noqa
            self.eps_vae.copy_(g("eps_vae"))
            self.z_target.copy_(g("z_target"))
            self.z_actor.copy_(g("z_actor"))

    def dominant_kernel(self):
        """The target QR-critic ensemble forward over the B*N sampled actions
        (d3a_mlp_fwd; MFMA 200-quantile head): the bulk of K3's FLOPs."""
        impl = self.impl
        net = impl.critic
        s = net.sizes
        BN = self.B * self.N

        def launch():
            mlp.forward(net, impl.targ, self.x_tq.data_ptr(), True, self.LX1, self.tq_acts,
                        keep_h=False, row_mean=self.tq_means, xgen=self.r_tq)
        flops = 2 * self.C * BN * sum(s[l] * s[l + 1] for l in range(len(s) - 1))
        x6 = ops.CRITIC_GEMM == "x6" and mlp.x6_wide_shape(net)
        return launch, flops, (f"d3a_mlp_fwd target QR critics ({'split-bf16 x6' if x6 else 'fp32'}"
                               f" MFMA): C={self.C} x {BN} rows x {'-'.join(map(str, s))}")

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

    def _side(self, i: int) -> torch.cuda.Stream:
        if not hasattr(self, "_sides"):
            self._sides = [torch.cuda.Stream(device=self.obs.device) for _ in range(2)]
        return self._sides[i]

    def _actor_prefix(self) -> None:
        """The actor loss's rows up to its critic pass: (s, clamp(z)) ->
        decoder -> residual policy -> (s, clamp(a + flex tanh)) rows."""
        impl, st = self.impl, self.impl.store
        # (the decoder's rows are built while it stages them: mlp.forward xgen;
        # the policy's are kept for its backward, with the decoded action)
        mlp.forward(impl.vae_dec, st, self.x_ad.data_ptr(), True, self.LX2, self.ad_acts,
                    keep_h=False, out_parts=self.pad, xgen=self.r_ad)
        # (the policy's rows and the decoded actions written by its forward:
        # the policy backward and the critic pass's residual read them)
        mlp.forward(impl.policy, st, self.x_pa.data_ptr(), True, self.LX1, self.pa_acts,
                    out_parts=self.ppi, xgen=self.r_pa, xgen_keep=True)

    def _enqueue(self, imitator: bool, critic: bool, actor: bool, targets: bool) -> None:
        impl = self.impl
        B, D, A, K, L = self.B, self.D, self.A, self.K, self.L
        st, tg = impl.store, impl.targ
        # the step's noise: on extra workgroups of the VAE encoder's parts-path
        # launch when the imitator update runs (it precedes every reader), else
        # its own launch
        ph = None
        if not self._external_noise:
            if imitator and _PHILOX_IN_ENC and self.pe is not None:
                ph = NAT.PhiloxJob()
                ph.out, ph.n_normal, ph.n_uniform = self.noise.data_ptr(), self.noise.numel(), 0
                ph.lo, ph.hi, ph.seed = -1.0, 1.0, self.seed
                ph.ctr, ph.ticket = self.rng_ctr.data_ptr(), self.rng_ticket.data_ptr()
            else:
                ops.philox_fill(self.noise, self.noise.numel(), 0, -1.0, 1.0, self.seed,
                                self.rng_ctr, self.rng_ticket)
        if impl._scaler is not None:
            ops.standardize(self.obs2, self.xobs2, self.sc_mean, self.sc_std, self.sc_eps)
        if not imitator:
            ops.call_desc("d3a_bcq_rows", self.r_q)
        # (else the VAE encoder's forward forms the (s, a) rows and writes
        # them for the critic passes and the encoder backward)
        # graph branches: the online critic forward on (s, a) reads only the
        # critic's pre-update parameters, so it runs beside the target pass on
        # side stream 1 (joined before the QR loss); the actor's decoder /
        # policy prefix needs only the updated imitator, so it runs beside the
        # critic update on side stream 2 (joined before the actor's critic
        # pass).  Independent nodes of the captured graph then
        # overlap instead of queueing one small launch behind another.
        main = torch.cuda.current_stream()
        branch = _BRANCHES and critic
        q_pending = a_pending = False
        # the fused tail: each Adam advances a counter it does not read --
        # imitator -> critic's, critic -> actor's, actor -> imitator's -- so
        # the critic and actor Adams read their step already advanced
        # (step_add 0); the critic / actor Adams soft-update their targets
        # (soft_span = critic + policy), the actor's pushes the
        # metric ring
        s_c0, s_c1 = impl.store.span(impl.critic.names())
        s_p0, s_p1 = impl.store.span(impl.policy.names())
        # (the span between the critic and policy segments holds only the
        # store's alignment padding, zeros in both copies)
        fused_tail = (_ADAM_TAIL and imitator and critic and actor and targets
                      and s_c1 <= s_p0 and (s_c0, s_p1) == tuple(impl.soft_span))
        if imitator:
            # update_imitator (bcq_impl.py:148-161)
            mlp.forward(impl.vae_enc, st, self.x_q.data_ptr(), True, self.LX1, self.ve_acts,
                        out_parts=self.pe, xgen=self.r_q, xgen_keep=True, philox=ph)
            ops.call_desc("d3a_bcq_vae_sample", self.vae_desc)
            mlp.forward(impl.vae_dec, st, self.x_vd.data_ptr(), True, self.LX2, self.vd_acts,
                        out_parts=self.pd)
            ops.call_desc("d3a_bcq_vae_loss", self.vae_desc)
            mlp.backward(self.vd_bwd, st, self.x_vd.data_ptr(), True, self.LX2, self.vd_acts,
                         self.dhead_d.data_ptr(), A, B * A, 0, B, dx=self.dx_vd)
            ops.call_desc("d3a_bcq_vae_enc_grad", self.vae_desc)
            mlp.backward(self.ve_bwd, st, self.x_q.data_ptr(), True, self.LX1, self.ve_acts,
                         self.dhead_e.data_ptr(), 2 * L, B * 2 * L, 0, B)
            self.imitator_opt.launch(
                tail=dict(counters=impl.counters, inc_mask=1) if fused_tail else None)
        if branch:
            # forked behind the imitator update, so the side work overlaps the
            # long target pass rather than the imitator chain's small launches
            s1 = self._side(0)
            s1.wait_stream(main)
            with torch.cuda.stream(s1):
                mlp.forward(impl.critic, st, self.x_q.data_ptr(), True, self.LX1, self.q_acts)
            q_pending = True
            if actor:
                s2 = self._side(1)
                s2.wait_stream(main)
                with torch.cuda.stream(s2):
                    self._actor_prefix()
                a_pending = True
        if critic:
            # compute_target (bcq_impl.py:215-226) over B*N sampled actions
            mlp.forward(impl.vae_dec, st, self.x_td.data_ptr(), True, self.LX2, self.td_acts,
                        keep_h=False, xgen=self.r_td)
            mlp.forward(impl.policy, tg, self.x_tp.data_ptr(), True, self.LX1, self.tp_acts,
                        keep_h=False, xgen=self.r_tp)
            means = mlp.forward(impl.critic, tg, self.x_tq.data_ptr(), True, self.LX1,
                                self.tq_acts, keep_h=False, row_mean=self.tq_means,
                                xgen=self.r_tq)
            self.target_desc.means = self.tq_means.data_ptr() if means else None
            q = self.qr_desc
            if means and _FUSED_TARGET:
                # the loss launch forms the target rows (d3a_bcq_target's
                # arithmetic) from the means and quantiles
                t = self.target_desc
                q.tg_q, q.tg_means, q.tg_N, q.tg_C, q.tg_lam = t.q, t.means, t.N, t.C, t.lam
            else:
                q.tg_means = None
                ops.call_desc("d3a_bcq_target", self.target_desc)
            # update_critic (ddpg_impl.py:138-165) with the quantile Huber loss
            if q_pending:
                main.wait_stream(self._side(0))
            else:
                mlp.forward(impl.critic, st, self.x_q.data_ptr(), True, self.LX1, self.q_acts)
            ops.call_desc("d3a_bcq_qr_loss", self.qr_desc)
            mlp.backward(self.cbwd, st, self.x_q.data_ptr(), True, self.LX1, self.q_acts,
                         self.dq.data_ptr(), K, B * K, 0, B)
            self.critic_opt.launch(
                tail=dict(targ=tg, tau=impl._tau, counters=impl.counters, inc_mask=2, step_add=0)
                if fused_tail else None)
        if actor:
            # compute_actor_loss (bcq_impl.py:132-146)
            if a_pending:
                main.wait_stream(self._side(1))
            else:
                self._actor_prefix()
            # (its rows built while staged: only dx is taken from this pass)
            mlp.forward(impl.critic, st, self.x_qa.data_ptr(), True, self.LX1, self.qa_acts,
                        members=1, xgen=self.r_qa)
            mlp.backward(self.abwd, st, self.x_qa.data_ptr(), True, self.LX1, self.qa_acts,
                         self.dconst.data_ptr(), K, B * K, 0, B, weight_grads=False, dx=self.adx,
                         members=1)
            ops.call_desc("d3a_bcq_actor_head", self.actor_desc)
            mlp.backward(self.pbwd, st, self.x_pa.data_ptr(), True, self.LX1, self.pa_acts,
                         self.dhead_pi.data_ptr(), A, B * A, 0, B)
            self.actor_opt.launch(
                tail=dict(targ=tg, tau=impl._tau, counters=impl.counters, inc_mask=4, step_add=0,
                          metrics=self.metrics, ring=self.ring, ring_ctr=self.ring_ctr)
                if fused_tail else None)
        if fused_tail:
            return
        s0, s1 = impl.soft_span
        mask = (1 if critic else 0) | (2 if actor else 0) | (4 if imitator else 0)
        ops.step_end(impl.counters, mask, self.metrics, self.ring, self.ring_ctr,
                     tg.data[s0:s1] if targets else None, st.data[s0:s1] if targets else None,
                     impl._tau)
