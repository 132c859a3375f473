"""CQLImpl on HIP kernels — drop-in for d3rlpy/algos/torch/cql_impl.py:21-243.

Same constructor arguments, same ``update_temp / update_alpha /
update_critic / update_actor / update_critic_target / update_actor_target``
methods and return types; plus ``update_step`` which runs the whole
``CQL._update`` schedule (algos/cql.py:234-258) as one device-side pipeline
(and, after the first call, as one HIP-graph replay).

Pipeline of one update_step (all on the current stream, no host sync):
  1  policy trunk+head on [obs; next_obs]  (2B rows; the policy is unchanged
     until update_actor, so this one evaluation serves update_temp,
     update_alpha, the critic's conservative term and target, and the actor)
  2  d3a_cql_sample: every action sample, log-prob and Q-input row
  3  critic ensemble forward over 6NB+B rows (alpha set | critic set | data)
     and the target ensemble over B rows
  4  d3a_cql_loss: temperature Adam, alpha Adam, TD target, dL/dQ per row
  5  critic backward over the 3NB+B critic rows, Adam (critic)
  6  critic forward at (s, tanh u) with the new critic, dQ/da, policy-head
     gradient, policy backward, Adam (actor)
  7  soft update of both targets (one launch over the flat buffer)

Row layout of the Q-input matrix x_q ([6NB+B][D+A], shared by the C critics):
  set s in {0: update_alpha, 1: update_critic}, rows s*3NB + blk*NB + b*N + n
    blk 0: (obs_b, tanh(mu(obs_b) + eps*std))      _compute_policy_is_values(obs_t, obs_t)
    blk 1: (obs_b, tanh(mu(next_b) + eps*std))     _compute_policy_is_values(obs_tp1, obs_t)
    blk 2: (obs_b, U(-1, 1))                       _compute_random_is_values(obs_t)
  rows 6NB + b: (obs_b, act_b)                     data values / TD error
"""
from __future__ import annotations

import math
import os
from typing import Dict, Optional, Sequence, Tuple

import numpy as np
import torch
from torch import nn

from .. import _native as NAT
from .. import mlp, ops
from .. import checkpoint as ckpt
from ..nets import AdamGroup, EnsembleMLP, GradSpace, OptimState, ParamStore
from .impl_base import DeviceBatch, ImplBase, as_device_batch

METRIC_NAMES = ("temp_loss", "temp", "alpha_loss", "alpha", "critic_loss", "actor_loss",
                "td_loss", "conservative_loss")


# actor phase: Q head + min-over-critics backward in one launch (d3a_head1_min)
_HEAD_MIN = os.environ.get("D3A_HEAD_MIN", "1") == "1"
# actor phase: dQ/da formed in d3a_sac_actor_head from the critic's first-layer
# pre-activation gradient (one input-gradient launch fewer)
_DQ_IN_HEAD = os.environ.get("D3A_DQ_IN_HEAD", "1") == "1"
# actor phase: the critic pass at (s, tanh u) and its backward to the action
# in one launch (d3a_sac_actor_q) for [n_in <= 64, 256, 256, 1] critics
_ACTOR_Q = os.environ.get("D3A_ACTOR_Q", "1") == "1"
_DQ_IN_HEAD_MAX_PAIRS = min(32, int(os.environ.get("D3A_DQ_IN_HEAD_MAX_PAIRS", "8")))
# full update_step: the soft target updates, counters and metric ring ride in
# the two Adam launches (d3a_adam_step) instead of a d3a_step_end launch
_ADAM_TAIL = os.environ.get("D3A_ADAM_TAIL", "1") == "1"
# the CQL loss stage (temperature / alpha Adam, TD, the conservative scale) in
# the slice critic backward's prologue instead of its own one-workgroup launch
# (d3a_q2_bwd_x6_cql; the new scalar state committed by the critic Adam);
# D3A_LOSS_IN_BWD=0 keeps the d3a_cql_loss launch (A/B)
_LOSS_IN_BWD = os.environ.get("D3A_LOSS_IN_BWD", "1") == "1"
# (A/B) the weight images' split jobs in the sampler's launch even where the
# policy forward is the parts path (D3A_SPLIT_IN_SAMPLER=1)
_SPLIT_IN_SAMPLER = os.environ.get("D3A_SPLIT_IN_SAMPLER", "0") == "1"

class CQLImpl(ImplBase):
    # conservative term + alpha (cql_impl.py); SACImpl (algos/sac.py) clears it
    _CONSERVATIVE = True

    def __init__(
        self,
        observation_shape: Sequence[int],
        action_size: int,
        actor_learning_rate: float,
        critic_learning_rate: float,
        temp_learning_rate: float,
        alpha_learning_rate: float,
        actor_optim_factory,
        critic_optim_factory,
        temp_optim_factory,
        alpha_optim_factory,
        actor_encoder_factory,
        critic_encoder_factory,
        q_func_factory,
        gamma: float,
        tau: float,
        n_critics: int,
        initial_temperature: float,
        initial_alpha: float,
        alpha_threshold: float,
        conservative_weight: float,
        n_action_samples: int,
        soft_q_backup: bool,
        use_gpu,
        scaler,
        action_scaler,
        reward_scaler,
    ):
        super().__init__(observation_shape, action_size, scaler, action_scaler, reward_scaler,
                         use_gpu)
        if q_func_factory.get_type() != "mean":
            raise NotImplementedError("CQL on HIP supports the 'mean' Q function")
        if len(observation_shape) != 1:
            raise NotImplementedError("CQL on HIP supports vector observations")
        if scaler is not None and scaler.get_type() != "standard":
            raise NotImplementedError("the HIP CQLImpl supports the 'standard' scaler")
        if action_scaler is not None or reward_scaler is not None:
            raise NotImplementedError("action/reward scalers are out of scope (SURVEY §2 #4)")
        self._actor_learning_rate = actor_learning_rate
        self._critic_learning_rate = critic_learning_rate
        self._temp_learning_rate = temp_learning_rate
        self._alpha_learning_rate = alpha_learning_rate
        self._actor_optim_factory = actor_optim_factory
        self._critic_optim_factory = critic_optim_factory
        self._temp_optim_factory = temp_optim_factory
        self._alpha_optim_factory = alpha_optim_factory
        self._actor_encoder_factory = actor_encoder_factory
        self._critic_encoder_factory = critic_encoder_factory
        self._q_func_factory = q_func_factory
        self._gamma = gamma
        self._tau = tau
        self._n_critics = n_critics
        self._initial_temperature = initial_temperature
        self._initial_alpha = initial_alpha
        self._alpha_threshold = alpha_threshold
        self._conservative_weight = conservative_weight
        self._n_action_samples = n_action_samples
        self._soft_q_backup = soft_q_backup
        self._min_logstd, self._max_logstd = -20.0, 2.0
        self._built = False
        self._ws: Dict[int, "_Workspace"] = {}
        self._dp = None

    # ------------------------------------------------------------------ build
    def build(self) -> None:
        dev = self.torch_device
        D, A, C = self._observation_shape[0], self._action_size, self._n_critics
        hq = list(self._critic_encoder_factory.hidden_units)
        hp = list(self._actor_encoder_factory.hidden_units)
        store = ParamStore()
        # critic first, then policy: mirrors DDPGBaseImpl.build order (ddpg_impl.py:95-111)
        self.critic = EnsembleMLP(store, "q", C, [D + A] + hq + [1])
        self.policy = EnsembleMLP(store, "pi", 1, [D] + hp + [2 * A])
        store.allocate(dev)
        self.store = store
        self._init_like_reference()
        self.targ = store.like()
        self.targ.data.copy_(store.data)
        # scalar parameters: log_temp, log_alpha (create_parameter((1,1), log(v)))
        self.log_temp = torch.full((1,), math.log(self._initial_temperature), device=dev)
        self.log_alpha = torch.full((1,), math.log(self._initial_alpha), device=dev)
        self.temp_m = torch.zeros(1, device=dev)
        self.temp_v = torch.zeros(1, device=dev)
        self.temp_step = torch.zeros(1, dtype=torch.int64, device=dev)
        self.alpha_m = torch.zeros(1, device=dev)
        self.alpha_v = torch.zeros(1, device=dev)
        self.alpha_step = torch.zeros(1, dtype=torch.int64, device=dev)
        # optimiser step counts: [0] critic, [1] actor (committed by d3a_step_end)
        self.counters = torch.zeros(8, dtype=torch.int64, device=dev)
        f = self._critic_optim_factory
        self.critic_state = OptimState(store, self.critic.names(), self._critic_learning_rate,
                                       f.betas, f.eps, step=self.counters[0:1])
        f = self._actor_optim_factory
        self.actor_state = OptimState(store, self.policy.names(), self._actor_learning_rate,
                                      f.betas, f.eps, step=self.counters[1:2])
        self._built = True

    # ---------------------------------------------------------- checkpoints
    def _critic_refs(self):
        """EnsembleContinuousQFunction.parameters() order and state-dict keys."""
        refs, L = [], self.critic.n_layers
        for c in range(self._n_critics):
            for l in range(L - 1):
                refs.append((f"_q_funcs.{c}._encoder._fcs.{l}.weight", self.critic.wname(l), c, None))
                refs.append((f"_q_funcs.{c}._encoder._fcs.{l}.bias", self.critic.bname(l), c, None))
            refs.append((f"_q_funcs.{c}._fc.weight", self.critic.wname(L - 1), c, None))
            refs.append((f"_q_funcs.{c}._fc.bias", self.critic.bname(L - 1), c, None))
        return refs

    def _policy_refs(self):
        """SquashedNormalPolicy.parameters() order: encoder fcs, _mu, _logstd."""
        refs, L, A = [], self.policy.n_layers, self._action_size
        for l in range(L - 1):
            refs.append((f"_encoder._fcs.{l}.weight", self.policy.wname(l), 0, None))
            refs.append((f"_encoder._fcs.{l}.bias", self.policy.bname(l), 0, None))
        mu, ls = slice(0, A), slice(A, 2 * A)
        refs += [("_mu.weight", self.policy.wname(L - 1), 0, mu),
                 ("_mu.bias", self.policy.bname(L - 1), 0, mu),
                 ("_logstd.weight", self.policy.wname(L - 1), 0, ls),
                 ("_logstd.bias", self.policy.bname(L - 1), 0, ls)]
        return refs

    def get_state_dict(self) -> Dict[str, dict]:
        """torch_utility.get_state_dict layout of the reference CQLImpl."""
        torch.cuda.synchronize()
        cr, pr = self._critic_refs(), self._policy_refs()
        tf, af = self._temp_optim_factory, self._alpha_optim_factory
        return {
            "_q_func": ckpt.module_state(self.store, cr),
            "_targ_q_func": ckpt.module_state(self.targ, cr),
            "_policy": ckpt.module_state(self.store, pr),
            "_targ_policy": ckpt.module_state(self.targ, pr),
            "_log_temp": {"_parameter": self.log_temp.detach().view(1, 1).cpu().clone()},
            "_log_alpha": {"_parameter": self.log_alpha.detach().view(1, 1).cpu().clone()},
            "_critic_optim": ckpt.adam_state(self.critic_state, cr),
            "_actor_optim": ckpt.adam_state(self.actor_state, pr),
            "_temp_optim": ckpt.scalar_adam_state(self.temp_m, self.temp_v, self.temp_step,
                                                  self._temp_learning_rate, tf.betas, tf.eps),
            "_alpha_optim": ckpt.scalar_adam_state(self.alpha_m, self.alpha_v, self.alpha_step,
                                                   self._alpha_learning_rate, af.betas, af.eps),
        }

    def set_state_dict(self, sd: Dict[str, dict]) -> None:
        cr, pr = self._critic_refs(), self._policy_refs()
        ckpt.load_module_state(self.store, cr, sd["_q_func"])
        ckpt.load_module_state(self.targ, cr, sd["_targ_q_func"])
        ckpt.load_module_state(self.store, pr, sd["_policy"])
        ckpt.load_module_state(self.targ, pr, sd["_targ_policy"])
        with torch.no_grad():
            self.log_temp.copy_(torch.as_tensor(sd["_log_temp"]["_parameter"]).view(-1))
            self.log_alpha.copy_(torch.as_tensor(sd["_log_alpha"]["_parameter"]).view(-1))
        ckpt.load_adam_state(self.critic_state, cr, sd["_critic_optim"])
        ckpt.load_adam_state(self.actor_state, pr, sd["_actor_optim"])
        ckpt.load_scalar_adam_state(self.temp_m, self.temp_v, self.temp_step, sd["_temp_optim"])
        ckpt.load_scalar_adam_state(self.alpha_m, self.alpha_v, self.alpha_step,
                                    sd["_alpha_optim"])
        torch.cuda.synchronize()

    def save_model(self, fname: str) -> None:
        torch.save(self.get_state_dict(), fname)

    def load_model(self, fname: str) -> None:
        self.set_state_dict(torch.load(fname, map_location="cpu", weights_only=True))

    def _init_like_reference(self) -> None:
        """nn.Linear default init in the reference construction order."""
        D, A, C = self._observation_shape[0], self._action_size, self._n_critics
        hq = list(self._critic_encoder_factory.hidden_units)
        hp = list(self._actor_encoder_factory.hidden_units)
        with torch.random.fork_rng(devices=[]):
            for c in range(C):
                sizes = [D + A] + hq
                for l in range(len(hq)):
                    self.critic.load_linear(l, c, nn.Linear(sizes[l], sizes[l + 1]))
                self.critic.load_linear(len(hq), c, nn.Linear(hq[-1], 1))
            sizes = [D] + hp
            for l in range(len(hp)):
                self.policy.load_linear(l, 0, nn.Linear(sizes[l], sizes[l + 1]))
            mu, ls = nn.Linear(hp[-1], A), nn.Linear(hp[-1], A)
            Wh, bh = self.policy.export_linear(len(hp), 0)
            with torch.no_grad():
                Wh[:A].copy_(mu.weight)
                Wh[A:].copy_(ls.weight)
                bh[:A].copy_(mu.bias)
                bh[A:].copy_(ls.bias)

    # ------------------------------------------------------- data parallel
    def enable_data_parallel(self, dp) -> None:
        """Average every gradient over the ranks of ``dp`` (d3rlpy_amd.dp,
        K4): call after build() on every rank, before the first update.
        Rank 0's parameters are broadcast so all replicas start identical."""
        if self._ws:
            raise RuntimeError("enable_data_parallel must precede the first update")
        self._dp = dp
        dp.broadcast_(self.store.data)
        dp.broadcast_(self.targ.data)
        dp.broadcast_(self.log_temp)
        dp.broadcast_(self.log_alpha)

    # ------------------------------------------------------------- workspace
    def _workspace(self, B: int) -> "_Workspace":
        ws = self._ws.get(B)
        if ws is None:
            ws = _Workspace(self, B)
            self._ws[B] = ws
        return ws

    # --------------------------------------------------------------- updates
    def update_step(self, batch, noise: Optional[Dict[str, torch.Tensor]] = None,
                    sync: bool = True, use_graph: bool = True):
        """Whole CQL._update: temp, alpha, critic, actor, both target updates."""
        flags = (self._temp_learning_rate > 0, self._alpha_learning_rate > 0, True, True, True)
        return self._run(batch, flags, noise, sync, use_graph)

    def update_temp(self, batch) -> Tuple[np.ndarray, np.ndarray]:
        m = self._run(batch, (True, False, False, False, False), None, True, False)
        return np.float32(m["temp_loss"]), np.float32(m["temp"])

    def update_alpha(self, batch) -> Tuple[np.ndarray, np.ndarray]:
        m = self._run(batch, (False, True, False, False, False), None, True, False)
        return np.float32(m["alpha_loss"]), np.float32(m["alpha"])

    def update_critic(self, batch) -> np.ndarray:
        m = self._run(batch, (False, False, True, False, False), None, True, False)
        return np.float32(m["critic_loss"])

    def update_actor(self, batch) -> np.ndarray:
        m = self._run(batch, (False, False, False, True, False), None, True, False)
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
        if self._dp is not None:
            vals = vals * np.float32(self._dp.scale)  # summed over ranks in the pipeline
        return {k: float(v) for k, v in zip(METRIC_NAMES, vals)}

    # ------------------------------------------------- device-side batches
    def staging_batch(self, batch_size: int) -> DeviceBatch:
        """DeviceBatch whose tensors ARE this Impl's input buffers: a gather
        into it feeds update_step with zero copies."""
        ws = self._workspace(batch_size)
        B = batch_size
        return DeviceBatch(ws.obs2[:B], ws.act, ws.rew, ws.obs2[B:], ws.term, ws.nsteps)

    def active_metric_names(self):
        names = []
        if self._temp_learning_rate > 0:
            names += ["temp_loss", "temp"]
        if self._alpha_learning_rate > 0:
            names += ["alpha_loss", "alpha"]
        return names + ["critic_loss", "actor_loss"]

    def metrics_ring(self, n_steps: int):
        for ws in self._ws.values():
            ws.ring_ctr.zero_()
        return n_steps

    def read_metrics_ring(self, handle):
        names = self.active_metric_names()
        if not self._ws:
            return names, np.zeros((0, len(names)), dtype=np.float32)
        ws = self._last_ws()
        cnt = int(ws.ring_ctr.item())
        k = min(cnt, ws.ring.shape[0])
        vals = ws.ring[:k].cpu().numpy()
        cols = [METRIC_NAMES.index(n) for n in names]
        return names, vals[:, cols]

    # ------------------------------------------------------------- inference
    def _policy_head(self, x: torch.Tensor) -> torch.Tensor:
        B = x.shape[0]
        acts = mlp.Acts.alloc(self.policy, B, self.torch_device)
        x = x.contiguous().float()
        mlp.forward(self.policy, self.store, x.data_ptr(), True, x.shape[1], acts)
        return acts.out[0]

    def _policy_module(self) -> nn.Module:
        from ..export import TanhMeanPolicy, mlp_module
        return TanhMeanPolicy(mlp_module(self.policy, self.store), self._action_size)

    def _predict_best_action(self, x: torch.Tensor) -> torch.Tensor:
        A = self._action_size
        return torch.tanh(self._policy_head(x)[:, :A])

    def _sample_action(self, x: torch.Tensor) -> torch.Tensor:
        A = self._action_size
        h = self._policy_head(x)
        std = h[:, A:].clamp(self._min_logstd, self._max_logstd).exp()
        return torch.tanh(h[:, :A] + torch.randn_like(std) * std)

    def _predict_value(self, x: torch.Tensor, action: torch.Tensor) -> torch.Tensor:
        xa = torch.cat([x.float(), action.float()], dim=1).contiguous()
        acts = mlp.Acts.alloc(self.critic, xa.shape[0], self.torch_device)
        mlp.forward(self.critic, self.store, xa.data_ptr(), True, xa.shape[1], acts)
        return acts.out  # [C][B]

    # ------------------------------------------------------------ inspection
    def critic_grad(self, name: str) -> torch.Tensor:
        return self._last_ws().critic_opt.grad(name)

    def policy_grad(self, name: str) -> torch.Tensor:
        return self._last_ws().actor_opt.grad(name)

    def _last_ws(self) -> "_Workspace":
        return next(iter(self._ws.values()))


class _Workspace:
    """Every device buffer of one update at batch size B (graph-capture safe)."""

    def __init__(self, impl: CQLImpl, B: int):
        dev = impl.torch_device
        self.impl = impl
        D, A, C = impl._observation_shape[0], impl._action_size, impl._n_critics
        # SAC (no conservative term) draws no importance samples: N = 0
        N = impl._n_action_samples if impl._CONSERVATIVE else 0
        self.B, self.D, self.A, self.C, self.N = B, D, A, C, N
        self.soft = bool(impl._soft_q_backup)
        NB = N * B
        self.NB = NB
        self.R = 6 * NB + B
        DA = D + A
        # Q-input rows padded to a multiple of 4 floats: 16-byte aligned rows let
        # the first-layer GEMMs use vector loads (the pad columns stay zero)
        self.LDX = LDX = (DA + 3) // 4 * 4
        z = lambda *s: torch.zeros(*s, dtype=torch.float32, device=dev)  # noqa: E731
        # staged batch: obs2 = [obs; next_obs]; with a standard scaler the
        # pipeline reads its transform xobs2 (d3a_standardize_f32, the
        # TorchMiniBatch scaling of torch_utility.py:179-181), else obs2 itself
        self.obs2 = z(2 * B, D)
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
        self.act = z(B, A)
        self.rew = z(B)
        self.term = z(B)
        self.nsteps = z(B)
        # noise: [eps_temp | eps_pi (2 sets x 2 x N x B x A) | eps_actor | eps_targ
        # (soft target only) | u_rand (2 x NB x A)]
        nt = B * A if self.soft else 0
        self.n_normal = (B + 4 * NB + B) * A + nt
        self.n_uniform = 2 * NB * A
        self.noise = z(self.n_normal + self.n_uniform)
        o = 0
        self.eps_temp = self.noise[o:o + B * A]; o += B * A
        self.eps_pi = self.noise[o:o + 4 * NB * A]; o += 4 * NB * A
        self.eps_actor = self.noise[o:o + B * A]; o += B * A
        self.eps_targ = self.noise[o:o + nt]; o += nt
        self.u_rand = self.noise[o:o + 2 * NB * A]
        # Philox counter of the step's draws (d3a_cql_sample draws them; the
        # step-end kernel advances it as counter slot 4)
        self.rng_ctr = impl.counters[4:5]
        self.seed = int(torch.randint(0, 2**62, (1,)).item())
        if impl._dp is not None:
            # rank 0's seed with the rank folded in: distinct noise per shard
            self.seed = impl._dp.rank_seed(self.seed)
        # policy forward on 2B rows
        self.pacts = mlp.Acts.alloc(impl.policy, 2 * B, dev)
        # the policy head as unit-part partial sums (d3a_mlp_fwd parts), summed
        # by the sampler and the actor head
        self.phead = (torch.zeros(NAT.MLP_PARTS, 1, 2 * B, 2 * A, dtype=torch.float32, device=dev)
                      if mlp.parts_ok(impl.policy) and impl.policy.C == 1 else None)
        # sample outputs
        self.x_q = z(self.R, LDX)
        self.x_targ = z(B, LDX)
        self.x_actor = z(B, LDX)
        self.logp_temp = z(B)
        self.logp_is = z(4 * NB)
        self.actor_u = z(B, A)
        self.actor_logp = z(B)
        self.logp_targ = z(B)
        # critic / target / actor-critic activations
        # bf16 throughput line (ops.CRITIC_PRECISION): the critic pass's kept
        # activations in bf16 select the bf16 forward / backward kernels
        bf16 = (ops.CRITIC_PRECISION == "bf16h" and mlp.q2_shape(impl.critic)
                and mlp.q2_ok(impl.critic, 3 * NB + B))
        self.qacts = mlp.Acts.alloc(impl.critic, self.R, dev,
                                    dtype=torch.bfloat16 if bf16 else torch.float32,
                                    with_mask=not bf16 and mlp.q2_shape(impl.critic))
        self.tacts = mlp.Acts.alloc(impl.critic, B, dev)
        self.aacts = mlp.Acts.alloc(impl.critic, B, dev)
        # the critic forward's W0 / W1 as split-bf16 operand images of the
        # online critics and their targets, formed from the step's weights by
        # the sampler's launch (d3a_cql_sample_desc.presplit) -- no launch of
        # their own, and no per-workgroup split in the forward
        self.wimg = (mlp.WeightImages(impl.critic, (impl.store, impl.targ), dev)
                     if mlp.presplit_ok(impl.critic) and not bf16 else None)
        # (the three-hidden-layer critic: its 256 x 256 stream matrices W1 / W2)
        if (self.wimg is None and not bf16 and mlp._X6_DEEP3 and mlp.x6_deep3_shape(impl.critic)
                and mlp.wide_presplit_ok(impl.critic)):
            self.wimg = mlp.WeightImages(impl.critic, (impl.store, impl.targ), dev, streams=True)
        self.dq = z(C, self.R)
        self.lse = z(2, C, B)
        # (loss stage in the critic backward) squared TD errors, the Adam bias
        # corrections and the staged scalar optimiser state
        self.td2 = z(C, B)
        self.bc = torch.zeros(4, dtype=torch.float64, device=dev)
        self.stage_s = z(8)
        self.adq = z(C, B)
        self.adx = z(C, B, DA)
        self.dhead = z(B, 2 * A)
        self.metrics = z(len(METRIC_NAMES))
        self.scalars = z(4)
        self.scalar_grads = z(2)  # data parallel: temp / alpha gradients
        # per-step metric history (read back once per epoch by the fitter)
        self.ring = z(1 << 16, len(METRIC_NAMES))
        self.ring_ctr = torch.zeros(1, dtype=torch.int64, device=dev)
        # backward spaces + optimisers
        self.Rc = 3 * NB + B
        self.cgrads = GradSpace(dev)
        # the critic backward reads rows [3NB, R): the slice kernel where it
        # applies (then the critic forward keeps h[0] and the mask bits only)
        self.cbwd = mlp.BackwardSpace(impl.critic, self.Rc, self.cgrads, dev, slice_r0=3 * NB)
        self.qacts.no_last_h = self.cbwd.slice
        self.abwd = mlp.BackwardSpace(impl.critic, B, None, dev)
        self.pgrads = GradSpace(dev)
        # the policy head's weight / bias gradients come from
        # d3a_sac_actor_head as one partial per batch row (see head_dz below)
        self.head_dz = not mlp._FUSED_BWD and impl.policy.sizes[-2] <= 256
        self.pbwd = mlp.BackwardSpace(impl.policy, B, self.pgrads, dev,
                                      head_partials=B if self.head_dz else None)
        assert not (self.head_dz and self.pbwd.fused)
        self.critic_opt = AdamGroup(impl.critic_state, self.cgrads)
        self.actor_opt = AdamGroup(impl.actor_state, self.pgrads)
        # share optimiser state across workspaces of other batch sizes
        prev = [w for w in impl._ws.values()]
        if prev:
            raise NotImplementedError("one batch size per CQLImpl is supported")
        self._graphs: Dict[Tuple, torch.cuda.CUDAGraph] = {}
        self._op_state = None  # tensors the update-step op declares mutated
        self._loss_in_bwd = False  # the last enqueue ran the loss stage in the backward
        self._ran_eager = set()
        self._build_descs()

    def _build_descs(self):
        impl = self.impl
        s = NAT.CqlSampleDesc()
        s.head = self.pacts.out.data_ptr()
        if self.phead is not None:
            s.head, s.head_parts, s.s_head_part = (self.phead.data_ptr(), NAT.MLP_PARTS,
                                                   2 * self.B * 2 * self.A)
        s.obs = self.xobs2.data_ptr()
        s.next_obs = self.xobs2.data_ptr() + 4 * self.B * self.D
        s.act = self.act.data_ptr()
        s.eps_temp = self.eps_temp.data_ptr()
        s.eps_pi = self.eps_pi.data_ptr()
        s.u_rand = self.u_rand.data_ptr()
        s.eps_actor = self.eps_actor.data_ptr()
        s.x_q, s.x_targ, s.x_actor = (self.x_q.data_ptr(), self.x_targ.data_ptr(),
                                      self.x_actor.data_ptr())
        s.logp_temp, s.logp_is = self.logp_temp.data_ptr(), self.logp_is.data_ptr()
        s.actor_u, s.actor_logp = self.actor_u.data_ptr(), self.actor_logp.data_ptr()
        s.B, s.D, s.A, s.N = self.B, self.D, self.A, self.N
        s.ldx = self.LDX
        s.min_logstd, s.max_logstd = impl._min_logstd, impl._max_logstd
        s.soft_target = int(self.soft)
        s.noise_base, s.rng_ctr = self.noise.data_ptr(), self.rng_ctr.data_ptr()
        s.eps_actor_out, s.seed, s.n_normal = self.eps_actor.data_ptr(), self.seed, self.n_normal
        if self.soft:
            s.eps_targ, s.logp_targ = self.eps_targ.data_ptr(), self.logp_targ.data_ptr()
        # the weight images' split jobs ride in the policy forward's launch
        # (extra workgroups on the CUs its few hundred rows leave idle) where
        # it is the parts path, else in the sampler's
        self.presplit_jobs = None
        if self.wimg is not None:
            if self.phead is not None and not _SPLIT_IN_SAMPLER:
                self.presplit_jobs = self.wimg.jobs()
            else:
                s.presplit = self.wimg.jobs()
        self.sample_desc = s

        l = NAT.CqlLossDesc()
        l.q, l.q_targ = self.qacts.out.data_ptr(), self.tacts.out.data_ptr()
        l.logp_temp, l.logp_is = self.logp_temp.data_ptr(), self.logp_is.data_ptr()
        l.rew, l.term, l.n_steps = self.rew.data_ptr(), self.term.data_ptr(), self.nsteps.data_ptr()
        l.log_temp, l.temp_m, l.temp_v, l.temp_step = (impl.log_temp.data_ptr(),
                                                       impl.temp_m.data_ptr(),
                                                       impl.temp_v.data_ptr(),
                                                       impl.temp_step.data_ptr())
        l.log_alpha, l.alpha_m, l.alpha_v, l.alpha_step = (impl.log_alpha.data_ptr(),
                                                           impl.alpha_m.data_ptr(),
                                                           impl.alpha_v.data_ptr(),
                                                           impl.alpha_step.data_ptr())
        l.dq, l.metrics, l.scalars = (self.dq.data_ptr(), self.metrics.data_ptr(),
                                      self.scalars.data_ptr())
        l.lse = self.lse.data_ptr()
        # the logsumexp and loss stages as one launch (a zeroed device ticket the
        # last stage-A workgroup counts on and resets) with D3A_LOSS_FUSED=1 --
        # off by default: bitwise equal but measured 35.4 us against 5.3 + 9.5
        # for the pair (K2 5,676 vs 6,376 steps/s): the device-scope release
        # fence each of the 64 workgroups needs before counting itself writes
        # back its XCD's L2 (eight L2s, not coherent with each other)
        self.loss_ticket = torch.zeros(1, dtype=torch.int32, device=self.lse.device)
        if os.environ.get("D3A_LOSS_FUSED", "0") == "1":
            l.ticket = self.loss_ticket.data_ptr()
        l.B, l.A, l.N, l.C, l.R = self.B, self.A, self.N, self.C, self.R
        l.gamma = impl._gamma
        tf, af = impl._temp_optim_factory, impl._alpha_optim_factory
        l.temp_lr, l.alpha_lr = impl._temp_learning_rate, impl._alpha_learning_rate
        # both scalar optimisers are AdamFactory instances with the same defaults
        assert tuple(tf.betas) == tuple(af.betas) and tf.eps == af.eps
        l.beta1, l.beta2, l.adam_eps = tf.betas[0], tf.betas[1], tf.eps
        l.alpha_threshold = impl._alpha_threshold
        l.conservative_weight = impl._conservative_weight
        l.scalar_grads = self.scalar_grads.data_ptr()
        l.grad_scale = 1.0 if impl._dp is None else impl._dp.scale
        l.soft_target, l.conservative = int(self.soft), int(impl._CONSERVATIVE)
        l.logp_targ = self.logp_targ.data_ptr()
        l.td2, l.bc, l.stage = self.td2.data_ptr(), self.bc.data_ptr(), self.stage_s.data_ptr()
        self.loss_desc = l

        h = NAT.SacActorHeadDesc()
        h.head = self.pacts.out.data_ptr()
        if self.phead is not None:
            h.head, h.head_parts, h.s_head_part = (self.phead.data_ptr(), NAT.MLP_PARTS,
                                                   2 * self.B * 2 * self.A)
        h.eps = self.eps_actor.data_ptr()
        h.u = self.actor_u.data_ptr()
        h.logp = self.actor_logp.data_ptr()
        h.dq_da = self.adx.data_ptr()
        h.ld_da, h.da_off, h.sda_c = self.D + self.A, self.D, self.B * (self.D + self.A)
        h.q, h.sqc = self.aacts.out.data_ptr(), self.B
        h.scalars = self.scalars.data_ptr()
        h.dhead, h.metrics = self.dhead.data_ptr(), self.metrics.data_ptr()
        h.B, h.A, h.C = self.B, self.A, self.C
        h.min_logstd, h.max_logstd = impl._min_logstd, impl._max_logstd
        # the policy head's input gradient goes straight into the trunk
        # backward's first dz buffer (per-layer backward path)
        if self.head_dz:
            pol = impl.policy
            Lp = pol.n_layers
            h.w_head = pol.W(Lp - 1, impl.store)
            h.h, h.ldh = self.pacts.h[Lp - 2].data_ptr(), pol.sizes[Lp - 1]
            h.dz, h.lddz = self.pbwd.dz[0].data_ptr(), self.pbwd.dz[0].shape[2]
            h.H = pol.sizes[Lp - 1]
            h.dW_part = self.pgrads.get(pol.wname(Lp - 1)).data_ptr()
            h.db_part = self.pgrads.get(pol.bname(Lp - 1)).data_ptr()
        if self._actor_q_desc() is not None:
            # d3a_sac_actor_q's parts of every member's q and unscaled dQ/da
            B, C, A = self.B, impl.critic.C, self.A
            h.q, h.sqc, h.sq_part = self.aq_q.data_ptr(), B, C * B
            h.dq_da, h.ld_da, h.da_off, h.sda_c = self.aq_j.data_ptr(), A, 0, B * A
            h.sda_part, h.n_part = C * B * A, NAT.ACTOR_Q_PARTS
            h.dq_min, h.dq_scale = 1, -1.0 / B
        self.head_desc = h

    # ---------------------------------------------------------------- inputs
    def stage(self, db: DeviceBatch, noise: Optional[Dict[str, torch.Tensor]]) -> None:
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
            self.set_noise(noise)

    def set_noise(self, nz: Dict[str, torch.Tensor]) -> None:
        """Inject the reference-shaped draws of oracle.cql.CQLNoise (parity mode)."""
        B, A, N, NB = self.B, self.A, self.N, self.NB
        dev = self.noise.device
        g = lambda k: torch.as_tensor(nz[k], dtype=torch.float32).to(dev).contiguous()  # noqa
        self.eps_temp.copy_(g("eps_temp").view(-1))
        ep = self.eps_pi.view(2, 2, N, B, A)
        ep[0, 0].copy_(g("alpha_pi_t").view(N, B, A))
        ep[0, 1].copy_(g("alpha_pi_tp1").view(N, B, A))
        ep[1, 0].copy_(g("critic_pi_t").view(N, B, A))
        ep[1, 1].copy_(g("critic_pi_tp1").view(N, B, A))
        ur = self.u_rand.view(2, NB, A)
        ur[0].copy_(g("alpha_rand").view(NB, A))
        ur[1].copy_(g("critic_rand").view(NB, A))
        self.eps_actor.copy_(g("eps_actor").view(-1))
        if self.soft:
            self.eps_targ.copy_(g("eps_targ").view(-1))

    # ------------------------------------------------------------ roofline
    def _head_min_desc(self):
        """d3a_head1_min descriptor for the actor phase (Q head + its backward
        through min over the critics, one launch), or None where the per-layer
        shapes do not fit it (then rowdot + d3a_head1_bwd)."""
        impl = self.impl
        net = impl.critic
        s = net.sizes
        H, B = s[-2], self.B
        if (s[-1] != 1 or net.n_layers < 2 or H % 4 or H > 256 or net.C > 8
                or mlp.fused_ok(net, B) or self.abwd.fused or not _HEAD_MIN):
            return None
        d = getattr(self, "_hm_desc", None)
        if d is None:
            d = NAT.Head1MinDesc()
            d.h, d.shb, d.ldh = self.aacts.h[-1].data_ptr(), self.aacts.R * H, H
            d.w, d.swb = net.W(net.n_layers - 1, impl.store), H
            d.b, d.sbb = net.b(net.n_layers - 1, impl.store), 1
            d.q, d.sqb = self.aacts.out.data_ptr(), self.aacts.R
            d.scale = -1.0 / B
            d.g_out, d.sgb = self.adq.data_ptr(), B
            dz = self.abwd.dz[0]
            d.dz, d.sdzb, d.lddz = dz.data_ptr(), dz.shape[1] * dz.shape[2], dz.shape[2]
            d.rows, d.n, d.C = B, H, net.C
            self._hm_desc = d
        return d

    def dominant_kernel(self):
        """(launch_fn, flops_per_launch, description) of the MFMA-bound hot
        kernel: the critic-ensemble forward over the step's Q rows -- all R =
        6NB+B with update_alpha on, the critic set's 3NB+B otherwise
        (cql.py:244-247) -- with the target ensemble over the B next-state rows
        as its aux pass: the pipeline's d3a_mlp_fwd launch exactly
        (activations kept for rows >= 3NB) -- or its hidden-layer GEMM when the
        per-layer path is in use."""
        impl = self.impl
        net, st = impl.critic, impl.store
        s = net.sizes
        R, C, DA, B = self.R, self.C, self.LDX, self.B
        r0 = 0 if impl._alpha_learning_rate > 0 else 3 * self.NB
        if mlp.fused_ok(net, R - r0):
            def launch():
                mlp.forward(net, st, self.x_q.data_ptr(), True, DA, self.qacts, r0, R,
                            h_from=3 * self.NB,
                            aux=(impl.targ, self.x_targ.data_ptr(), DA, self.tacts),
                            wparts=self.wimg.wparts(0, 1) if self.wimg is not None else None)
            flops = 2 * C * (R - r0 + B) * sum(s[l] * s[l + 1] for l in range(len(s) - 1))
            gemm = "fp32"
            if mlp.q2_shape(net):
                if self.qacts.h[0].dtype == torch.bfloat16:
                    gemm = "bf16, bf16 kept activations"
                elif ops.CRITIC_PRECISION == "bf16":
                    gemm = "bf16 x1"
                elif ops.CRITIC_GEMM == "x6":
                    gemm = ("split-bf16 x6, pre-split W images" if self.wimg is not None
                            else "split-bf16 x6")
            elif (mlp.x6_deep3_shape(net) and mlp._X6_DEEP3 and ops.CRITIC_GEMM == "x6"
                  and (R - r0 + B) * C >= 8192):
                # the three-hidden-layer critic on d3a_mlp_fwd_x6 (register Q head)
                gemm = ("split-bf16 x6, three hidden layers, pre-split W images"
                        if self.wimg is not None else "split-bf16 x6, three hidden layers")
            return launch, flops, (f"d3a_mlp_fwd critic ensemble ({gemm} MFMA): C={C} x "
                                   f"({R - r0} + {B} target) rows x {'-'.join(map(str, s))}")
        H, Hin = s[2], s[1]
        h0, h1 = self.qacts.h[0], self.qacts.h[1]

        def launch():
            ops.linear_fwd(h0.data_ptr(), False, Hin, net.W(1, st), net.b(1, st), h1.data_ptr(),
                           C, R, Hin, H, relu=True, ldy=H, sxb=R * Hin, syb=R * H)
        flops = 2 * C * R * Hin * H
        return launch, flops, f"gemm_f32 critic layer-2 fwd: C={C} x [{R}x{Hin}]@[{Hin}x{H}]"

    def backward_kernel(self):
        """(launch_fn, flops_per_launch, description) of the critic weight-
        gradient backward over the critic set's 3NB+B rows -- the pipeline's
        launch exactly (cql_impl.py:110-125 through ddpg_impl.py:119-133), on
        the forward's kept activations of the last step; None when it is not
        one launch.  FLOPs: dh1 and dW2 (2 C R 256^2 each) + dW1 (2 C R 256
        n_in)."""
        impl = self.impl
        net, st = impl.critic, impl.store
        if not self.cbwd.q2:
            return None
        NB, R, C, DA = self.NB, self.R, self.C, self.LDX
        r0 = 3 * NB

        # (the pipeline's launch: with the loss stage in its prologue when the
        # last update ran it there -- recomputing that step's scalars from the
        # same inputs and the same uncommitted state, so repeated launches
        # write the same values)
        lib = self.loss_desc if self._loss_in_bwd else None

        def launch():
            mlp.backward(self.cbwd, st, self.x_q.data_ptr(), True, DA, self.qacts,
                         self.dq.data_ptr() + 4 * r0, 1, R, r0, self.Rc,
                         g_scale=self.scalars.data_ptr() + 8, n_scaled=3 * NB, cql_loss=lib)
        s = net.sizes
        flops = 2 * C * self.Rc * (2 * s[1] * s[2] + s[0] * s[1])
        kind = ("slice, split-bf16 x3 mask-factored" + (", CQL loss stage in the prologue" if lib
                                                         else "") if self.cbwd.slice else
                "256-row blocks, split-bf16 x3 mask-factored" if ops.CRITIC_GEMM == "x6"
                else "fp32 MFMA")
        return launch, flops, (f"d3a_q2_bwd critic weight gradients ({kind}): C={C} x "
                               f"{self.Rc} rows x {'-'.join(map(str, s))}")

    # ------------------------------------------------------------- pipeline
    def execute(self, flags, use_graph: bool) -> None:
        key = tuple(bool(f) for f in flags) + (self._external_noise,)
        if not use_graph:
            self._enqueue(*flags)
            return
        g = self._graphs.get(key)
        if g is None:
            if key not in self._ran_eager:
                # first call: run eagerly (loads code objects, real update)
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
        ops.replay_update(g, self._op_state, cql=True)

    def _enqueue(self, temp: bool, alpha: bool, critic: bool, actor: bool, targets: bool) -> None:
        impl = self.impl
        B, D, A, C, N, NB, R = self.B, self.D, self.A, self.C, self.N, self.NB, self.R
        DA = self.LDX  # row stride of the (padded) Q-input matrices
        sampled = temp or alpha or critic or actor
        # the sample stage draws the step's noise itself unless it was injected
        self.sample_desc.gen_noise = int(not self._external_noise)
        self.sample_desc.seed = self.seed
        if impl._scaler is not None:
            ops.standardize(self.obs2, self.xobs2, self.sc_mean, self.sc_std, self.sc_eps)
        if sampled:
            # 1. policy on [obs; next_obs]
            mlp.forward(impl.policy, impl.store, self.xobs2.data_ptr(), True, D, self.pacts,
                        out_parts=self.phead, presplit=self.presplit_jobs)
            # 2. samples and Q inputs
            ops.call_desc("d3a_cql_sample", self.sample_desc)
        if alpha or critic:
            # 3. critic forward (alpha set only when update_alpha runs)
            r0 = 0 if alpha else 3 * NB
            # the critic backward reads the activations of rows [3NB, R) only;
            # the target ensemble over the B next-state rows rides in the same
            # launch (aux pass) when the critic is updated
            targ = (impl.targ, self.x_targ.data_ptr(), DA, self.tacts) if critic else None
            mlp.forward(impl.critic, impl.store, self.x_q.data_ptr(), True, DA, self.qacts, r0, R,
                        h_from=3 * NB, aux=targ,
                        wparts=self.wimg.wparts(0, 1) if self.wimg is not None else None)
        dp = impl._dp
        # the loss stage inside the slice critic backward (d3a_q2_bwd_x6_cql)
        loss_in_bwd = (_LOSS_IN_BWD and critic and dp is None and impl._CONSERVATIVE
                       and not self.soft and self.cbwd.slice and not self.loss_desc.ticket)
        self.loss_desc.split = int(loss_in_bwd)
        self._loss_in_bwd = loss_in_bwd
        if temp or alpha or critic:
            l = self.loss_desc
            l.update_temp, l.update_alpha, l.update_critic = int(temp), int(alpha), int(critic)
            if dp is not None and (temp or alpha):
                # scalar gradients -> all-reduce -> Adam + critic stage
                l.dp_phase = 1
                ops.call_desc("d3a_cql_loss", l)
                dp.all_reduce_sum(self.scalar_grads)
                l.dp_phase = 2
                ops.call_desc("d3a_cql_loss", l)
                l.dp_phase = 0
            else:
                ops.call_desc("d3a_cql_loss", l)
        rng = 16 if sampled and not self._external_noise else 0  # counters[4] += 1
        # whole update: Adam launches carry the targets' soft update and the
        # step bookkeeping (critic Adam: counters[1] += 1, so the actor Adam
        # reads its step already advanced; actor Adam: counters[0] and the
        # sampler counter, metric ring)
        fused_tail = _ADAM_TAIL and critic and actor and targets
        mscale = 1.0 if dp is None else dp.scale
        if critic:
            # 5. critic backward on rows [3NB, R) and Adam
            r0 = 3 * NB
            # dq of the 3NB importance-sampled rows is scaled by scalars[2]
            # (alpha-dependent factor from the loss kernel) as it is read
            mlp.backward(self.cbwd, impl.store, self.x_q.data_ptr(), True, DA, self.qacts,
                         self.dq.data_ptr() + 4 * r0, 1, R, r0, self.Rc,
                         g_scale=self.scalars.data_ptr() + 8, n_scaled=3 * NB,
                         cql_loss=self.loss_desc if loss_in_bwd else None)
            tail = None
            if fused_tail:
                tail = dict(targ=impl.targ, tau=impl._tau, counters=impl.counters, inc_mask=2)
            if loss_in_bwd:
                # the backward staged the new temperature / alpha state
                tail = dict(tail or {}, commit_src=self.stage_s,
                            commit_dst=(impl.log_temp, impl.temp_m, impl.temp_v, impl.log_alpha,
                                        impl.alpha_m, impl.alpha_v),
                            commit_step=(impl.temp_step if temp else None,
                                         impl.alpha_step if alpha else None))
            self._apply(self.critic_opt, dp, tail)
        if actor:
            if not (temp or alpha or critic):
                # scalars[0] = exp(log_temp) is produced by the loss kernel
                l = self.loss_desc
                l.update_temp, l.update_alpha, l.update_critic = 0, 0, 0
                ops.call_desc("d3a_cql_loss", l)
            # 6. actor: Q(s, tanh u) with the updated critic, dQ/da, policy backward
            # dL/dq = -1/B on the argmin critic (backward of min over the ensemble)
            aq = self._actor_q_desc()
            hd = self.head_desc
            if aq is not None:
                # every member's q and unscaled dQ_c/da (four parts) in one
                # launch; the actor head sums the parts and applies the min's
                # backward (dq_min, set in _build_descs)
                ops.call_desc("d3a_sac_actor_q", aq)
            else:
                self._actor_critic_layers(B, A, DA)
            # the head's work in the trunk backward's prologue where the
            # shape takes it (d3a_q2_bwd_actor_head), else head then trunk
            fused_head = self.head_dz and mlp.backward(
                self.pbwd, impl.store, self.xobs2.data_ptr(), True, D, self.pacts,
                self.dhead.data_ptr(), 2 * A, 2 * B * 2 * A, 0, B, head_ready=True,
                head_desc=hd) is True
            if not fused_head:
                ops.call_desc("d3a_sac_actor_head", hd)
                mlp.backward(self.pbwd, impl.store, self.xobs2.data_ptr(), True, D, self.pacts,
                             self.dhead.data_ptr(), 2 * A, 2 * B * 2 * A, 0, B,
                             head_ready=self.head_dz)
            tail = None
            if fused_tail:
                if dp is not None:
                    dp.all_reduce_sum(self.metrics)  # logged losses: mean over ranks
                tail = dict(targ=impl.targ, tau=impl._tau, counters=impl.counters,
                            inc_mask=1 | rng, step_add=0, metrics=self.metrics, ring=self.ring,
                            ring_ctr=self.ring_ctr, metric_scale=mscale)
            self._apply(self.actor_opt, dp, tail)
        if fused_tail:
            return
        # 7. soft update of both targets + metric ring + optimiser step counters
        if dp is not None:
            dp.all_reduce_sum(self.metrics)  # logged losses: mean over ranks
        ops.step_end(impl.counters, (1 if critic else 0) | (2 if actor else 0) | rng, self.metrics,
                     self.ring, self.ring_ctr, impl.targ.data if targets else None,
                     impl.store.data if targets else None, impl._tau, metric_scale=mscale)

    def _actor_q_desc(self):
        """d3a_sac_actor_q descriptor (the actor phase's critic pass, forward
        and backward to the action, one launch), or None where the critic's
        shape does not fit it (then the per-layer path)."""
        impl = self.impl
        net = impl.critic
        s = net.sizes
        if (not _ACTOR_Q or len(s) != 4 or s[1] != 256 or s[2] != 256 or s[3] != 1
                or s[0] > 64 or self.A > 16):
            return None
        d = getattr(self, "_aq_desc", None)
        if d is None:
            st = impl.store
            P, B, C, A = NAT.ACTOR_Q_PARTS, self.B, net.C, self.A
            dev = self.x_actor.device
            self.aq_q = torch.zeros(P, C, B, dtype=torch.float32, device=dev)
            self.aq_j = torch.zeros(P, C, B, A, dtype=torch.float32, device=dev)
            d = NAT.SacActorQDesc()
            d.x, d.ldx = self.x_actor.data_ptr(), self.LDX
            d.W0, d.b0 = net.W(0, st), net.b(0, st)
            d.W1, d.b1 = net.W(1, st), net.b(1, st)
            d.wh, d.bh = net.W(2, st), net.b(2, st)
            d.q, d.dq_da = self.aq_q.data_ptr(), self.aq_j.data_ptr()
            d.B, d.C, d.n_in, d.A, d.da_off = B, C, s[0], A, self.D
            self._aq_desc = d
        return d

    def _actor_critic_layers(self, B: int, A: int, DA: int) -> None:
        """The actor phase's critic pass on the per-layer path: forward, the
        Q head and min-over-members backward, input gradients (dQ/da into
        self.adx, or formed by the actor head from the first layer's dz)."""
        impl = self.impl
        hm = self._head_min_desc()
        mlp.forward(impl.critic, impl.store, self.x_actor.data_ptr(), True, DA, self.aacts,
                    skip_head=hm is not None)
        hd = self.head_desc
        hd.dq_dz = None
        if hm is not None:
            # the Q head and its min-over-members backward in one launch
            ops.call_desc("d3a_head1_min", hm)
            net = impl.critic
            # measured: faster than the input-gradient launch for C * A <= 8
            # (K2: 6 pairs), slower for K4's 16 pairs
            fuse = (_DQ_IN_HEAD and net.n_layers >= 2 and net.C <= 4
                    and net.C * A <= _DQ_IN_HEAD_MAX_PAIRS and net.sizes[1] <= 256)
            dz0 = mlp.backward(self.abwd, impl.store, self.x_actor.data_ptr(), True, DA,
                               self.aacts, self.adq.data_ptr(), 1, B, 0, B,
                               weight_grads=False, dx=None if fuse else self.adx,
                               head_ready=True)
            if fuse:
                # dQ/da from the first layer's pre-activation gradient, in
                # the actor head (the last input-gradient launch is skipped)
                hd.dq_dz, hd.lddqz = dz0.data_ptr(), dz0.shape[2]
                hd.sdz_c = dz0.shape[1] * dz0.shape[2]
                hd.w0, hd.ldw0 = net.W(0, impl.store), net.sizes[0]
                hd.sw0_c, hd.H0 = net.sizes[1] * net.sizes[0], net.sizes[1]
        else:
            mlp.backward(self.abwd, impl.store, self.x_actor.data_ptr(), True, DA,
                         self.aacts, self.adq.data_ptr(), 1, B, 0, B, weight_grads=False,
                         dx=self.adx, q_min=self.aacts.out.data_ptr(), sq_b=B,
                         q_scale=-1.0 / B, g_out=self.adq.data_ptr())

    @staticmethod
    def _apply(opt: AdamGroup, dp, tail: Optional[dict] = None) -> None:
        """Adam; with data parallelism: reduce the split-K partials, SUM
        all-reduce the one gradient copy, Adam on it scaled by 1/world.
        ``tail``: the fused soft update / bookkeeping (AdamGroup.launch)."""
        if dp is None:
            opt.launch(tail=tail)
            return
        opt.reduce()
        dp.all_reduce_sum(opt.grad_span())
        opt.launch(reduced=True, grad_scale=dp.scale, tail=tail)
