"""SAC — d3rlpy/algos/sac.py:19-218 on the HIP tanh-Gaussian actor-critic
pipeline of CQLImpl.

SACImpl (algos/torch/sac_impl.py:27-162) is CQLImpl without the conservative
term and without log_alpha: the critic loss is the plain ensemble TD error
(ddpg_impl.py:154-167) against the soft target
``min_c Q_targ(s', a') - exp(log_temp) * log pi(a'|s')`` with a' a fresh
policy sample at s' (sac_impl.py:148-162).  The pipeline is CQLImpl's with
N = 0 importance samples (x_q holds only the B data rows), the logsumexp
stage skipped and the soft-target sample drawn in ``d3a_cql_sample``.
Constructor arguments and defaults are the reference's (sac.py:118-165);
``_update`` keeps its schedule and metric names (sac.py:195-214).
"""
from __future__ import annotations

import math
from typing import Any, Dict, Optional, Sequence

import torch

from .. import checkpoint as ckpt
from ..constants import ActionSpace
from ..factories import AdamFactory, OptimizerFactory, check_encoder, check_q_func, check_use_gpu
from .base import AlgoBase
from .cql import _resolve
from .cql_impl import CQLImpl


class SACImpl(CQLImpl):
    """algos/torch/sac_impl.py:27-162."""

    _CONSERVATIVE = False

    def __init__(self, observation_shape, action_size, actor_learning_rate,
                 critic_learning_rate, temp_learning_rate, actor_optim_factory,
                 critic_optim_factory, temp_optim_factory, actor_encoder_factory,
                 critic_encoder_factory, q_func_factory, gamma, tau, n_critics,
                 initial_temperature, use_gpu, scaler, action_scaler, reward_scaler):
        super().__init__(
            observation_shape=observation_shape, action_size=action_size,
            actor_learning_rate=actor_learning_rate, critic_learning_rate=critic_learning_rate,
            temp_learning_rate=temp_learning_rate, alpha_learning_rate=0.0,
            actor_optim_factory=actor_optim_factory, critic_optim_factory=critic_optim_factory,
            temp_optim_factory=temp_optim_factory, alpha_optim_factory=temp_optim_factory,
            actor_encoder_factory=actor_encoder_factory,
            critic_encoder_factory=critic_encoder_factory, q_func_factory=q_func_factory,
            gamma=gamma, tau=tau, n_critics=n_critics, initial_temperature=initial_temperature,
            initial_alpha=1.0, alpha_threshold=0.0, conservative_weight=0.0,
            n_action_samples=0, soft_q_backup=True, use_gpu=use_gpu, scaler=scaler,
            action_scaler=action_scaler, reward_scaler=reward_scaler)

    def update_alpha(self, batch):
        raise AttributeError("SACImpl has no update_alpha (sac_impl.py)")

    def update_step(self, batch, noise=None, sync: bool = True, use_graph: bool = True):
        """Whole SAC._update: temp (if its lr > 0), critic, actor, targets."""
        flags = (self._temp_learning_rate > 0, False, True, True, True)
        return self._run(batch, flags, noise, sync, use_graph)

    def active_metric_names(self):
        names = ["temp_loss", "temp"] if self._temp_learning_rate > 0 else []
        return names + ["critic_loss", "actor_loss"]

    def get_state_dict(self) -> Dict[str, dict]:
        """torch_utility.get_state_dict layout of the reference SACImpl
        (no _log_alpha / _alpha_optim)."""
        sd = super().get_state_dict()
        del sd["_log_alpha"], sd["_alpha_optim"]
        return sd

    def set_state_dict(self, sd: Dict[str, dict]) -> None:
        cr, pr = self._critic_refs(), self._policy_refs()
        ckpt.load_module_state(self.store, cr, sd["_q_func"])
        ckpt.load_module_state(self.targ, cr, sd["_targ_q_func"])
        ckpt.load_module_state(self.store, pr, sd["_policy"])
        ckpt.load_module_state(self.targ, pr, sd["_targ_policy"])
        with torch.no_grad():
            self.log_temp.copy_(torch.as_tensor(sd["_log_temp"]["_parameter"]).view(-1))
            self.log_alpha.fill_(math.log(1.0))
        ckpt.load_adam_state(self.critic_state, cr, sd["_critic_optim"])
        ckpt.load_adam_state(self.actor_state, pr, sd["_actor_optim"])
        ckpt.load_scalar_adam_state(self.temp_m, self.temp_v, self.temp_step, sd["_temp_optim"])
        torch.cuda.synchronize()


class SAC(AlgoBase):
    """algos/sac.py:19-218 with the HIP SACImpl."""

    def __init__(
        self,
        *,
        actor_learning_rate: float = 3e-4,
        critic_learning_rate: float = 3e-4,
        temp_learning_rate: float = 3e-4,
        actor_optim_factory: OptimizerFactory = AdamFactory(),
        critic_optim_factory: OptimizerFactory = AdamFactory(),
        temp_optim_factory: OptimizerFactory = AdamFactory(),
        actor_encoder_factory="default",
        critic_encoder_factory="default",
        q_func_factory="mean",
        batch_size: int = 256,
        n_frames: int = 1,
        n_steps: int = 1,
        gamma: float = 0.99,
        tau: float = 0.005,
        n_critics: int = 2,
        initial_temperature: float = 1.0,
        use_gpu=True,
        scaler=None,
        action_scaler=None,
        reward_scaler=None,
        impl: Optional[SACImpl] = None,
        **kwargs: Any,
    ):
        super().__init__(batch_size=batch_size, n_frames=n_frames, n_steps=n_steps, gamma=gamma,
                         scaler=scaler, action_scaler=action_scaler,
                         reward_scaler=reward_scaler, kwargs=kwargs)
        self._actor_learning_rate = actor_learning_rate
        self._critic_learning_rate = critic_learning_rate
        self._temp_learning_rate = temp_learning_rate
        self._actor_optim_factory = actor_optim_factory
        self._critic_optim_factory = critic_optim_factory
        self._temp_optim_factory = temp_optim_factory
        self._actor_encoder_factory = check_encoder(actor_encoder_factory)
        self._critic_encoder_factory = check_encoder(critic_encoder_factory)
        self._q_func_factory = check_q_func(q_func_factory)
        self._tau = tau
        self._n_critics = n_critics
        self._initial_temperature = initial_temperature
        self._use_gpu = check_use_gpu(use_gpu)
        self._impl = impl

    def _create_impl(self, observation_shape: Sequence[int], action_size: int) -> None:
        self._impl = SACImpl(
            observation_shape=observation_shape,
            action_size=action_size,
            actor_learning_rate=self._actor_learning_rate,
            critic_learning_rate=self._critic_learning_rate,
            temp_learning_rate=self._temp_learning_rate,
            actor_optim_factory=self._actor_optim_factory,
            critic_optim_factory=self._critic_optim_factory,
            temp_optim_factory=self._temp_optim_factory,
            actor_encoder_factory=_resolve(self._actor_encoder_factory, observation_shape),
            critic_encoder_factory=_resolve(self._critic_encoder_factory, observation_shape),
            q_func_factory=self._q_func_factory,
            gamma=self._gamma,
            tau=self._tau,
            n_critics=self._n_critics,
            initial_temperature=self._initial_temperature,
            use_gpu=self._use_gpu,
            scaler=self._scaler,
            action_scaler=self._action_scaler,
            reward_scaler=self._reward_scaler,
        )
        self._impl.build()

    def _update(self, batch) -> Dict[str, float]:
        """algos/sac.py:195-214 — metrics keys as in the reference."""
        m = self._impl.update_step(batch, sync=True)
        return {k: m[k] for k in self._impl.active_metric_names()}

    def _update_async(self, batch) -> None:
        self._impl.update_step(batch, sync=False)

    def get_action_type(self) -> ActionSpace:
        return ActionSpace.CONTINUOUS
