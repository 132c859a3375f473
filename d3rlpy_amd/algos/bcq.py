"""BCQ — d3rlpy/algos/bcq.py:20-284 with the HIP BCQImpl.

Constructor arguments and defaults are the reference's (:171-203).  The HIP
Impl implements the quantile-regression critics of the K3 configuration
(``q_func_factory="qr"``); ``_update`` keeps the reference schedule
(:261-279: imitator every step, critic from ``rl_start_step``, actor and both
targets every ``update_actor_interval`` steps) and its metric names.
"""
from __future__ import annotations

from typing import Any, Dict, Optional, Sequence

from ..constants import ActionSpace
from ..factories import AdamFactory, OptimizerFactory, check_encoder, check_q_func, check_use_gpu
from .base import AlgoBase
from .bcq_impl import BCQImpl


class BCQ(AlgoBase):
    def __init__(
        self,
        *,
        actor_learning_rate: float = 1e-3,
        critic_learning_rate: float = 1e-3,
        imitator_learning_rate: float = 1e-3,
        actor_optim_factory: OptimizerFactory = AdamFactory(),
        critic_optim_factory: OptimizerFactory = AdamFactory(),
        imitator_optim_factory: OptimizerFactory = AdamFactory(),
        actor_encoder_factory="default",
        critic_encoder_factory="default",
        imitator_encoder_factory="default",
        q_func_factory="mean",
        batch_size: int = 100,
        n_frames: int = 1,
        n_steps: int = 1,
        gamma: float = 0.99,
        tau: float = 0.005,
        n_critics: int = 2,
        update_actor_interval: int = 1,
        lam: float = 0.75,
        n_action_samples: int = 100,
        action_flexibility: float = 0.05,
        rl_start_step: int = 0,
        beta: float = 0.5,
        use_gpu=True,
        scaler=None,
        action_scaler=None,
        reward_scaler=None,
        impl: Optional[BCQImpl] = None,
        **kwargs: Any,
    ):
        super().__init__(batch_size=batch_size, n_frames=n_frames, n_steps=n_steps, gamma=gamma,
                         scaler=scaler, action_scaler=action_scaler,
                         reward_scaler=reward_scaler, kwargs=kwargs)
        self._actor_learning_rate = actor_learning_rate
        self._critic_learning_rate = critic_learning_rate
        self._imitator_learning_rate = imitator_learning_rate
        self._actor_optim_factory = actor_optim_factory
        self._critic_optim_factory = critic_optim_factory
        self._imitator_optim_factory = imitator_optim_factory
        self._actor_encoder_factory = check_encoder(actor_encoder_factory)
        self._critic_encoder_factory = check_encoder(critic_encoder_factory)
        self._imitator_encoder_factory = check_encoder(imitator_encoder_factory)
        self._q_func_factory = check_q_func(q_func_factory)
        self._tau = tau
        self._n_critics = n_critics
        self._update_actor_interval = update_actor_interval
        self._lam = lam
        self._n_action_samples = n_action_samples
        self._action_flexibility = action_flexibility
        self._rl_start_step = rl_start_step
        self._beta = beta
        self._use_gpu = check_use_gpu(use_gpu)
        self._impl = impl

    def _create_impl(self, observation_shape: Sequence[int], action_size: int) -> None:
        self._impl = BCQImpl(
            observation_shape=observation_shape,
            action_size=action_size,
            actor_learning_rate=self._actor_learning_rate,
            critic_learning_rate=self._critic_learning_rate,
            imitator_learning_rate=self._imitator_learning_rate,
            actor_optim_factory=self._actor_optim_factory,
            critic_optim_factory=self._critic_optim_factory,
            imitator_optim_factory=self._imitator_optim_factory,
            actor_encoder_factory=_resolve(self._actor_encoder_factory, observation_shape),
            critic_encoder_factory=_resolve(self._critic_encoder_factory, observation_shape),
            imitator_encoder_factory=_resolve(self._imitator_encoder_factory, observation_shape),
            q_func_factory=self._q_func_factory,
            gamma=self._gamma,
            tau=self._tau,
            n_critics=self._n_critics,
            lam=self._lam,
            n_action_samples=self._n_action_samples,
            action_flexibility=self._action_flexibility,
            beta=self._beta,
            use_gpu=self._use_gpu,
            scaler=self._scaler,
            action_scaler=self._action_scaler,
            reward_scaler=self._reward_scaler,
        )
        self._impl.build()

    def _flags(self):
        rl = self._grad_step >= self._rl_start_step
        actor = rl and self._grad_step % self._update_actor_interval == 0
        return (True, rl, actor, actor)

    def _update(self, batch) -> Dict[str, float]:
        """algos/bcq.py:261-279 — metric keys as in the reference."""
        flags = self._flags()
        m = self._impl._run(batch, flags, None, True, True)
        out = {"imitator_loss": m["imitator_loss"]}
        if flags[1]:
            out["critic_loss"] = m["critic_loss"]
        if flags[2]:
            out["actor_loss"] = m["actor_loss"]
        return out

    def _update_async(self, batch) -> None:
        self._impl._run(batch, self._flags(), None, False, True)

    def sample_action(self, x):
        """BCQ does not support sampling action."""
        raise NotImplementedError("BCQ does not support sampling action.")

    def get_action_type(self) -> ActionSpace:
        return ActionSpace.CONTINUOUS


def _resolve(factory, observation_shape):
    return factory.resolve(observation_shape) if hasattr(factory, "resolve") else factory
