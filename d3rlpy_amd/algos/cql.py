"""CQL — d3rlpy/algos/cql.py:22-262 with the HIP CQLImpl.

Constructor arguments and defaults are the reference's (algos/cql.py:139-167);
``_update`` keeps the reference's schedule and metric names
(algos/cql.py:234-258) but runs it as one fused device pipeline
(CQLImpl.update_step).
"""
from __future__ import annotations

from typing import Any, Dict, Optional, Sequence

from ..constants import ActionSpace
from ..factories import AdamFactory, OptimizerFactory, check_encoder, check_q_func, check_use_gpu
from .base import AlgoBase
from .cql_impl import CQLImpl
from .discrete_cql_impl import DiscreteCQLImpl


class CQL(AlgoBase):
    def __init__(
        self,
        *,
        actor_learning_rate: float = 1e-4,
        critic_learning_rate: float = 3e-4,
        temp_learning_rate: float = 1e-4,
        alpha_learning_rate: float = 1e-4,
        actor_optim_factory: OptimizerFactory = AdamFactory(),
        critic_optim_factory: OptimizerFactory = AdamFactory(),
        temp_optim_factory: OptimizerFactory = AdamFactory(),
        alpha_optim_factory: OptimizerFactory = AdamFactory(),
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
        initial_alpha: float = 1.0,
        alpha_threshold: float = 10.0,
        conservative_weight: float = 5.0,
        n_action_samples: int = 10,
        soft_q_backup: bool = False,
        use_gpu=True,
        scaler=None,
        action_scaler=None,
        reward_scaler=None,
        impl: Optional[CQLImpl] = None,
        **kwargs: Any,
    ):
        super().__init__(batch_size=batch_size, n_frames=n_frames, n_steps=n_steps, gamma=gamma,
                         scaler=scaler, action_scaler=action_scaler,
                         reward_scaler=reward_scaler, kwargs=kwargs)
        self._actor_learning_rate = actor_learning_rate
        self._critic_learning_rate = critic_learning_rate
        self._temp_learning_rate = temp_learning_rate
        self._alpha_learning_rate = alpha_learning_rate
        self._actor_optim_factory = actor_optim_factory
        self._critic_optim_factory = critic_optim_factory
        self._temp_optim_factory = temp_optim_factory
        self._alpha_optim_factory = alpha_optim_factory
        self._actor_encoder_factory = check_encoder(actor_encoder_factory)
        self._critic_encoder_factory = check_encoder(critic_encoder_factory)
        self._q_func_factory = check_q_func(q_func_factory)
        self._tau = tau
        self._n_critics = n_critics
        self._initial_temperature = initial_temperature
        self._initial_alpha = initial_alpha
        self._alpha_threshold = alpha_threshold
        self._conservative_weight = conservative_weight
        self._n_action_samples = n_action_samples
        self._soft_q_backup = soft_q_backup
        self._use_gpu = check_use_gpu(use_gpu)
        self._impl = impl

    def _create_impl(self, observation_shape: Sequence[int], action_size: int) -> None:
        self._impl = CQLImpl(
            observation_shape=observation_shape,
            action_size=action_size,
            actor_learning_rate=self._actor_learning_rate,
            critic_learning_rate=self._critic_learning_rate,
            temp_learning_rate=self._temp_learning_rate,
            alpha_learning_rate=self._alpha_learning_rate,
            actor_optim_factory=self._actor_optim_factory,
            critic_optim_factory=self._critic_optim_factory,
            temp_optim_factory=self._temp_optim_factory,
            alpha_optim_factory=self._alpha_optim_factory,
            actor_encoder_factory=_resolve(self._actor_encoder_factory, observation_shape),
            critic_encoder_factory=_resolve(self._critic_encoder_factory, observation_shape),
            q_func_factory=self._q_func_factory,
            gamma=self._gamma,
            tau=self._tau,
            n_critics=self._n_critics,
            initial_temperature=self._initial_temperature,
            initial_alpha=self._initial_alpha,
            alpha_threshold=self._alpha_threshold,
            conservative_weight=self._conservative_weight,
            n_action_samples=self._n_action_samples,
            soft_q_backup=self._soft_q_backup,
            use_gpu=self._use_gpu,
            scaler=self._scaler,
            action_scaler=self._action_scaler,
            reward_scaler=self._reward_scaler,
        )
        self._impl.build()

    def _update(self, batch) -> Dict[str, float]:
        """algos/cql.py:234-258 — metrics keys as in the reference."""
        m = self._impl.update_step(batch, sync=True)
        keys = []
        if self._temp_learning_rate > 0:
            keys += ["temp_loss", "temp"]
        if self._alpha_learning_rate > 0:
            keys += ["alpha_loss", "alpha"]
        keys += ["critic_loss", "actor_loss"]
        return {k: m[k] for k in keys}

    def _update_async(self, batch) -> None:
        self._impl.update_step(batch, sync=False)

    def get_action_type(self) -> ActionSpace:
        return ActionSpace.CONTINUOUS


class DiscreteCQL(AlgoBase):
    """algos/cql.py:265-375 with the HIP DiscreteCQLImpl (IQN Q-function on
    pixels, K5).  Constructor defaults are the reference's (:316-333);
    ``_update`` = DQN._update (algos/dqn.py:127-132): one update, and the
    target hard sync every ``target_update_interval`` steps (folded into the
    update's last launch)."""

    def __init__(
        self,
        *,
        learning_rate: float = 6.25e-5,
        optim_factory: OptimizerFactory = AdamFactory(),
        encoder_factory="default",
        q_func_factory="mean",
        batch_size: int = 32,
        n_frames: int = 1,
        n_steps: int = 1,
        gamma: float = 0.99,
        n_critics: int = 1,
        target_update_interval: int = 8000,
        alpha: float = 1.0,
        use_gpu=True,
        scaler=None,
        reward_scaler=None,
        impl: Optional[DiscreteCQLImpl] = None,
        **kwargs: Any,
    ):
        super().__init__(batch_size=batch_size, n_frames=n_frames, n_steps=n_steps, gamma=gamma,
                         scaler=scaler, action_scaler=None, reward_scaler=reward_scaler,
                         kwargs=kwargs)
        self._learning_rate = learning_rate
        self._optim_factory = optim_factory
        self._encoder_factory = check_encoder(encoder_factory)
        self._q_func_factory = check_q_func(q_func_factory)
        self._n_critics = n_critics
        self._target_update_interval = target_update_interval
        self._alpha = alpha
        self._use_gpu = check_use_gpu(use_gpu)
        self._impl = impl

    def _create_impl(self, observation_shape: Sequence[int], action_size: int) -> None:
        self._impl = DiscreteCQLImpl(
            observation_shape=observation_shape,
            action_size=action_size,
            learning_rate=self._learning_rate,
            optim_factory=self._optim_factory,
            encoder_factory=_resolve(self._encoder_factory, observation_shape),
            q_func_factory=self._q_func_factory,
            gamma=self._gamma,
            n_critics=self._n_critics,
            alpha=self._alpha,
            use_gpu=self._use_gpu,
            scaler=self._scaler,
            reward_scaler=self._reward_scaler,
        )
        self._impl.build()

    def _sync_target(self) -> bool:
        return self._grad_step % self._target_update_interval == 0

    def _update(self, batch) -> Dict[str, float]:
        m = self._impl.update_step(batch, update_target=self._sync_target(), sync=True)
        return {"loss": m["loss"]}

    def _update_async(self, batch) -> None:
        self._impl.update_step(batch, update_target=self._sync_target(), sync=False)

    def get_action_type(self) -> ActionSpace:
        return ActionSpace.DISCRETE


def _resolve(factory, observation_shape):
    return factory.resolve(observation_shape) if hasattr(factory, "resolve") else factory
