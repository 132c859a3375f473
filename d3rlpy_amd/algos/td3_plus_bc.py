"""TD3PlusBC — d3rlpy/algos/td3_plus_bc.py:18-195 with the HIP TD3PlusBCImpl.

Constructor arguments and defaults are the reference's (:96-118, including
``scaler="standard"``); ``_update`` keeps the delayed-actor schedule
(:177-192: actor + both targets when ``grad_step % update_actor_interval ==
0``) and metric names, but each step is one fused device pipeline
(TD3PlusBCImpl.update_step).
"""
from __future__ import annotations

from typing import Any, Dict, Optional, Sequence

from ..constants import ActionSpace
from ..factories import AdamFactory, OptimizerFactory, check_encoder, check_q_func, check_use_gpu
from .base import AlgoBase
from .td3_plus_bc_impl import TD3PlusBCImpl


class TD3PlusBC(AlgoBase):
    def __init__(
        self,
        *,
        actor_learning_rate: float = 3e-4,
        critic_learning_rate: float = 3e-4,
        actor_optim_factory: OptimizerFactory = AdamFactory(),
        critic_optim_factory: OptimizerFactory = AdamFactory(),
        actor_encoder_factory="default",
        critic_encoder_factory="default",
        q_func_factory="mean",
        batch_size: int = 256,
        n_frames: int = 1,
        n_steps: int = 1,
        gamma: float = 0.99,
        tau: float = 0.005,
        n_critics: int = 2,
        target_smoothing_sigma: float = 0.2,
        target_smoothing_clip: float = 0.5,
        alpha: float = 2.5,
        update_actor_interval: int = 2,
        use_gpu=True,
        scaler="standard",
        action_scaler=None,
        reward_scaler=None,
        impl: Optional[TD3PlusBCImpl] = None,
        **kwargs: Any,
    ):
        super().__init__(batch_size=batch_size, n_frames=n_frames, n_steps=n_steps, gamma=gamma,
                         scaler=scaler, action_scaler=action_scaler,
                         reward_scaler=reward_scaler, kwargs=kwargs)
        self._actor_learning_rate = actor_learning_rate
        self._critic_learning_rate = critic_learning_rate
        self._actor_optim_factory = actor_optim_factory
        self._critic_optim_factory = critic_optim_factory
        self._actor_encoder_factory = check_encoder(actor_encoder_factory)
        self._critic_encoder_factory = check_encoder(critic_encoder_factory)
        self._q_func_factory = check_q_func(q_func_factory)
        self._tau = tau
        self._n_critics = n_critics
        self._target_smoothing_sigma = target_smoothing_sigma
        self._target_smoothing_clip = target_smoothing_clip
        self._alpha = alpha
        self._update_actor_interval = update_actor_interval
        self._use_gpu = check_use_gpu(use_gpu)
        self._impl = impl

    def _create_impl(self, observation_shape: Sequence[int], action_size: int) -> None:
        self._impl = TD3PlusBCImpl(
            observation_shape=observation_shape,
            action_size=action_size,
            actor_learning_rate=self._actor_learning_rate,
            critic_learning_rate=self._critic_learning_rate,
            actor_optim_factory=self._actor_optim_factory,
            critic_optim_factory=self._critic_optim_factory,
            actor_encoder_factory=_resolve(self._actor_encoder_factory, observation_shape),
            critic_encoder_factory=_resolve(self._critic_encoder_factory, observation_shape),
            q_func_factory=self._q_func_factory,
            gamma=self._gamma,
            tau=self._tau,
            n_critics=self._n_critics,
            target_smoothing_sigma=self._target_smoothing_sigma,
            target_smoothing_clip=self._target_smoothing_clip,
            alpha=self._alpha,
            use_gpu=self._use_gpu,
            scaler=self._scaler,
            action_scaler=self._action_scaler,
            reward_scaler=self._reward_scaler,
        )
        self._impl.build()

    def _actor_step(self) -> bool:
        return self._grad_step % self._update_actor_interval == 0

    def _update(self, batch) -> Dict[str, float]:
        """algos/td3_plus_bc.py:177-192 — metric keys as in the reference."""
        actor = self._actor_step()
        m = self._impl.update_step(batch, update_actor=actor, sync=True)
        out = {"critic_loss": m["critic_loss"]}
        if actor:
            out["actor_loss"] = m["actor_loss"]
        return out

    def _update_async(self, batch) -> None:
        self._impl.update_step(batch, update_actor=self._actor_step(), sync=False)

    def get_action_type(self) -> ActionSpace:
        return ActionSpace.CONTINUOUS


def _resolve(factory, observation_shape):
    return factory.resolve(observation_shape) if hasattr(factory, "resolve") else factory
