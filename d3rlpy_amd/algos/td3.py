"""TD3 and DDPG — d3rlpy/algos/td3.py:19-203 and ddpg.py:19-178 on the HIP
deterministic actor-critic pipeline of TD3PlusBCImpl.

TD3Impl (algos/torch/td3_impl.py:14-78) and DDPGImpl (ddpg_impl.py:232-263)
are TD3PlusBCImpl without the behaviour-cloning term: the actor loss is
-mean Q_0(s, pi(s)) (ddpg_impl.py:244-249).  DDPG's target action is the
target policy's own, clamped to [-1, 1] (ddpg_impl.py:251-260): no smoothing
noise is drawn (sigma = clip = 0 in d3a_td3_target leaves tanh(mu') as is).
Constructor arguments and defaults are the reference's (td3.py:106-130,
ddpg.py:99-121); ``_update`` keeps their schedules and metric names
(td3.py:182-203: actor + both targets every ``update_actor_interval``-th step;
ddpg.py:167-174: all four every step).
"""
from __future__ import annotations

from typing import Any, Dict, Optional, Sequence

from ..constants import ActionSpace
from ..factories import AdamFactory, OptimizerFactory, check_encoder, check_q_func, check_use_gpu
from .base import AlgoBase
from .td3_plus_bc_impl import TD3PlusBCImpl


class TD3Impl(TD3PlusBCImpl):
    """algos/torch/td3_impl.py:14-78: target smoothing, DDPG actor loss."""

    _BC = False

    def __init__(self, observation_shape, action_size, actor_learning_rate, critic_learning_rate,
                 actor_optim_factory, critic_optim_factory, actor_encoder_factory,
                 critic_encoder_factory, q_func_factory, gamma, tau, n_critics,
                 target_smoothing_sigma, target_smoothing_clip, use_gpu, scaler, action_scaler,
                 reward_scaler):
        super().__init__(
            observation_shape=observation_shape, action_size=action_size,
            actor_learning_rate=actor_learning_rate, critic_learning_rate=critic_learning_rate,
            actor_optim_factory=actor_optim_factory, critic_optim_factory=critic_optim_factory,
            actor_encoder_factory=actor_encoder_factory,
            critic_encoder_factory=critic_encoder_factory, q_func_factory=q_func_factory,
            gamma=gamma, tau=tau, n_critics=n_critics,
            target_smoothing_sigma=target_smoothing_sigma,
            target_smoothing_clip=target_smoothing_clip, alpha=0.0, use_gpu=use_gpu,
            scaler=scaler, action_scaler=action_scaler, reward_scaler=reward_scaler)


class DDPGImpl(TD3Impl):
    """algos/torch/ddpg_impl.py:232-263: unsmoothed target action."""

    def __init__(self, observation_shape, action_size, actor_learning_rate, critic_learning_rate,
                 actor_optim_factory, critic_optim_factory, actor_encoder_factory,
                 critic_encoder_factory, q_func_factory, gamma, tau, n_critics, use_gpu, scaler,
                 action_scaler, reward_scaler):
        super().__init__(
            observation_shape=observation_shape, action_size=action_size,
            actor_learning_rate=actor_learning_rate, critic_learning_rate=critic_learning_rate,
            actor_optim_factory=actor_optim_factory, critic_optim_factory=critic_optim_factory,
            actor_encoder_factory=actor_encoder_factory,
            critic_encoder_factory=critic_encoder_factory, q_func_factory=q_func_factory,
            gamma=gamma, tau=tau, n_critics=n_critics, target_smoothing_sigma=0.0,
            target_smoothing_clip=0.0, use_gpu=use_gpu, scaler=scaler,
            action_scaler=action_scaler, reward_scaler=reward_scaler)


class TD3(AlgoBase):
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
        update_actor_interval: int = 2,
        use_gpu=True,
        scaler=None,
        action_scaler=None,
        reward_scaler=None,
        impl: Optional[TD3Impl] = None,
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
        self._update_actor_interval = update_actor_interval
        self._use_gpu = check_use_gpu(use_gpu)
        self._impl = impl

    def _create_impl(self, observation_shape: Sequence[int], action_size: int) -> None:
        self._impl = TD3Impl(
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
            use_gpu=self._use_gpu,
            scaler=self._scaler,
            action_scaler=self._action_scaler,
            reward_scaler=self._reward_scaler,
        )
        self._impl.build()

    def _actor_step(self) -> bool:
        return self._grad_step % self._update_actor_interval == 0

    def _update(self, batch) -> Dict[str, float]:
        """algos/td3.py:182-203 — metric keys as in the reference."""
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


class DDPG(AlgoBase):
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
        batch_size: int = 100,
        n_frames: int = 1,
        n_steps: int = 1,
        gamma: float = 0.99,
        tau: float = 0.005,
        n_critics: int = 1,
        use_gpu=True,
        scaler=None,
        action_scaler=None,
        reward_scaler=None,
        impl: Optional[DDPGImpl] = None,
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
        self._use_gpu = check_use_gpu(use_gpu)
        self._impl = impl

    def _create_impl(self, observation_shape: Sequence[int], action_size: int) -> None:
        self._impl = DDPGImpl(
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
            use_gpu=self._use_gpu,
            scaler=self._scaler,
            action_scaler=self._action_scaler,
            reward_scaler=self._reward_scaler,
        )
        self._impl.build()

    def _update(self, batch) -> Dict[str, float]:
        """algos/ddpg.py:167-174."""
        m = self._impl.update_step(batch, update_actor=True, sync=True)
        return {"critic_loss": m["critic_loss"], "actor_loss": m["actor_loss"]}

    def _update_async(self, batch) -> None:
        self._impl.update_step(batch, update_actor=True, sync=False)

    def get_action_type(self) -> ActionSpace:
        return ActionSpace.CONTINUOUS


def _resolve(factory, observation_shape):
    return factory.resolve(observation_shape) if hasattr(factory, "resolve") else factory
