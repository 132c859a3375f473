"""DQN and DoubleDQN — d3rlpy/algos/dqn.py:19-233 on the HIP pixel pipeline of
DiscreteCQLImpl.

DQNImpl (algos/torch/dqn_impl.py:27-159) / DoubleDQNImpl (:162-171) are
DiscreteCQLImpl without the conservative term (alpha = 0: loss = the Huber TD
error of DiscreteMeanQFunction.compute_error, mean_q_function.py:25-40); DQN's
target action is the target network's argmax, DoubleDQN's the online
network's.  The mean Q-function (the reference default) runs both; the IQN
Q-function runs DoubleDQN.  Constructor arguments and defaults are the
reference's (dqn.py:72-125); ``_update`` keeps its schedule and metric name
(dqn.py:127-132: update, then the hard target sync every
``target_update_interval`` steps, folded into the update's last launch).
"""
from __future__ import annotations

from typing import Any, Optional, Sequence

from ..factories import AdamFactory, OptimizerFactory, check_use_gpu
from .cql import DiscreteCQL, _resolve
from .discrete_cql_impl import DiscreteCQLImpl


class DoubleDQNImpl(DiscreteCQLImpl):
    """algos/torch/dqn_impl.py:162-171 (DQNImpl.update with the online argmax)."""

    def __init__(self, observation_shape, action_size, learning_rate, optim_factory,
                 encoder_factory, q_func_factory, gamma, n_critics, use_gpu, scaler,
                 reward_scaler):
        super().__init__(observation_shape=observation_shape, action_size=action_size,
                         learning_rate=learning_rate, optim_factory=optim_factory,
                         encoder_factory=encoder_factory, q_func_factory=q_func_factory,
                         gamma=gamma, n_critics=n_critics, alpha=0.0, use_gpu=use_gpu,
                         scaler=scaler, reward_scaler=reward_scaler)


class DQNImpl(DoubleDQNImpl):
    """algos/torch/dqn_impl.py:27-159: target a* = argmax_a Q_targ(s', a)."""

    _DOUBLE = False


class DQN(DiscreteCQL):
    """algos/dqn.py:19-135 with the HIP DQNImpl."""

    _IMPL = DQNImpl

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
        use_gpu=True,
        scaler=None,
        reward_scaler=None,
        impl: Optional[DQNImpl] = None,
        **kwargs: Any,
    ):
        super().__init__(learning_rate=learning_rate, optim_factory=optim_factory,
                         encoder_factory=encoder_factory, q_func_factory=q_func_factory,
                         batch_size=batch_size, n_frames=n_frames, n_steps=n_steps, gamma=gamma,
                         n_critics=n_critics, target_update_interval=target_update_interval,
                         alpha=0.0, use_gpu=use_gpu, scaler=scaler, reward_scaler=reward_scaler,
                         impl=impl, **kwargs)

    def _create_impl(self, observation_shape: Sequence[int], action_size: int) -> None:
        self._impl = self._IMPL(
            observation_shape=observation_shape,
            action_size=action_size,
            learning_rate=self._learning_rate,
            optim_factory=self._optim_factory,
            encoder_factory=_resolve(self._encoder_factory, observation_shape),
            q_func_factory=self._q_func_factory,
            gamma=self._gamma,
            n_critics=self._n_critics,
            use_gpu=self._use_gpu,
            scaler=self._scaler,
            reward_scaler=self._reward_scaler,
        )
        self._impl.build()


class DoubleDQN(DQN):
    """algos/dqn.py:138-233 with the HIP DoubleDQNImpl."""

    _IMPL = DoubleDQNImpl


__all__ = ["DQN", "DoubleDQN", "DQNImpl", "DoubleDQNImpl"]
