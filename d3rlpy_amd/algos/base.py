"""AlgoBase — d3rlpy/algos/base.py:24-170 (predict / predict_value / sample_action)."""
from __future__ import annotations

from typing import Optional, Tuple, Union

import numpy as np

from ..base import IMPL_NOT_INITIALIZED_ERROR, LearnableBase


class AlgoBase(LearnableBase):
    def predict(self, x) -> np.ndarray:
        """Greedy action(s) for observation(s) ``x`` (algos/base.py:107-127)."""
        assert self._impl is not None, IMPL_NOT_INITIALIZED_ERROR
        return self._impl.predict_best_action(x)

    def predict_value(self, x, action, with_std: bool = False
                      ) -> Union[np.ndarray, Tuple[np.ndarray, np.ndarray]]:
        assert self._impl is not None, IMPL_NOT_INITIALIZED_ERROR
        return self._impl.predict_value(x, action, with_std)

    def sample_action(self, x) -> np.ndarray:
        assert self._impl is not None, IMPL_NOT_INITIALIZED_ERROR
        return self._impl.sample_action(x)

    def build_with_env(self, env) -> None:
        """algos/base.py build_with_env: shapes from the env's spaces."""
        from ..online import get_action_size_from_env
        self.create_impl(self._process_observation_shape(env.observation_space.shape),
                         get_action_size_from_env(env))

    def collect(self, env, buffer=None, explorer=None, deterministic: bool = False,
                n_steps: int = 1000000, show_progress: bool = True,
                timelimit_aware: bool = True):
        """algos/base.py collect: fill a ReplayBuffer from ``env`` without
        updates; returns the buffer."""
        from ..online import ReplayBuffer, collect
        if buffer is None:
            buffer = ReplayBuffer(1000000, env=env)
        collect(self, env, buffer, explorer, deterministic=deterministic, n_steps=n_steps,
                show_progress=show_progress, timelimit_aware=timelimit_aware)
        return buffer

    def fit_online(self, env, buffer=None, explorer=None, n_steps: int = 1000000,
                   n_steps_per_epoch: int = 10000, update_interval: int = 1,
                   update_start_step: int = 0, random_steps: int = 0, eval_env=None,
                   eval_epsilon: float = 0.0, save_metrics: bool = True,
                   save_interval: int = 1, experiment_name: Optional[str] = None,
                   with_timestamp: bool = True, logdir: str = "d3rlpy_logs",
                   verbose: bool = True, show_progress: bool = True,
                   tensorboard_dir: Optional[str] = None, timelimit_aware: bool = True,
                   callback=None):
        """algos/base.py:187-260: online training on a gym-style env (old
        ``reset() -> obs`` / ``step(a) -> (obs, r, done, info)`` API) with the
        HBM-resident ReplayBuffer (default maxlen 1,000,000)."""
        from ..online import ReplayBuffer, train_single_env
        if buffer is None:
            buffer = ReplayBuffer(1000000, env=env)
        return train_single_env(self, env, buffer, explorer, n_steps=n_steps,
                                n_steps_per_epoch=n_steps_per_epoch,
                                update_interval=update_interval,
                                update_start_step=update_start_step,
                                random_steps=random_steps, eval_env=eval_env,
                                eval_epsilon=eval_epsilon, save_metrics=save_metrics,
                                save_interval=save_interval, experiment_name=experiment_name,
                                with_timestamp=with_timestamp, logdir=logdir, verbose=verbose,
                                show_progress=show_progress, tensorboard_dir=tensorboard_dir,
                                timelimit_aware=timelimit_aware, callback=callback)

    def save_policy(self, fname: str, hip_ops: bool = False) -> None:
        """algos/base.py:77-103: greedy policy as TorchScript (.pt) or ONNX (.onnx);
        ``hip_ops`` (extension): MLPs through torch.ops.d3rlpy_amd.mlp_forward."""
        assert self._impl is not None, IMPL_NOT_INITIALIZED_ERROR
        self._impl.save_policy(fname, hip_ops=hip_ops)

    def copy_policy_from(self, algo: "AlgoBase") -> None:
        assert self._impl is not None and algo.impl is not None, IMPL_NOT_INITIALIZED_ERROR
        self._impl.copy_policy_from(algo.impl)

    def copy_q_function_from(self, algo: "AlgoBase") -> None:
        assert self._impl is not None and algo.impl is not None, IMPL_NOT_INITIALIZED_ERROR
        self._impl.copy_q_function_from(algo.impl)
