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

    def save_policy(self, fname: str) -> None:
        """algos/base.py:77-103: greedy policy as TorchScript (.pt) or ONNX (.onnx)."""
        assert self._impl is not None, IMPL_NOT_INITIALIZED_ERROR
        self._impl.save_policy(fname)

    def copy_policy_from(self, algo: "AlgoBase") -> None:
        assert self._impl is not None and algo.impl is not None, IMPL_NOT_INITIALIZED_ERROR
        self._impl.copy_policy_from(algo.impl)

    def copy_q_function_from(self, algo: "AlgoBase") -> None:
        assert self._impl is not None and algo.impl is not None, IMPL_NOT_INITIALIZED_ERROR
        self._impl.copy_q_function_from(algo.impl)
