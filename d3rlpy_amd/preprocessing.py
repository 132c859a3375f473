"""Observation scalers used on the hot path (d3rlpy/preprocessing/scalers.py).

StandardScaler (:248-373): statistics fitted on the host exactly as the
reference does (two numpy passes over the transitions' observations,
:320-341); on the HIP path the transform ``(x - mean) / (std + eps)`` is
fused into the minibatch staging of the Impl instead of being re-applied to
freshly copied tensors in every ``update_*`` call (torch_utility.py:179-181).
PixelScaler (:80-110): ``x / 255``, fused into the uint8 frame decode.
"""
from __future__ import annotations

from typing import Any, Dict, Optional

import numpy as np


class Scaler:
    TYPE = "none"

    def get_type(self) -> str:
        return self.TYPE

    def get_params(self, deep: bool = False) -> Dict[str, Any]:
        raise NotImplementedError


class PixelScaler(Scaler):
    TYPE = "pixel"

    def fit_dataset(self, dataset) -> None:
        pass

    def transform(self, x):
        return x.float() / 255.0

    def reverse_transform(self, x):
        return (x * 255.0).long()

    def get_params(self, deep: bool = False) -> Dict[str, Any]:
        return {}


class StandardScaler(Scaler):
    TYPE = "standard"

    def __init__(self, dataset=None, mean: Optional[np.ndarray] = None,
                 std: Optional[np.ndarray] = None, eps: float = 1e-3):
        self._mean = None
        self._std = None
        self._eps = eps
        if dataset is not None:
            self.fit_dataset(dataset)
        elif mean is not None and std is not None:
            self._mean = np.asarray(mean)
            self._std = np.asarray(std)

    def fit_dataset(self, dataset) -> None:
        """scalers.py:320-341, over every transition's observation."""
        if self._mean is not None and self._std is not None:
            return
        from .dataset import transition_table
        t_row = transition_table(dataset.episode_bounds())[0]
        obs = np.asarray(dataset.observations)[t_row].astype(np.float64)
        mean = obs.sum(axis=0) / obs.shape[0]
        std = np.sqrt(((obs - mean) ** 2).sum(axis=0) / obs.shape[0])
        self._mean = mean.reshape((1,) + mean.shape)
        self._std = std.reshape((1,) + std.shape)

    @property
    def mean(self):
        return self._mean

    @property
    def std(self):
        return self._std

    @property
    def eps(self) -> float:
        return self._eps

    def transform(self, x):
        import torch
        mean = torch.tensor(self._mean, dtype=torch.float32, device=x.device)
        std = torch.tensor(self._std, dtype=torch.float32, device=x.device)
        return (x - mean) / (std + self._eps)

    def reverse_transform(self, x):
        import torch
        mean = torch.tensor(self._mean, dtype=torch.float32, device=x.device)
        std = torch.tensor(self._std, dtype=torch.float32, device=x.device)
        return ((std + self._eps) * x) + mean

    def get_params(self, deep: bool = False) -> Dict[str, Any]:
        mean = None if self._mean is None else (self._mean.copy() if deep else self._mean)
        std = None if self._std is None else (self._std.copy() if deep else self._std)
        return {"mean": mean, "std": std, "eps": self._eps}


SCALER_LIST = {"pixel": PixelScaler, "standard": StandardScaler}


def create_scaler(name: str, **kwargs: Any) -> Scaler:
    assert name in SCALER_LIST, f"{name} seems not to be registered."
    if name == "standard":
        kw = {k: (np.asarray(v) if v is not None and k in ("mean", "std") else v)
              for k, v in kwargs.items()}
        return StandardScaler(**kw)
    return SCALER_LIST[name](**kwargs)


def check_scaler(value) -> Optional[Scaler]:
    """argument_utility.py:48-61."""
    if isinstance(value, Scaler):
        return value
    if isinstance(value, str):
        return create_scaler(value)
    if value is None:
        return None
    raise ValueError("This argument must be str or Scaler object.")
