"""Common Impl surface — mirrors d3rlpy/algos/torch/base.py:28-224 (TorchImplBase).

``predict_best_action`` / ``sample_action`` / ``predict_value`` keep the
reference's numpy-in / numpy-out contract (algos/torch/base.py:52-84,
algos/torch/utility.py:279-302).  Batches may be the host
``TransitionMiniBatch``-like object of the reference (numpy arrays, copied to
HBM once per update instead of once per ``update_*`` call as
torch_utility.py:259-266 does) or a ``DeviceBatch`` already in HBM (no copy).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Sequence, Tuple, Union

import numpy as np
import torch

from ..factories import check_use_gpu


@dataclass
class DeviceBatch:
    """A minibatch resident in HBM (the fast-path counterpart of
    TransitionMiniBatch, dataset.pyx:1099-1175).  Field names follow it."""

    obs: torch.Tensor        # [B, *obs_shape] f32 (or u8 frames)
    act: torch.Tensor        # [B, A] f32 or [B] i32
    rew: torch.Tensor        # [B] f32
    next_obs: torch.Tensor   # [B, *obs_shape]
    term: torch.Tensor       # [B] f32
    n_steps: torch.Tensor    # [B] f32

    @property
    def batch_size(self) -> int:
        return int(self.obs.shape[0])

    # reference attribute names (TransitionMiniBatch properties)
    @property
    def observations(self):
        return self.obs

    @property
    def actions(self):
        return self.act

    @property
    def rewards(self):
        return self.rew.view(-1, 1)

    @property
    def next_observations(self):
        return self.next_obs

    @property
    def terminals(self):
        return self.term.view(-1, 1)

    def __len__(self) -> int:
        return self.batch_size


def _to_dev(a, device, dtype=None) -> torch.Tensor:
    if isinstance(a, torch.Tensor):
        t = a
    else:
        arr = np.asarray(a)
        t = torch.from_numpy(np.ascontiguousarray(arr))
    if dtype is not None and t.dtype != dtype:
        t = t.to(dtype)
    return t.to(device, non_blocking=True)


def as_device_batch(batch, device: torch.device) -> DeviceBatch:
    if isinstance(batch, DeviceBatch):
        return batch
    obs = batch.observations
    is_img = np.asarray(obs).dtype == np.uint8 if not isinstance(obs, torch.Tensor) \
        else obs.dtype == torch.uint8
    odt = torch.uint8 if is_img else torch.float32
    act = batch.actions
    adt = torch.int32 if np.asarray(act).dtype.kind in "iu" else torch.float32
    return DeviceBatch(
        obs=_to_dev(obs, device, odt),
        act=_to_dev(act, device, adt),
        rew=_to_dev(batch.rewards, device, torch.float32).view(-1),
        next_obs=_to_dev(batch.next_observations, device, odt),
        term=_to_dev(batch.terminals, device, torch.float32).view(-1),
        n_steps=_to_dev(batch.n_steps, device, torch.float32).view(-1),
    )


class ImplBase:
    def __init__(self, observation_shape: Sequence[int], action_size: int, scaler,
                 action_scaler, reward_scaler, use_gpu=None):
        self._observation_shape = tuple(observation_shape)
        self._action_size = action_size
        self._scaler = scaler
        self._action_scaler = action_scaler
        self._reward_scaler = reward_scaler
        device = check_use_gpu(use_gpu)
        if device is None:
            # the reference's use_gpu=False / None is its CPU path
            raise NotImplementedError(
                "use_gpu=False / None selects the reference's CPU path; the HIP engine has "
                "no CPU compute path (pass use_gpu=True, a device id or a Device)")
        if not torch.cuda.is_available():
            raise RuntimeError("d3rlpy_amd requires a HIP GPU (no CPU fallback)")
        self._device = f"cuda:{device.get_id()}"
        self.torch_device = torch.device(self._device)

    # ---- inference (numpy in / numpy out) ---------------------------------
    def _as_input(self, x) -> torch.Tensor:
        t = _to_dev(x, self.torch_device, torch.float32)
        assert t.ndim > 1, "Input must have batch dimension."
        if self._scaler is not None:
            t = self._scaler.transform(t)
        return t

    def predict_best_action(self, x) -> np.ndarray:
        with torch.no_grad():
            a = self._predict_best_action(self._as_input(x))
            if self._action_scaler is not None:
                a = self._action_scaler.reverse_transform(a)
            return a.cpu().numpy()

    def sample_action(self, x) -> np.ndarray:
        with torch.no_grad():
            a = self._sample_action(self._as_input(x))
            if self._action_scaler is not None:
                a = self._action_scaler.reverse_transform(a)
            return a.cpu().numpy()

    def predict_value(self, x, action, with_std: bool
                      ) -> Union[np.ndarray, Tuple[np.ndarray, np.ndarray]]:
        """ContinuousQFunctionMixin.predict_value (algos/torch/utility.py:279-302)."""
        xt = self._as_input(x)
        at = _to_dev(action, self.torch_device, torch.float32)
        assert xt.shape[0] == at.shape[0]
        if self._action_scaler is not None:
            at = self._action_scaler.transform(at)
        with torch.no_grad():
            values = self._predict_value(xt, at).cpu().numpy()  # [C][B]
        values = np.transpose(values.reshape(values.shape[0], values.shape[1], -1), [1, 0, 2])
        mean_values = values.mean(axis=1).reshape(-1)
        stds = np.std(values, axis=1).reshape(-1)
        if with_std:
            return mean_values, stds
        return mean_values

    def save_policy(self, fname: str, hip_ops: bool = False) -> None:
        """algos/torch/base.py:87-127: the greedy policy (behind the scalers)
        as TorchScript ``.pt`` or ``.onnx``, built by ``_policy_module``.
        ``hip_ops=True`` (extension): MLP trunks call the registered HIP op
        torch.ops.d3rlpy_amd.mlp_forward instead of plain torch layers."""
        from .. import export
        prev = export._HIP_OPS
        export._HIP_OPS = bool(hip_ops)
        try:
            module = self._policy_module()
        finally:
            export._HIP_OPS = prev
        export.save_traced(module, self._observation_shape, self.torch_device, fname,
                           self._scaler, self._action_scaler)

    def _policy_module(self) -> torch.nn.Module:
        raise NotImplementedError

    def _predict_best_action(self, x: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    def _sample_action(self, x: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    def _predict_value(self, x: torch.Tensor, action: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    # ---- properties (algos/torch/base.py:202-224) --------------------------
    @property
    def observation_shape(self) -> Sequence[int]:
        return self._observation_shape

    @property
    def action_size(self) -> int:
        return self._action_size

    @property
    def device(self) -> str:
        return self._device

    @property
    def scaler(self):
        return self._scaler

    @property
    def action_scaler(self):
        return self._action_scaler

    @property
    def reward_scaler(self):
        return self._reward_scaler
