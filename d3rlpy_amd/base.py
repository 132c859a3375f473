"""LearnableBase — the fit / fitter / update surface of d3rlpy/base.py:130-1044.

Kept identical: constructor arguments, ``__setattr__`` propagation to the
Impl (base.py:181-185), ``fit`` / ``fitter`` epoch/step structure
(base.py:349-687), ``update`` (:746-758) incrementing ``grad_step`` after
``_update``, ``create_impl`` / ``build_with_dataset``, ``get_params`` /
``set_params``, ``save_params`` / ``from_json`` (params.json), per-epoch
metric means in ``loss_history``.

Different by design (MI355X-first):
  * the dataset is uploaded to HBM once (DeviceDataset) and every minibatch
    is gathered on device; ``fit`` never copies a batch from the host;
  * inside ``fitter`` the per-step losses stay on device (a ring buffer
    written by the update graph) and are read back once per epoch instead of
    four ``loss.cpu()`` syncs per step (cql_impl.py:139-141, sac_impl.py:144-146,
    ddpg_impl.py:152,183);
  * the logger is offline-only (CSV + params.json; no wandb/tensorboard
    network calls, cf. logger.py:85).
"""
from __future__ import annotations

import json
import os
import time
import weakref
from collections import defaultdict
from typing import Any, Callable, DefaultDict, Dict, Generator, List, Optional, Sequence, Tuple

import numpy as np

from .dataset import DeviceDataset, Episode, MDPDataset, Transition
from .factories import (AdamFactory, EncoderFactory, OptimizerFactory, QFunctionFactory,
                        create_encoder_factory, create_q_func_factory)
from .iterators import RandomIterator, RoundIterator, TransitionIterator

IMPL_NOT_INITIALIZED_ERROR = "The neural network parameters are not initialized. " \
    "Pleaes call build_with_dataset, build_with_env, or directly call fit method."


def _mean_present(col: np.ndarray) -> float:
    present = col[~np.isnan(col)]
    return float(np.mean(present)) if present.size else float("nan")


def _serialize(v: Any) -> Any:
    if isinstance(v, (EncoderFactory, QFunctionFactory)):
        return {"type": v.get_type(), "params": v.get_params()}
    if isinstance(v, OptimizerFactory):
        return v.get_params()
    if hasattr(v, "get_type") and hasattr(v, "get_params"):  # scalers
        return {"type": v.get_type(), "params": v.get_params()}
    return v


def _json_default(o: Any) -> Any:
    """logger.py:21-28 (default_json_encoder)."""
    if isinstance(o, np.integer):
        return int(o)
    if isinstance(o, np.floating):
        return float(o)
    if isinstance(o, np.ndarray):
        return o.tolist()
    raise ValueError(f"invalid object type: {type(o)}")


def _deserialize(key: str, v: Any) -> Any:
    if key.endswith("optim_factory") and isinstance(v, dict):
        params = dict(v)
        name = params.pop("optim_cls", "Adam")
        if name == "Adam":
            return AdamFactory(**params)
        return OptimizerFactory(name, **params)
    if key.endswith("encoder_factory") and isinstance(v, dict):
        return create_encoder_factory(v["type"], **v["params"])
    if key == "q_func_factory" and isinstance(v, dict):
        return create_q_func_factory(v["type"], **v["params"])
    if key == "scaler" and isinstance(v, dict):
        from .preprocessing import create_scaler
        return create_scaler(v["type"], **v["params"])
    return v


class LearnableBase:
    def __init__(self, batch_size: int, n_frames: int, n_steps: int, gamma: float,
                 scaler=None, action_scaler=None, reward_scaler=None, real_ratio: float = 1.0,
                 generated_maxlen: int = 100000, kwargs: Optional[Dict[str, Any]] = None):
        from .preprocessing import check_scaler
        self._batch_size = batch_size
        self._n_frames = n_frames
        self._n_steps = n_steps
        self._gamma = gamma
        self._scaler = check_scaler(scaler)
        self._action_scaler = action_scaler
        self._reward_scaler = reward_scaler
        if action_scaler is not None or reward_scaler is not None:
            raise NotImplementedError("action/reward scalers are out of scope (SURVEY §2 #4)")
        self._real_ratio = real_ratio
        self._generated_maxlen = generated_maxlen
        self._impl = None
        self._eval_results: DefaultDict[str, List[float]] = defaultdict(list)
        self._loss_history: DefaultDict[str, List[float]] = defaultdict(list)
        self._active_logger = None
        self._grad_step = 0
        # (weakref to the MDPDataset, its version, the HBM copy): one entry, so
        # a new or changed dataset releases the previous copy
        self._device_dataset_cache: Optional[Tuple[Any, int, DeviceDataset]] = None

    def __setattr__(self, name: str, value: Any) -> None:
        super().__setattr__(name, value)
        # propagate property updates to implementation object (base.py:181-185)
        if hasattr(self, "_impl") and self._impl and hasattr(self._impl, name):
            setattr(self._impl, name, value)

    # ------------------------------------------------------------ params
    def get_params(self, deep: bool = True) -> Dict[str, Any]:
        rets = {}
        for key in dir(self):
            if key.startswith("__") or key in ("_impl", "_eval_results", "_loss_history",
                                               "_active_logger", "_grad_step",
                                               "_device_dataset_cache"):
                continue
            if not key.startswith("_"):
                continue
            value = getattr(self, key)
            if callable(value) and not isinstance(value, (EncoderFactory, QFunctionFactory,
                                                          OptimizerFactory)):
                continue
            if hasattr(value, "get_params") or isinstance(value, (int, float, str, bool, list,
                                                                   tuple, type(None))):
                rets[key[1:]] = value
        return rets

    def set_params(self, **params: Any) -> "LearnableBase":
        for key, val in params.items():
            if hasattr(self, key):
                try:
                    setattr(self, key, val)
                except AttributeError:
                    pass
            else:
                assert hasattr(self, "_" + key), f"{key} does not exist."
                setattr(self, "_" + key, val)
        return self

    def save_params(self, logdir: str) -> None:
        """params.json in the reference schema (base.py:823-850, logger.py:100-110):
        every hyper-parameter, ``algorithm``, ``observation_shape``,
        ``action_size``; factories / scalers as {"type", "params"}, optimiser
        factories as their get_params(), ``use_gpu`` as a device id or null."""
        assert self._impl is not None, IMPL_NOT_INITIALIZED_ERROR
        params: Dict[str, Any] = {}
        for k, v in self.get_params(deep=False).items():
            if k == "impl":
                continue
            if k == "use_gpu":
                v = None if v is None or v is False else (
                    0 if v is True else (v.get_id() if hasattr(v, "get_id") else int(v)))
            params[k] = _serialize(v)
        params["algorithm"] = self.__class__.__name__
        params["observation_shape"] = list(self._impl.observation_shape)
        params["action_size"] = int(self._impl.action_size)
        with open(os.path.join(logdir, "params.json"), "w") as f:
            json.dump(params, f, indent=2, default=_json_default)

    @classmethod
    def params_from_json(cls, fname: str, use_gpu=True):
        """(observation_shape, action_size, constructor kwargs) of a params.json
        written by the reference or by save_params (base.py:186-232)."""
        with open(fname) as f:
            params = json.load(f)
        observation_shape = tuple(params.pop("observation_shape"))
        action_size = params.pop("action_size")
        # the reference passes every remaining key through **kwargs and its
        # constructors ignore ``algorithm``: a params.json of a related class
        # (DQN -> DoubleDQN, a subclass) loads too
        params.pop("algorithm", None)
        params = {k: _deserialize(k, v) for k, v in params.items()}
        params["use_gpu"] = use_gpu
        return observation_shape, action_size, params

    @classmethod
    def from_json(cls, fname: str, use_gpu=True) -> "LearnableBase":
        observation_shape, action_size, params = cls.params_from_json(fname, use_gpu)
        algo = cls(**params)
        algo.create_impl(observation_shape, action_size)
        return algo

    # ------------------------------------------------------------ build
    def create_impl(self, observation_shape: Sequence[int], action_size: int) -> None:
        self._create_impl(observation_shape, action_size)

    def _create_impl(self, observation_shape: Sequence[int], action_size: int) -> None:
        raise NotImplementedError

    def _process_observation_shape(self, observation_shape: Sequence[int]) -> Sequence[int]:
        if len(observation_shape) == 3:
            n_channels = observation_shape[0]
            image_size = observation_shape[1:]
            observation_shape = (self._n_frames * n_channels, *image_size)
        return observation_shape

    def build_with_dataset(self, dataset: MDPDataset) -> None:
        self.create_impl(self._process_observation_shape(dataset.get_observation_shape()),
                         dataset.get_action_size())

    # ------------------------------------------------------------ training
    def _device_dataset(self, dataset) -> DeviceDataset:
        if isinstance(dataset, DeviceDataset):
            return dataset
        if not isinstance(dataset, MDPDataset):
            raise NotImplementedError(
                "fit() on the HIP engine takes an MDPDataset (uploaded to HBM once)")
        c = self._device_dataset_cache
        if c is not None and c[0]() is dataset and c[1] == dataset.version:
            return c[2]
        self._device_dataset_cache = None  # drop the stale copy before uploading
        ddata = DeviceDataset(dataset)
        self._device_dataset_cache = (weakref.ref(dataset), dataset.version, ddata)
        return ddata

    def fit(self, dataset, n_epochs: Optional[int] = None, n_steps: Optional[int] = None,
            n_steps_per_epoch: int = 10000, save_metrics: bool = True,
            experiment_name: Optional[str] = None, with_timestamp: bool = True,
            logdir: str = "d3rlpy_logs", allow_overwrite: bool = False,
            wandb_project: str = "BASE", verbose: bool = True, show_progress: bool = True,
            tensorboard_dir: Optional[str] = None, eval_episodes=None, save_interval: int = 1,
            scorers=None, shuffle: bool = True, callback=None, *,
            index_source: str = "device") -> List[Tuple[int, Dict[str, float]]]:
        return list(self.fitter(dataset, n_epochs, n_steps, n_steps_per_epoch, save_metrics,
                                experiment_name, with_timestamp, logdir, allow_overwrite,
                                wandb_project, verbose, show_progress, tensorboard_dir,
                                eval_episodes, save_interval, scorers, shuffle, callback,
                                index_source=index_source))

    def fitter(self, dataset, n_epochs: Optional[int] = None, n_steps: Optional[int] = None,
               n_steps_per_epoch: int = 10000, save_metrics: bool = True,
               experiment_name: Optional[str] = None, with_timestamp: bool = True,
               logdir: str = "d3rlpy_logs", allow_overwrite: bool = False,
               wandb_project: str = "BASE", verbose: bool = True, show_progress: bool = True,
               tensorboard_dir: Optional[str] = None, eval_episodes=None,
               save_interval: int = 1, scorers=None, shuffle: bool = True, callback=None, *,
               index_source: str = "device"
               ) -> Generator[Tuple[int, Dict[str, float]], None, None]:
        """base.py:349-687.  Extension (keyword-only): ``index_source`` of the
        n_steps mode's RandomIterator — "device" (Philox on the GPU, default)
        or "numpy" (the reference's np.random.randint stream, uploaded per
        step)."""
        from .logger import OfflineLogger
        if tensorboard_dir is not None:
            raise NotImplementedError("tensorboard logging is out of scope (offline logger only)")
        if wandb_project not in (None, "BASE"):
            raise NotImplementedError("wandb logging is out of scope (no network access)")
        ddata = self._device_dataset(dataset)
        if isinstance(dataset, MDPDataset):
            discrete = dataset.is_action_discrete()
            from .constants import ActionSpace
            at = self.get_action_type()
            if at != ActionSpace.BOTH:
                assert (at == ActionSpace.DISCRETE) == discrete, "action space mismatch"
        if self._scaler is not None and isinstance(dataset, MDPDataset):
            self._scaler.fit_dataset(dataset)
        if self._impl is None:
            obs_shape = self._process_observation_shape(ddata.observation_shape)
            self.create_impl(obs_shape, ddata.action_size)
        # the iterator gathers straight into the Impl's input buffers (no copies)
        out = self._impl.staging_batch(self._batch_size) \
            if hasattr(self._impl, "staging_batch") else None
        iterator: TransitionIterator
        if n_epochs is None and n_steps is not None:
            assert n_steps >= n_steps_per_epoch
            n_epochs = n_steps // n_steps_per_epoch
            iterator = RandomIterator(ddata, n_steps_per_epoch, batch_size=self._batch_size,
                                      n_steps=self._n_steps, gamma=self._gamma,
                                      n_frames=self._n_frames, real_ratio=self._real_ratio,
                                      generated_maxlen=self._generated_maxlen, out=out,
                                      index_source=index_source)
        elif n_epochs is not None and n_steps is None:
            iterator = RoundIterator(ddata, batch_size=self._batch_size, n_steps=self._n_steps,
                                     gamma=self._gamma, n_frames=self._n_frames,
                                     real_ratio=self._real_ratio,
                                     generated_maxlen=self._generated_maxlen, shuffle=shuffle,
                                     out=out)
        else:
            raise ValueError("Either of n_epochs or n_steps must be given.")

        name = experiment_name or self.__class__.__name__
        logger = OfflineLogger(name, save_metrics=save_metrics, root_dir=logdir,
                               verbose=verbose, with_timestamp=with_timestamp)
        self._active_logger = logger
        if save_metrics:
            self.save_params(logger.logdir)
        self._eval_results = defaultdict(list)
        self._loss_history = defaultdict(list)

        total_step = 0
        for epoch in range(1, n_epochs + 1):
            iterator.reset()
            ring = self._impl.metrics_ring(len(iterator))
            t0 = time.perf_counter()
            for itr in range(len(iterator)):
                batch = next(iterator)
                self._update_async(batch)
                self._grad_step += 1
                total_step += 1
                if callback:
                    callback(self, epoch, total_step)
            names, values = self._impl.read_metrics_ring(ring)
            elapsed = time.perf_counter() - t0
            # NaN marks "not computed at this step" (e.g. TD3's delayed actor
            # loss); the reference logs such a metric only on the steps that
            # produce it, so the epoch mean skips those rows
            epoch_loss = {n: _mean_present(values[:, i]) for i, n in enumerate(names)}
            self._loss_history["epoch"].append(epoch)
            self._loss_history["step"].append(total_step)
            for k, v in epoch_loss.items():
                self._loss_history[k].append(v)
            if scorers and eval_episodes:
                # base.py:806-821: scorer(algo, episodes) per named scorer, added
                # to the same epoch record (add_metric before commit)
                scores = self._evaluate(eval_episodes, scorers)
                epoch_loss.update(scores)
            logger.add_epoch(epoch, total_step, epoch_loss,
                             {"time_step": elapsed / max(1, len(iterator))})
            if save_metrics and epoch % save_interval == 0:
                logger.save_model(total_step, self)
            yield epoch, dict(epoch_loss)
        logger.close()
        self._active_logger = None

    def _evaluate(self, episodes, scorers: Dict[str, Callable[[Any, Any], float]]
                  ) -> Dict[str, float]:
        """base.py:806-821."""
        out = {}
        for name, scorer in scorers.items():
            score = scorer(self, episodes)
            out[name] = score
            if score is not None:
                self._eval_results[name].append(score)
        return out

    def update(self, batch) -> Dict[str, float]:
        """base.py:746-758: one gradient step on ``batch``; returns metrics."""
        assert self._impl is not None, IMPL_NOT_INITIALIZED_ERROR
        loss = self._update(batch)
        self._grad_step += 1
        return loss

    def _update(self, batch) -> Dict[str, float]:
        raise NotImplementedError

    def _update_async(self, batch) -> None:
        """Enqueue one update; metrics stay on device (fitter only)."""
        raise NotImplementedError

    def get_action_type(self):
        raise NotImplementedError

    # ------------------------------------------------------------ save / load
    def save_model(self, fname: str) -> None:
        assert self._impl is not None, IMPL_NOT_INITIALIZED_ERROR
        self._impl.save_model(fname)

    def load_model(self, fname: str) -> None:
        assert self._impl is not None, IMPL_NOT_INITIALIZED_ERROR
        self._impl.load_model(fname)

    # ------------------------------------------------------------ properties
    @property
    def batch_size(self) -> int:
        return self._batch_size

    @batch_size.setter
    def batch_size(self, batch_size: int) -> None:
        self._batch_size = batch_size

    @property
    def n_frames(self) -> int:
        return self._n_frames

    @property
    def n_steps(self) -> int:
        return self._n_steps

    @property
    def gamma(self) -> float:
        return self._gamma

    @property
    def scaler(self):
        return self._scaler

    @property
    def impl(self):
        return self._impl

    @property
    def observation_shape(self):
        return self._impl.observation_shape if self._impl else None

    @property
    def action_size(self):
        return self._impl.action_size if self._impl else None

    @property
    def active_logger(self):
        return self._active_logger

    @property
    def grad_step(self) -> int:
        return self._grad_step

    def set_grad_step(self, grad_step: int) -> None:
        self._grad_step = grad_step

    @property
    def loss_history(self):
        return self._loss_history
