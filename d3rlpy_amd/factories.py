"""Configuration factories with the reference's names, TYPE strings and params.

Mirrors d3rlpy/models/optimizers.py (OptimizerFactory, AdamFactory),
d3rlpy/models/encoders.py (EncoderFactory family, ENCODER_LIST :407-442),
d3rlpy/models/q_functions.py (QFunctionFactory family, Q_FUNC_LIST :324-359)
and d3rlpy/argument_utility.py (check_encoder / check_q_func / check_use_gpu).

On the HIP engine these are *descriptions*: the Impl reads their parameters
and builds flat-buffer networks; configurations the engine does not
implement raise NotImplementedError at build time (the reference's error
convention for unsupported paths, e.g. algos/torch/bcq_impl.py:212-213).
"""
from __future__ import annotations

import copy
from typing import Any, ClassVar, Dict, Optional, Sequence, Tuple, Union


# ---------------------------------------------------------------- optimisers
class OptimizerFactory:
    def __init__(self, optim_cls: Union[type, str] = "Adam", **kwargs: Any):
        self._optim_name = optim_cls if isinstance(optim_cls, str) else optim_cls.__name__
        self._optim_kwargs = kwargs

    @property
    def optim_name(self) -> str:
        return self._optim_name

    def get_params(self, deep: bool = False) -> Dict[str, Any]:
        params = copy.deepcopy(self._optim_kwargs) if deep else dict(self._optim_kwargs)
        return {"optim_cls": self._optim_name, **params}

    # Adam hyper-parameters as seen by the HIP Adam kernel
    @property
    def betas(self) -> Tuple[float, float]:
        self._require_adam()
        b = self._optim_kwargs.get("betas", (0.9, 0.999))
        return float(b[0]), float(b[1])

    @property
    def eps(self) -> float:
        self._require_adam()
        return float(self._optim_kwargs.get("eps", 1e-8))

    def _require_adam(self) -> None:
        kw = self._optim_kwargs
        if self._optim_name != "Adam" or kw.get("weight_decay", 0) != 0 or kw.get("amsgrad", False):
            raise NotImplementedError(
                "the HIP engine implements torch.optim.Adam (weight_decay=0, amsgrad=False)")

    def create(self, params, lr: float):  # reference API: build a torch optimizer
        import torch.optim as optim
        return getattr(optim, self._optim_name)(params, lr=lr, **self._optim_kwargs)


class AdamFactory(OptimizerFactory):
    """models/optimizers.py:106-138."""

    def __init__(self, betas: Tuple[float, float] = (0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0, amsgrad: bool = False, **kwargs: Any):
        super().__init__("Adam", betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=amsgrad)


# ------------------------------------------------------------------ encoders
class EncoderFactory:
    TYPE: ClassVar[str] = "none"

    def get_type(self) -> str:
        return self.TYPE

    def get_params(self, deep: bool = False) -> Dict[str, Any]:
        raise NotImplementedError


class VectorEncoderFactory(EncoderFactory):
    TYPE: ClassVar[str] = "vector"

    def __init__(self, hidden_units: Optional[Sequence[int]] = None, activation: str = "relu",
                 use_batch_norm: bool = False, dropout_rate: Optional[float] = None,
                 use_dense: bool = False):
        self._hidden_units = list(hidden_units) if hidden_units is not None else [256, 256]
        self._activation = activation
        self._use_batch_norm = use_batch_norm
        self._dropout_rate = dropout_rate
        self._use_dense = use_dense

    @property
    def hidden_units(self) -> Sequence[int]:
        self._require_plain()
        return self._hidden_units

    def _require_plain(self) -> None:
        if self._activation != "relu" or self._use_batch_norm or self._dropout_rate is not None \
                or self._use_dense:
            raise NotImplementedError(
                "the HIP engine implements relu MLP encoders without batch-norm/dropout/dense")

    def get_params(self, deep: bool = False) -> Dict[str, Any]:
        return {"hidden_units": copy.deepcopy(self._hidden_units) if deep else self._hidden_units,
                "activation": self._activation, "use_batch_norm": self._use_batch_norm,
                "dropout_rate": self._dropout_rate, "use_dense": self._use_dense}


class PixelEncoderFactory(EncoderFactory):
    """encoders.py:86-163: Nature-DQN conv stack + fc."""

    TYPE: ClassVar[str] = "pixel"

    def __init__(self, filters: Optional[Sequence[Sequence[int]]] = None, feature_size: int = 512,
                 activation: str = "relu", use_batch_norm: bool = False,
                 dropout_rate: Optional[float] = None):
        self._filters = [list(f) for f in filters] if filters else [[32, 8, 4], [64, 4, 2],
                                                                   [64, 3, 1]]
        self._feature_size = feature_size
        self._activation = activation
        self._use_batch_norm = use_batch_norm
        self._dropout_rate = dropout_rate

    @property
    def filters(self):
        return [list(f) for f in self._filters]

    @property
    def feature_size(self) -> int:
        return self._feature_size

    def get_params(self, deep: bool = False) -> Dict[str, Any]:
        return {"filters": copy.deepcopy(self._filters), "feature_size": self._feature_size,
                "activation": self._activation, "use_batch_norm": self._use_batch_norm,
                "dropout_rate": self._dropout_rate}


class DefaultEncoderFactory(EncoderFactory):
    """encoders.py: picks Pixel for 3-D observations, Vector otherwise."""

    TYPE: ClassVar[str] = "default"

    def __init__(self, activation: str = "relu", use_batch_norm: bool = False,
                 dropout_rate: Optional[float] = None):
        self._activation = activation
        self._use_batch_norm = use_batch_norm
        self._dropout_rate = dropout_rate

    def resolve(self, observation_shape: Sequence[int]) -> EncoderFactory:
        if len(observation_shape) == 3:
            return PixelEncoderFactory(activation=self._activation,
                                       use_batch_norm=self._use_batch_norm,
                                       dropout_rate=self._dropout_rate)
        return VectorEncoderFactory(activation=self._activation,
                                    use_batch_norm=self._use_batch_norm,
                                    dropout_rate=self._dropout_rate)

    @property
    def hidden_units(self) -> Sequence[int]:
        return self.resolve((1,)).hidden_units  # type: ignore[attr-defined]

    def get_params(self, deep: bool = False) -> Dict[str, Any]:
        return {"activation": self._activation, "use_batch_norm": self._use_batch_norm,
                "dropout_rate": self._dropout_rate}


ENCODER_LIST = {c.TYPE: c for c in (VectorEncoderFactory, PixelEncoderFactory,
                                    DefaultEncoderFactory)}


def create_encoder_factory(name: str, **kwargs: Any) -> EncoderFactory:
    assert name in ENCODER_LIST, f"{name} seems not to be registered."
    return ENCODER_LIST[name](**kwargs)


# --------------------------------------------------------------- Q functions
class QFunctionFactory:
    TYPE: ClassVar[str] = "none"

    def __init__(self, share_encoder: bool = False):
        if share_encoder:
            raise NotImplementedError("share_encoder=True is not supported by the HIP engine")
        self._share_encoder = share_encoder

    def get_type(self) -> str:
        return self.TYPE

    @property
    def share_encoder(self) -> bool:
        return self._share_encoder

    def get_params(self, deep: bool = False) -> Dict[str, Any]:
        return {"share_encoder": self._share_encoder}


class MeanQFunctionFactory(QFunctionFactory):
    TYPE: ClassVar[str] = "mean"

    def __init__(self, share_encoder: bool = False, **kwargs: Any):
        super().__init__(share_encoder)


class QRQFunctionFactory(QFunctionFactory):
    TYPE: ClassVar[str] = "qr"

    def __init__(self, share_encoder: bool = False, n_quantiles: int = 32, **kwargs: Any):
        super().__init__(share_encoder)
        self._n_quantiles = n_quantiles

    @property
    def n_quantiles(self) -> int:
        return self._n_quantiles

    def get_params(self, deep: bool = False) -> Dict[str, Any]:
        return {"share_encoder": self._share_encoder, "n_quantiles": self._n_quantiles}


class IQNQFunctionFactory(QFunctionFactory):
    TYPE: ClassVar[str] = "iqn"

    def __init__(self, share_encoder: bool = False, n_quantiles: int = 64,
                 n_greedy_quantiles: int = 32, embed_size: int = 64, **kwargs: Any):
        super().__init__(share_encoder)
        self._n_quantiles = n_quantiles
        self._n_greedy_quantiles = n_greedy_quantiles
        self._embed_size = embed_size

    @property
    def n_quantiles(self) -> int:
        return self._n_quantiles

    @property
    def n_greedy_quantiles(self) -> int:
        return self._n_greedy_quantiles

    @property
    def embed_size(self) -> int:
        return self._embed_size

    def get_params(self, deep: bool = False) -> Dict[str, Any]:
        return {"share_encoder": self._share_encoder, "n_quantiles": self._n_quantiles,
                "n_greedy_quantiles": self._n_greedy_quantiles, "embed_size": self._embed_size}


Q_FUNC_LIST = {c.TYPE: c for c in (MeanQFunctionFactory, QRQFunctionFactory,
                                   IQNQFunctionFactory)}


def create_q_func_factory(name: str, **kwargs: Any) -> QFunctionFactory:
    assert name in Q_FUNC_LIST, f"{name} seems not to be registered."
    return Q_FUNC_LIST[name](**kwargs)


# ---------------------------------------------------------- argument checks
def check_encoder(value: Union[EncoderFactory, str]) -> EncoderFactory:
    """argument_utility.py:20-30."""
    if isinstance(value, EncoderFactory):
        return value
    if isinstance(value, str):
        return create_encoder_factory(value)
    raise ValueError("This argument must be str or EncoderFactory object.")


def check_q_func(value: Union[QFunctionFactory, str]) -> QFunctionFactory:
    """argument_utility.py:33-43."""
    if isinstance(value, QFunctionFactory):
        return value
    if isinstance(value, str):
        return create_q_func_factory(value)
    raise ValueError("This argument must be str or QFunctionFactory object.")


def check_use_gpu(value):
    """argument_utility.py:96-114: True -> Device(0) (Device(LOCAL_RANK) in a
    multi-process launch, WORLD_SIZE > 1), int -> Device(int),
    a Device as is, False / None -> None (the reference's CPU).  The HIP
    engine has no CPU path: an Impl built with None raises
    NotImplementedError (algos/impl_base.py)."""
    from .gpu import Device
    # isinstance cannot tell bool from int
    if type(value) == bool:
        if not value:
            return None
        # one process per GPU (torchrun / bench.launch_ranks): a bare True is
        # this rank's GPU, LOCAL_RANK, not GPU 0 -- otherwise every rank's
        # parameters would land on cuda:0 beside a dataset and communicator
        # on cuda:LOCAL_RANK.  Single-process runs keep the reference's 0.
        import os
        if int(os.environ.get("WORLD_SIZE", "1")) > 1 and "LOCAL_RANK" in os.environ:
            return Device(int(os.environ["LOCAL_RANK"]))
        return Device(0)
    if type(value) == int:
        return Device(value)
    if isinstance(value, Device):
        return value
    if value is None:
        return None
    raise ValueError("This argument must be bool, int or Device.")
