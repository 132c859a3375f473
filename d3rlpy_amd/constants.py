"""d3rlpy/constants.py equivalents used by the hot path."""
from enum import Enum

IMPL_NOT_INITIALIZED_ERROR = (
    "The neural network parameters are not initialized. Pleaes call build_with_dataset, "
    "build_with_env, or directly call fit or fit_online method."
)


class ActionSpace(Enum):
    CONTINUOUS = 1
    DISCRETE = 2
    BOTH = 3
