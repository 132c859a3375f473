"""Device: the GPU id an algorithm runs on (d3rlpy/gpu.py:14-72).

Same semantics as the reference: ``get_id()``; deep-copied inside
``context.parallel()`` it advances to the next visible GPU (round-robin over
``get_gpu_count()``), which is how replicas of one configuration land on
different GPUs when a scikit-learn utility clones the algorithm per job.
``get_gpu_count`` counts HIP devices with torch (the reference uses GPUtil,
which is not in this image); counting does not initialise the GPU.
"""
from typing import Any, Dict

from .context import get_parallel_flag


def get_gpu_count() -> int:
    import torch
    return torch.cuda.device_count()


class Device:
    _idx: int

    def __init__(self, idx: int = 0):
        self._idx = idx

    def get_id(self) -> int:
        return self._idx

    def __deepcopy__(self, memo: Any) -> "Device":
        if get_parallel_flag():
            # round-robin for sklearn.base.clone under parallel()
            self._idx += 1
            if self._idx >= get_gpu_count():
                self._idx = 0
        return self.__class__(self._idx)

    def __eq__(self, obj: Any) -> bool:
        if isinstance(obj, Device):
            return self._idx == obj.get_id()
        raise ValueError("Device cannot be compared with non Device objects.")

    def __ne__(self, obj: Any) -> bool:
        return not self.__eq__(obj)

    def __hash__(self) -> int:
        return hash(("Device", self._idx))

    def __repr__(self) -> str:
        return f"Device(idx={self._idx})"

    def get_params(self, deep: bool = False) -> Dict[str, Any]:
        return {"idx": self._idx}
