"""The C-ABI as PyTorch custom ops: ``torch.ops.d3rlpy_amd.*``.

``load()`` loads libd3rlpy_amd_torch.so (csrc/torch_ops.cpp, built by
``_build.build``), which registers the ``d3rlpy_amd`` op namespace through
TORCH_LIBRARY with HIP (CUDA-key) and Meta implementations — SURVEY §8(b).
There is no fallback: a missing library raises.

    from d3rlpy_amd import torch_ops
    ops = torch_ops.load()
    y = ops.linear(x, W, b, True)           # every ensemble member, one launch
    q = ops.mlp_forward(x, [W0, W1, W2], [b0, b1, b2])
"""
from __future__ import annotations

import os

import torch

_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libd3rlpy_amd_torch.so")
_loaded = False


def load():
    """Register the ops (idempotent) and return the ``torch.ops.d3rlpy_amd`` namespace."""
    global _loaded
    if not _loaded:
        if not os.path.exists(_LIB):
            raise RuntimeError(f"{_LIB} is missing: run d3rlpy_amd._build.build() "
                               "(no CPU fallback)")
        from . import _native
        _native.lib()  # the C-ABI library the op library links against
        torch.ops.load_library(_LIB)
        _loaded = True
    return torch.ops.d3rlpy_amd


def library_path() -> str:
    return _LIB
