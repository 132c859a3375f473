"""d3rlpy_amd — MI355X-native (gfx950) offline-RL update engine.

Keeps d3rlpy v1.1.0's Algo / Impl surface (fit / update / predict and the
per-algorithm ``update_*`` methods) for the per-batch critic/actor update of
CQL (and, as they land, TD3+BC, BCQ and DiscreteCQL), with the arithmetic in
hand-written HIP kernels (``csrc/``, C-ABI in ``include/d3rlpy_amd.h``).
There is no CPU compute path: the native library must be built
(``python -m d3rlpy_amd._build``) and a HIP device must be present.
"""
__version__ = "0.1.0"
