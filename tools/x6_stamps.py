"""Phase timing of d3a_q2_fwd_x6 from in-kernel s_memtime stamps (diagnostic
build: D3A_X6_PROBE=16 selects the stamped instantiation; results stay right).

Runs the K2 critic-forward shape (as tools/bench_fwd.py) a few times, then
one stamped launch, and prints per phase the median / p10 / p90 cycles over
the workgroups (wave 0 of each): prologue (x staging), first production,
each 64-unit chunk of layer 2, the layer-2 epilogue (kept h2 rows, head dot)
and the head write-out; plus the kernel's span in cycles against its HIP-event
duration (the in-kernel clock)."""
import os
import subprocess
import sys

os.environ["D3A_X6_PROBE"] = "16"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ctypes as C  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

from d3rlpy_amd import _native as N  # noqa: E402
from d3rlpy_amd import ops  # noqa: E402


def main():
    sys.argv = [sys.argv[0], "--x6", "--reps", "20"]
    import bench_fwd  # noqa: F401  (runs the K2 forward shape with the stamped build)
    bench_fwd.main()
    n = 2048 * 10
    buf = (C.c_ulonglong * n)()
    rc = N.lib().d3a_x6_stamps(buf, n)
    assert rc == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(2048, 10).astype(np.int64)
    a = a[a[:, 0] > 0]
    names = ["prologue", "produce0", "chunk0", "chunk1", "chunk2", "chunk3", "epilogue", "head out"]
    d = np.diff(a[:, :9], axis=1)
    print(f"workgroups {len(a)}; cycles per phase (median / p10 / p90):")
    for i, nm in enumerate(names):
        v = d[:, i]
        print(f"  {nm:10s} {np.median(v):9.0f} {np.percentile(v, 10):9.0f} {np.percentile(v, 90):9.0f}")
    span = a[:, 8].max() - a[:, 0].min()
    tot = a[:, 8] - a[:, 0]
    print(f"  total/wg   {np.median(tot):9.0f}; start skew {a[:, 0].max() - a[:, 0].min()} cycles; "
          f"kernel span {span} cycles")


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    main()
