"""Phase stamps of K3's target-pass kernel (mlp_x6_wide_kernel, D3A_WIDE_STAMPS=1):
per-workgroup cycles of each phase and the spread of start times (how the 800
workgroups fall into rounds on the CUs).

    D3A_WIDE_STAMPS=1 python tools/bench_wide.py > out.json
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    assert os.environ.get("D3A_WIDE_STAMPS") == "1", "run with D3A_WIDE_STAMPS=1"
    from d3rlpy_amd import _native as N
    torch.cuda.set_device(0)
    algo, it = bench.build_workload(0, 100_000, "bcq")
    bench.gpu_steps(algo, it, 5)
    torch.cuda.synchronize()
    launch, flops, desc = next(iter(algo.impl._ws.values())).dominant_kernel()
    out = {"kernel": desc, "phase_names": ["second tile: weight reloads", "x barrier", "layer 1 + image 1",
                                                  "layer 2", "image 2", "head", "stores + mean"]}
    # D3A_WIDE_ABL: 0 as built; 1 no W1 refetch, 2 no layer-1 production in the
    # loop, 4 no loop barriers, 8 no Wh refetch, 16 no input loads, 32 / 64 no
    # W1 / Wh split (timing only)
    for abl in [int(a) for a in os.environ.get("ABLS", "0,1,2,4,8,16,9,15,32,64,96").split(",")]:
        os.environ["D3A_WIDE_ABL"] = str(abl)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for _ in range(10):
            launch()
        ev[0].record()
        for _ in range(20):
            launch()
        ev[1].record()
        torch.cuda.synchronize()
        us = ev[0].elapsed_time(ev[1]) * 1000 / 20
        n = 1024 * 9
        buf = (ctypes.c_ulonglong * n)()
        assert N.lib().d3a_wide_stamps(buf, n) == 0
        st = np.array(buf, dtype=np.float64).reshape(1024, 9)
        st = st[st[:, 8] != 0]  # workgroups of this launch (the grid may be < 1024)
        life = st[:, 8].copy()
        st = st[st[:, 0] != 0][:, :8]  # ... with a second tile
        ph = np.diff(st, axis=1)
        out[f"abl{abl}"] = {"avg_us": round(us, 2),
                            "phase_cycles_mean": [round(float(v)) for v in ph.mean(0)],
                            "tile_cycles_mean": round(float((st[:, 7] - st[:, 0]).mean())),
                            "wg_cycles_mean": round(float(life.mean())), "wg_cycles_max": round(float(life.max()))}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
