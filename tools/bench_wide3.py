"""Phase stamps of the CQL reproduction critic's three-layer x6 forward
(mlp_x6_wide_kernel<32, true, true, 3, true>, D3A_WIDE_STAMPS=1): per-workgroup
cycles from the tile's start to each phase boundary (0 start, 1 before the
input barrier, 2 after it, 3 image 1 written, 4 layer-2 products issued,
5 image 2 written, 6 layer-3 products issued, 7 head written) and the
workgroup lifetimes.

    D3A_WIDE_STAMPS=1 python tools/bench_wide3.py
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
    algo, it = bench.build_workload(0, 100_000, "cqlrepro")
    bench.gpu_steps(algo, it, 5)
    torch.cuda.synchronize()
    launch, flops, desc = next(iter(algo.impl._ws.values())).dominant_kernel()
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
    st = st[st[:, 8] != 0]
    life = st[:, 8].copy()
    ok = st[(st[:, 0] != 0) & (st[:, 7] != 0)][:, :8]
    rel = ok - ok[:, :1]
    out = {"kernel": desc, "avg_us": round(us, 2), "n_wg": int(len(life)),
           "cum_cycles_mean": [round(float(v)) for v in rel.mean(0)],
           "phase_cycles_mean": [round(float(v)) for v in np.diff(ok, axis=1).mean(0)],
           "wg_cycles_mean": round(float(life.mean())), "wg_cycles_max": round(float(life.max())),
           # (single-tile workgroups: lifetime - tile = the kernel prologue)
           "prologue_cycles_mean": round(float((st[(st[:, 0] != 0) & (st[:, 7] != 0)][:, 8]
                                               - (ok[:, 7] - ok[:, 0])).mean()))}
    # every wave: cycles from the workgroup's tile start (wave 0's stamp 0)
    wb = (ctypes.c_ulonglong * (512 * 64))()
    assert N.lib().d3a_wide_wave_stamps(wb, 512 * 64) == 0
    ws = np.array(wb, dtype=np.float64).reshape(512, 8, 8)
    ws = ws[(ws != 0).all(axis=(1, 2))]
    rel = ws - ws[:, :1, :1]
    out["wave_cum_cycles_mean"] = [[round(float(v)) for v in rel[:, w].mean(0)] for w in range(8)]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
