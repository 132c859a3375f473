"""Phase stamps of the K2 slice critic backward (D3A_BWD_STAMPS=1): the
pipeline's launch (with the CQL loss stage in its prologue, or without it:
--plain) after a few updates; mean cycles per phase for the row waves (wave 0)
and the col waves (wave 4) over the workgroups, and workgroup 0's."""
import argparse
import ctypes
import json
import os
import sys

os.environ["D3A_BWD_STAMPS"] = "1"
import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--plain", action="store_true")
    a = ap.parse_args()
    from d3rlpy_amd.algos import cql_impl
    if a.plain:
        cql_impl._LOSS_IN_BWD = False
    from d3rlpy_amd import _native as N
    torch.cuda.set_device(0)
    algo, it = bench.build_workload(0, 100_000, "cql")
    bench.gpu_steps(algo, it, 30)
    torch.cuda.synchronize()
    ws = next(iter(algo.impl._ws.values()))
    launch, _, desc = ws.backward_kernel()
    for _ in range(200):
        launch()
    torch.cuda.synchronize()
    n = 256 * 2 * 8
    buf = (ctypes.c_ulonglong * n)()
    assert N.lib().d3a_bwd_stamps(buf, n) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(256, 2, 8).astype(np.int64)
    out = {"kernel": desc}
    for wv, name in ((0, "row_wave0"), (1, "col_wave4")):
        ph = np.diff(st[:, wv, :7], axis=1)
        out[name] = {"phase_mean": [round(float(v), 1) for v in ph.mean(0)],
                     "phase_wg0": [int(v) for v in ph[0]],
                     "total_mean": round(float((st[:, wv, 6] - st[:, wv, 0]).mean()), 1),
                     "total_max": int((st[:, wv, 6] - st[:, wv, 0]).max())}
    out["start_spread"] = int(st[:, 0, 0].max() - st[:, 0, 0].min())
    out["end_spread"] = int(st[:, 0, 6].max() - st[:, 0, 0].min())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
