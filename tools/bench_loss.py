"""Time the CQL loss stage (d3a_cql_loss) by section: the K2 workload's own
descriptor launched alone with update_temp / update_alpha / update_critic
switched on and off (a graph of 50 calls replayed 10 times; the
scalar states drift, which does not change the work).  JSON lines."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from d3rlpy_amd import ops  # noqa: E402


def main():
    torch.cuda.set_device(0)
    algo, it = bench.build_workload(0, 200_000, "cql")
    bench.gpu_steps(algo, it, 5)
    torch.cuda.synchronize()
    ws = next(iter(algo.impl._ws.values()))
    l = ws.loss_desc
    for temp, alpha, critic in ((1, 1, 1), (0, 0, 1), (1, 0, 0), (0, 1, 0), (0, 0, 0)):
        l.update_temp, l.update_alpha, l.update_critic = temp, alpha, critic
        ops.call_desc("d3a_cql_loss", l)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with ops.graph_capture(g):  # 50 back-to-back calls, replayed (no host gaps)
            for _ in range(50):
                ops.call_desc("d3a_cql_loss", l)
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        print(json.dumps({"temp": temp, "alpha": alpha, "critic": critic,
                          "us_per_call": round(e0.elapsed_time(e1) * 1000 / 500, 2)}), flush=True)
    l.update_temp, l.update_alpha, l.update_critic = 1, 1, 1


if __name__ == "__main__":
    main()
