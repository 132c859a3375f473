"""Launch only the bench's dominant kernel (for a rocprofv3 --pmc pass).

    rocprofv3 --pmc FETCH_SIZE -d OUT -o run --output-format csv -- \
        python3 tools/pmc_dominant.py [--algo cql] [--reps 20]

Builds the same workload as bench.py, runs a few warm updates (so every
buffer holds real data), then launches the dominant kernel --reps times.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--algo", default="cql")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--transitions", type=int, default=200_000)
    ap.add_argument("--precision", choices=["fp32", "bf16", "bf16h"], default="fp32")
    ap.add_argument("--critic-gemm", choices=["fp32", "x6"], default=None)
    ap.add_argument("--backward", action="store_true",
                    help="launch the critic backward (backward_kernel) instead: the bench "
                         "line's lead kernel when it outlasts the forward")
    ap.add_argument("--desc-out", default=None,
                    help="write {desc, flops} of the launched kernel here (bench.py matches a "
                         "traffic file to its line by this desc)")
    a = ap.parse_args()
    from d3rlpy_amd import ops
    if a.precision != "fp32":
        ops.set_critic_precision(a.precision)
    if a.critic_gemm:
        ops.set_critic_gemm(a.critic_gemm)
    torch.cuda.set_device(0)
    algo, it = bench.build_workload(0, a.transitions, a.algo)
    bench.gpu_steps(algo, it, 5)
    torch.cuda.synchronize()
    wsp = next(iter(algo.impl._ws.values()))
    launch, flops, desc = wsp.backward_kernel() if a.backward else wsp.dominant_kernel()
    for _ in range(a.reps):
        launch()
    torch.cuda.synchronize()
    print(desc, flops)
    if a.desc_out:
        import json
        with open(a.desc_out, "w") as f:
            json.dump({"desc": desc, "flops": flops, "algo": a.algo}, f)


if __name__ == "__main__":
    main()
