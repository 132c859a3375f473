"""Eager K2 CQL update steps (no graph: one dispatch per kernel) for a
rocprofv3 --pmc pass over every kernel of the step.

    rocprofv3 --pmc ... -d OUT -o run --output-format csv -- python3 tools/pmc_step.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    torch.cuda.set_device(0)
    algo, it = bench.build_workload(0, 200_000, "cql")
    impl = algo.impl
    for _ in range(12):
        batch = next(it)
        impl.update_step(batch, sync=False, use_graph=False)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
