"""The ensemble-Q layer GEMM (K2 critic layer 1: 2 members x 15,616 rows x
256 x 256, y = relu(x W^T + b)) in fp32 MFMA (d3a_gemm_f32, automatic tile)
and split-bf16 (d3a_gemm_sbf16, 3 and 6 terms): one JSON line per variant,
interleaved rounds, median; roofline against the dense peak of the matrix
instruction each variant issues (fp32 157.3 TF, bf16 2,500 TF: issued bf16
FLOP = terms x the algorithmic FLOP)."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from d3rlpy_amd import ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    C, R, H = 2, 15616, 256
    x = torch.relu(torch.randn(R, H, device=dev, generator=g))
    W = torch.randn(C, H, H, device=dev, generator=g) * 0.0625
    b = torch.randn(C, H, device=dev, generator=g)
    y = torch.empty(C, R, H, device=dev)
    flops = 2 * C * R * H * H
    runs = {
        "fp32_mfma": lambda: ops.linear_fwd(x.data_ptr(), True, H, W.data_ptr(), b.data_ptr(),
                                            y.data_ptr(), C, R, H, H, relu=True, ldy=H, sxb=0,
                                            syb=R * H),
        "sbf16x3": lambda: ops.gemm_sbf16(x, W, b, y, terms=3, relu=True),
        "sbf16x6": lambda: ops.gemm_sbf16(x, W, b, y, terms=6, relu=True),
    }
    times = {k: [] for k in runs}
    reps = 50
    for _ in range(5):
        for k, fn in runs.items():
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / 1e3 / reps)
    for k in runs:
        t = statistics.median(times[k])
        terms = {"fp32_mfma": 1, "sbf16x3": 3, "sbf16x6": 6}[k]
        peak = 157.3 if k == "fp32_mfma" else 2500.0
        issued = flops * terms / t / 1e12
        print(json.dumps({"metric": "ensemble-Q layer GEMM throughput (K2 critic layer 1)",
                          "variant": k, "us": round(t * 1e6, 2),
                          "effective_tflops": round(flops / t / 1e12, 2),
                          "issued_tflops": round(issued, 2), "peak_tflops": peak,
                          "frac_of_peak": round(issued / peak, 4),
                          "shape": f"{C} x [{R} x {H}] @ [{H} x {H}]"}))


if __name__ == "__main__":
    main()
