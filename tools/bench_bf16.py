"""Microbenchmark of the bf16 critic kernels on the K2 shapes: d3a_q2_fwd_bf16
(2 x (15,616 + 256) rows) and d3a_q2_bwd_bf16 (2 x 7,936 rows), average
launch time by HIP events on the launching stream and the fraction of the
2.5 PF dense bf16 peak (D3A_BF16_PROBE selects the backward's timing probes)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from d3rlpy_amd import _native as N  # noqa: E402
from d3rlpy_amd import ops  # noqa: E402


def timed(fn, reps=200):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    dev, C, H, n_in = "cuda", 2, 256, 14
    g = torch.Generator(device=dev).manual_seed(0)
    # backward
    rows = 7936
    x = torch.randn(rows, 16, device=dev, generator=g)
    h1 = torch.relu(torch.randn(C, rows, H, device=dev, generator=g)).to(torch.bfloat16)
    h2 = torch.relu(torch.randn(C, rows, H, device=dev, generator=g)).to(torch.bfloat16)
    gr = torch.randn(C, rows, device=dev, generator=g) * 1e-2
    gs = torch.tensor([0.7], device=dev)
    W2 = torch.randn(C, H, H, device=dev, generator=g) * 0.06
    w3 = torch.randn(C, H, device=dev, generator=g) * 0.06
    P = (rows + 255) // 256
    outs = [torch.zeros(P, C, H, n_in, device=dev), torch.zeros(P, C, H, device=dev),
            torch.zeros(P, C, H, H, device=dev), torch.zeros(P, C, H, device=dev),
            torch.zeros(P, C, H, device=dev), torch.zeros(P, C, device=dev)]
    d = N.Q2BwdDesc()
    d.x, d.ldx, d.sxb = x.data_ptr(), 16, 0
    d.h1, d.h2, d.sh, d.ldh = h1.data_ptr(), h2.data_ptr(), rows * H, H
    d.g, d.sgb, d.gscale, d.n_scaled = gr.data_ptr(), rows, gs.data_ptr(), rows * 30 // 31
    d.W2, d.sW2, d.w3, d.sw3 = W2.data_ptr(), H * H, w3.data_ptr(), H
    d.dW1, d.db1, d.dW2, d.db2, d.dW3, d.db3 = [t.data_ptr() for t in outs]
    d.rows, d.n_in, d.C = rows, n_in, C
    us = timed(lambda: ops.call_desc("d3a_q2_bwd_bf16", d))
    flops = 2 * C * rows * (2 * H * H + H * 32)
    print(json.dumps({"kernel": "d3a_q2_bwd_bf16", "probe": os.environ.get("D3A_BF16_PROBE", "0"),
                      "avg_us": round(us, 2), "tflops": round(flops / us / 1e6, 1),
                      "frac_bf16_peak": round(flops / us / 1e6 / 2500.0, 4)}))


if __name__ == "__main__":
    main()
