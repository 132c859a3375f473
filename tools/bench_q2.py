"""Microbenchmark of d3a_q2_bwd on the K2 CQL critic-backward shape (7,936 rows
x 2 members, 14 -> 256 -> 256 -> 1): average launch time by HIP events on the
launching stream, and the fp32 MFMA fraction of the 4.21 GFLOP it performs
(dX 2.08 + dW2 2.08 + dW1 0.06, padded to 32 inputs).  Used for the rocprofv3
PMC passes of the kernel (tools/gpu_r03_pmc_q2.sh)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from d3rlpy_amd import _native as N  # noqa: E402
from d3rlpy_amd import ops  # noqa: E402

H = 256


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=7936)
    ap.add_argument("--n-in", type=int, default=14)
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--x6", action="store_true", help="d3a_q2_bwd_x6 (split-bf16, fp32-accurate)")
    ap.add_argument("--mask", choices=["none", "rows", "slice"], default="none",
                    help="x6 only: rows = the forward's row mask bits (m2, the 256-row-block "
                         "kernel); slice = row + transposed mask bits (m2 + m2t, the slice kernel "
                         "of q2_x6_bwd2.hip: no h2, P row blocks)")
    a = ap.parse_args()
    rows, n_in, Cm, dev = a.rows, a.n_in, 2, "cuda"
    ldx = (n_in + 3) // 4 * 4
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(rows, ldx, device=dev, generator=g)
    h1 = torch.relu(torch.randn(Cm, rows, H, device=dev, generator=g))
    h2 = torch.relu(torch.randn(Cm, rows, H, device=dev, generator=g))
    gr = torch.randn(Cm, rows, device=dev, generator=g) * 1e-2
    gs = torch.tensor([0.7], device=dev)
    W2 = torch.randn(Cm, H, H, device=dev, generator=g) * 0.06
    w3 = torch.randn(Cm, H, device=dev, generator=g) * 0.06
    P = (rows + 255) // 256
    if a.mask == "slice":
        P = N.lib().d3a_q2_bwd_x6t_splits(rows, Cm)
    outs = [torch.zeros(P, Cm, H, n_in, device=dev), torch.zeros(P, Cm, H, device=dev),
            torch.zeros(P, Cm, H, H, device=dev), torch.zeros(P, Cm, H, device=dev),
            torch.zeros((16 if a.mask == "slice" else 1) * P, Cm, H, device=dev),
            torch.zeros(P, Cm, device=dev)]
    b2 = torch.randn(Cm, H, device=dev, generator=g) * 0.1
    words = torch.randint(-2 ** 31, 2 ** 31 - 1, (Cm, rows, H // 32), device=dev, generator=g,
                          dtype=torch.int64).to(torch.int32)
    wordsT = torch.randint(-2 ** 31, 2 ** 31 - 1, (Cm, (rows + 31) // 32, H), device=dev,
                           generator=g, dtype=torch.int64).to(torch.int32)
    entry = "d3a_q2_bwd_x6" if a.x6 else "d3a_q2_bwd"
    d = N.Q2BwdDesc()
    d.x, d.ldx, d.sxb = x.data_ptr(), ldx, 0
    d.h1, d.h2, d.sh, d.ldh = h1.data_ptr(), h2.data_ptr(), rows * H, H
    d.g, d.sgb, d.gscale, d.n_scaled = gr.data_ptr(), rows, gs.data_ptr(), rows * 30 // 31
    d.W2, d.sW2, d.w3, d.sw3 = W2.data_ptr(), H * H, w3.data_ptr(), H
    d.dW1, d.db1, d.dW2, d.db2, d.dW3, d.db3 = [t.data_ptr() for t in outs]
    d.rows, d.n_in, d.C = rows, n_in, Cm
    if a.mask in ("rows", "slice"):
        d.m2, d.sm2 = words.data_ptr(), rows * (H // 32)
    if a.mask == "slice":
        d.m2t, d.sm2t = wordsT.data_ptr(), wordsT.shape[1] * H
        d.b2, d.sb2 = b2.data_ptr(), H
        d.h2 = None
    for _ in range(5):
        ops.call_desc(entry, d)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(a.reps):
        ops.call_desc(entry, d)
    e1.record(s)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / a.reps
    flops = 2 * Cm * rows * (2 * H * H + H * 32)
    print(json.dumps({"kernel": entry, "mask": a.mask, "P": P, "rows": rows, "n_in": n_in,
                      "avg_us": round(us, 2),
                      "tflops": round(flops / us / 1e6, 2),
                      "frac_fp32_peak": round(flops / us / 1e6 / 157.3, 4)}))


if __name__ == "__main__":
    main()
