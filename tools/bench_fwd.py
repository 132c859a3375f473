"""Microbenchmark of d3a_mlp_fwd on the K2 CQL critic-forward shape: 2 members
x (15,616 Q rows, activations kept for rows >= 7,680, + 256 target rows as the
aux pass) x 14 -> 256 -> 256 -> 1.  Average launch time by HIP events on the
launching stream and the fp32 MFMA fraction of the 4.41 GFLOP it performs.
Used for A/B runs of the kernel and its rocprofv3 PMC passes."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from d3rlpy_amd import _native as N  # noqa: E402
from d3rlpy_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=15616)
    ap.add_argument("--h-from", type=int, default=7680)
    ap.add_argument("--aux", type=int, default=256)
    ap.add_argument("--n-in", type=int, default=14)
    ap.add_argument("--bm", type=int, default=0)
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--C", type=int, default=2)
    ap.add_argument("--J", type=int, default=1)
    ap.add_argument("--bf16", action="store_true", help="d3a_q2_fwd_bf16 (bf16 kept activations)")
    ap.add_argument("--x6", action="store_true", help="d3a_q2_fwd_x6 (split-bf16 x6, fp32-accurate)")
    ap.add_argument("--hmask", action="store_true", help="x6: also write the bf16 mask image of h2")
    ap.add_argument("--slice", action="store_true",
                    help="x6: the production critic forward of the slice backward -- row and "
                         "transposed mask bits, no kept h2")
    ap.add_argument("--pre", action="store_true",
                    help="x6: W0 / W1 streamed as pre-split images (d3a_x6_split, desc.wp)")
    ap.add_argument("--warm", type=int, default=5, help="untimed launches before the timed ones")
    ap.add_argument("--stamps", action="store_true",
                    help="with D3A_X6_PROBE=16: per-phase s_memtime cycles of wave 0, averaged "
                         "over the workgroups")
    a = ap.parse_args()
    if a.slice:
        a.hmask = True
    dev, C, H = "cuda", a.C, 256
    sizes = [a.n_in, H, H, a.J]
    ldx = (a.n_in + 3) // 4 * 4
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(a.rows, ldx, device=dev, generator=g)
    xa = torch.randn(max(a.aux, 1), ldx, device=dev, generator=g)
    # parameters: one buffer per store, [W0 b0 W1 b1 W2 b2] per member-major layer
    n_par = sum(C * (sizes[l] * sizes[l + 1] + sizes[l + 1]) for l in range(3))
    n_par = (n_par + 3) // 4 * 4
    store = torch.randn(2 * n_par, device=dev, generator=g) * 0.06
    offs, o = [], 0
    for l in range(3):
        w = o
        o += C * sizes[l] * sizes[l + 1]
        o = (o + 3) // 4 * 4
        b = o
        o += C * sizes[l + 1]
        o = (o + 3) // 4 * 4
        offs.append((w, b))
    h = [torch.zeros(C, a.rows, H, device=dev,
                     dtype=torch.bfloat16 if a.bf16 else torch.float32) for _ in range(2)]
    entry = "d3a_q2_fwd_bf16" if a.bf16 else "d3a_q2_fwd_x6" if a.x6 else "d3a_mlp_fwd"
    out = torch.zeros(C, a.rows, a.J, device=dev)
    aout = torch.zeros(C, max(a.aux, 1), a.J, device=dev)
    d = N.MlpFwdDesc()
    d.block_rows = a.bm
    d.x, d.ldx, d.sxb = x.data_ptr(), ldx, 0
    d.n_in, d.n_hidden, d.H, d.n_out = a.n_in, 2, H, 1
    for l in range(3):
        d.W[l] = store.data_ptr() + 4 * offs[l][0]
        d.b[l] = store.data_ptr() + 4 * offs[l][1]
        d.sW[l], d.sb[l] = sizes[l + 1] * sizes[l], sizes[l + 1]
    for l in range(2):
        d.h[l] = h[l].data_ptr()
    d.sh = a.rows * H
    d.out, d.sout, d.ldout = out.data_ptr(), a.rows * a.J, a.J
    d.r0, d.rows, d.C, d.h_from = 0, a.rows, C, a.h_from
    if a.hmask:
        hm = torch.zeros(C, a.rows, H // 32, device=dev, dtype=torch.int32)
        d.hmask, d.s_hmask = hm.data_ptr(), a.rows * (H // 32)
    if a.slice:
        hmt = torch.zeros(C, (a.rows + 31) // 32, H, device=dev, dtype=torch.int32)
        d.hmaskT, d.s_hmaskT = hmt.data_ptr(), hmt[0].numel()
        d.h[1] = None
    if a.aux:
        d.aux_x, d.aux_ldx, d.aux_sxb, d.aux_wdelta = xa.data_ptr(), ldx, 0, n_par
        d.aux_out, d.aux_sout, d.aux_rows = aout.data_ptr(), a.aux * a.J, a.aux
    if a.pre:
        xl = (a.n_in + 15) // 16 * 16
        imgs = []
        for si in range(2 if a.aux else 1):
            w0 = torch.zeros(C * H * xl * 3, dtype=torch.bfloat16, device=dev)
            w1 = torch.zeros(C * H * H * 3, dtype=torch.bfloat16, device=dev)
            sd = N.X6SplitDesc()
            for i, (l, im, k, kp) in enumerate(((0, w0, a.n_in, xl), (1, w1, H, H))):
                sd.job[i].src = store.data_ptr() + 4 * (si * n_par + offs[l][0])
                sd.job[i].dst, sd.job[i].rows, sd.job[i].k, sd.job[i].kpad = im.data_ptr(), C * H, k, kp
            sd.n_jobs = 2
            ops.call_desc("d3a_x6_split", sd)
            imgs.append((w0, w1))
        d.wp[0], d.wp[1] = imgs[0][0].data_ptr(), imgs[0][1].data_ptr()
        if a.aux:
            d.aux_wp[0], d.aux_wp[1] = imgs[1][0].data_ptr(), imgs[1][1].data_ptr()
    for _ in range(a.warm):
        ops.call_desc(entry, d)
    torch.cuda.synchronize()
    # check against torch fp32 on a row sample
    W = [store[offs[l][0]:offs[l][0] + C * sizes[l] * sizes[l + 1]].view(C, sizes[l + 1], sizes[l])
         for l in range(3)]
    bb = [store[offs[l][1]:offs[l][1] + C * sizes[l + 1]].view(C, 1, sizes[l + 1]) for l in range(3)]
    xs = x[:, :a.n_in]
    r1 = torch.relu(xs @ W[0].transpose(1, 2) + bb[0])
    r2 = torch.relu(r1 @ W[1].transpose(1, 2) + bb[1])
    q = r2 @ W[2].transpose(1, 2) + bb[2]
    err = ((q - out).abs().max() / q.abs().max()).item()
    herr = (None if a.slice else
            ((r2[:, a.h_from:] - h[1][:, a.h_from:].float()).abs().max()).item())
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(a.reps):
        ops.call_desc(entry, d)
    e1.record(s)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / a.reps
    flops = 2 * C * (a.rows + a.aux) * sum(sizes[l] * sizes[l + 1] for l in range(3))
    stamps = None
    if a.stamps:
        import ctypes
        n = 2048 * 10
        buf = (ctypes.c_ulonglong * n)()
        assert N.lib().d3a_x6_stamps(buf, n) == 0
        import numpy as np
        st = np.frombuffer(buf, dtype=np.uint64).reshape(2048, 10).astype(np.int64)
        nwg = min(2048, (a.rows + 127) // 128 * C)
        st = st[:nwg]
        ph = np.diff(st[:, :9], axis=1)
        stamps = {"phase_cycles_mean": [round(float(v), 1) for v in ph.mean(0)],
                  "total_cycles_mean": round(float((st[:, 8] - st[:, 0]).mean()), 1)}
    print(json.dumps({"kernel": entry, "pre": a.pre, "hmask": a.hmask, "slice": a.slice, "rows": a.rows, "aux": a.aux, "bm": a.bm, "C": C, "J": a.J,
                      "variant": os.environ.get("D3A_FWD_PROBE", "") + os.environ.get("D3A_X6_PROBE", "") + ("generic" if os.environ.get("D3A_FWD_Q2") == "0" else ""),
                      "stamps": stamps,
                      "avg_us": round(us, 2), "tflops": round(flops / us / 1e6, 2),
                      "frac_fp32_peak": round(flops / us / 1e6 / 157.3, 4),
                      "max_rel_err_q": err, "max_abs_err_h2": herr}))


if __name__ == "__main__":
    main()
