"""Tile-variant sweep of d3a_gemm_f32 on the CQL (K2) GEMM shapes.

Interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24);
random operands; prints TFLOP/s per (shape, variant): median of rounds.
"""
import json
import sys

import torch

sys.path.insert(0, ".")
from d3rlpy_amd import ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    C, R, Rc, H, DA = 2, 15616, 7936, 256, 14
    X = torch.randn(R, H, device=dev, generator=g)
    Xc = torch.randn(C, Rc, H, device=dev, generator=g)
    W = torch.randn(C, H, H, device=dev, generator=g) * 0.06
    b = torch.randn(C, H, device=dev, generator=g)
    Y = torch.empty(C, R, H, device=dev)
    dZ = torch.randn(C, Rc, H, device=dev, generator=g)
    dW = torch.empty(32, C, H, H, device=dev)
    db = torch.empty(32, C, H, device=dev)
    out = torch.empty(C, Rc, H, device=dev)

    shapes = {
        "fwd_l2[2x15616x256x256]": (2 * C * R * H * H, lambda v: ops.gemm(
            X.data_ptr(), W.data_ptr(), Y.data_ptr(), R, H, H, batch=C, sA=(0, H, 1),
            sB=(H * H, 1, H), sC=(R * H, H, 1), bias=b.data_ptr(), sbias=H, relu=True, variant=v)),
        "dW2[2x256x256x7936] s31": (2 * C * Rc * H * H, lambda v: ops.linear_bwd_w(
            dZ.data_ptr(), H, Rc * H, Xc.data_ptr(), H, Rc * H, dW.data_ptr(), C, Rc, H, H, 31,
            db=db.data_ptr(), variant=v)),
        "dW2[2x256x256x7936] s16": (2 * C * Rc * H * H, lambda v: ops.linear_bwd_w(
            dZ.data_ptr(), H, Rc * H, Xc.data_ptr(), H, Rc * H, dW.data_ptr(), C, Rc, H, H, 16,
            db=db.data_ptr(), variant=v)),
        "dX[2x7936x256x256]+mask": (2 * C * Rc * H * H, lambda v: ops.gemm(
            dZ.data_ptr(), W.data_ptr(), out.data_ptr(), Rc, H, H, batch=C, sA=(Rc * H, H, 1),
            sB=(H * H, H, 1), sC=(Rc * H, H, 1), mask=Xc.data_ptr(), sM=(Rc * H, H, 1),
            variant=v)),
        "pol_fwd[512x256x256]": (2 * 512 * H * H, lambda v: ops.gemm(
            X.data_ptr(), W.data_ptr(), Y.data_ptr(), 512, H, H, batch=1, sA=(0, H, 1),
            sB=(H * H, 1, H), sC=(R * H, H, 1), bias=b.data_ptr(), sbias=H, relu=True,
            variant=v)),
    }
    variants = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else \
        [0, 3, 5, 11, 12, 13, 14, 15, 16, 17, 18]
    res = {k: {v: [] for v in variants} for k in shapes}
    reps = 20
    for rnd in range(3):
        for name, (flops, fn) in shapes.items():
            for v in variants:
                for _ in range(2):
                    fn(v)
                s = torch.cuda.current_stream()
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(reps):
                    fn(v)
                e1.record(s)
                torch.cuda.synchronize()
                t = e0.elapsed_time(e1) / 1e3 / reps
                res[name][v].append(t)
    out_tbl = {}
    for name, (flops, _) in shapes.items():
        row = {}
        for v in variants:
            ts = sorted(res[name][v])
            med = ts[len(ts) // 2]
            row[v] = {"us": round(med * 1e6, 2), "tflops": round(flops / med / 1e12, 1)}
        out_tbl[name] = row
        print(name, " ".join(f"v{v}:{row[v]['us']}us/{row[v]['tflops']}TF" for v in variants))
    print(json.dumps(out_tbl))


if __name__ == "__main__":
    main()
