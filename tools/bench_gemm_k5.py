"""Variant / split sweep of d3a_gemm_f32 on the DiscreteCQL-IQN (K5) GEMM
shapes: IQN embed forward and weight gradient, encoder fc forward / weight
gradient.  Interleaved rounds, median us per (shape, variant, splits)."""
import sys

import torch

sys.path.insert(0, ".")
from d3rlpy_amd import ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    B, K, F, E, FLAT = 512, 64, 512, 64, 3136
    R = 3 * B * K
    prior = torch.rand(4 * B * K, E, device=dev, generator=g)
    Wemb = torch.randn(F, E, device=dev, generator=g) * 0.1
    bemb = torch.randn(F, device=dev, generator=g)
    phi = torch.empty(4 * B * K, F, device=dev)
    dphi = torch.randn(R, F, device=dev, generator=g)
    dW = torch.empty(128 * F * max(E, FLAT), device=dev)
    db = torch.empty(128 * F, device=dev)
    yt = torch.randn(2 * B, FLAT, device=dev, generator=g)
    Wfc = torch.randn(F, FLAT, device=dev, generator=g) * 0.02
    bfc = torch.randn(F, device=dev, generator=g)
    h = torch.empty(2 * B, F, device=dev)
    dz = torch.randn(B, F, device=dev, generator=g)

    cases = []
    for v in (0, 2, 3, 9, 10):
        cases.append((f"embed_fwd[131072x512x64] v{v}", 2 * 4 * B * K * E * F, lambda v=v: ops.gemm(
            prior.data_ptr(), Wemb.data_ptr(), phi.data_ptr(), 4 * B * K, F, E, sA=(0, E, 1),
            sB=(0, 1, E), sC=(0, F, 1), bias=bemb.data_ptr(), relu=True, variant=v)))
    for v in (0, 9, 10):
        for s in (32, 64, 128):
            cases.append((f"embed_dW[512x64x98304] v{v} s{s}", 2 * R * E * F, lambda v=v, s=s:
                          ops.linear_bwd_w(dphi.data_ptr(), F, R * F, prior.data_ptr(), E, R * E,
                                           dW.data_ptr(), 1, R, E, F, s, db=db.data_ptr(),
                                           variant=v)))
    for v in (0, 2, 3, 9, 10):
        cases.append((f"fc_fwd[1024x512x3136] v{v}", 2 * 2 * B * FLAT * F, lambda v=v: ops.gemm(
            yt.data_ptr(), Wfc.data_ptr(), h.data_ptr(), 2 * B, F, FLAT, sA=(0, FLAT, 1),
            sB=(0, 1, FLAT), sC=(0, F, 1), bias=bfc.data_ptr(), relu=True, variant=v)))
    for v in (0, 9):
        for s in (1, 4, 16):
            cases.append((f"fc_dW[512x3136x512] v{v} s{s}", 2 * B * FLAT * F, lambda v=v, s=s:
                          ops.linear_bwd_w(dz.data_ptr(), F, B * F, yt.data_ptr(), FLAT,
                                           B * FLAT, dW.data_ptr(), 1, B, FLAT, F, s,
                                           db=db.data_ptr(), variant=v)))
    res = {c[0]: [] for c in cases}
    for rnd in range(5):
        for name, flops, fn in cases:
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) * 100.0)  # us per call
    for name, flops, fn in cases:
        t = sorted(res[name])[2]
        print(f"{name:42s} {t:8.1f} us  {flops / t / 1e6:7.1f} TF")


if __name__ == "__main__":
    main()
