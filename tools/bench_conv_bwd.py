"""Time d3a_conv_bwd_w on the K5 encoder's three layers (batch 512, the
online obs rows) -- D3A_CONV_BWD_X6=0/1 selects the fp32-MFMA or the
split-bf16 kernel.  Prints one JSON line per layer: us per launch, TFLOP/s,
the split count, and the max relative error against an fp64 torch reference."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from d3rlpy_amd import _native as N, ops  # noqa: E402

dev = torch.device("cuda:0")
B = int(os.environ.get("B", "512"))
LAYERS = [(4, 84, 84, 32, 8, 4, True), (32, 20, 20, 64, 4, 2, False), (64, 9, 9, 64, 3, 1, False)]
g = torch.Generator().manual_seed(0)
for (C, H, W, CO, K, S, u8) in LAYERS:
    OH, OW = (H - K) // S + 1, (W - K) // S + 1
    d = N.ConvDesc()
    d.B, d.C, d.H, d.W, d.KH, d.KW, d.S, d.OH, d.OW, d.CO = B, C, H, W, K, K, S, OH, OW, CO
    splits = int(os.environ.get("SPLITS", "0")) or int(N.lib().d3a_conv_bwd_w_splits(d))
    if u8:
        x = torch.randint(0, 256, (B, C, H, W), generator=g, dtype=torch.uint8)
        xn = x.double() / 255.0
    else:
        xn = torch.relu(torch.randn(B, C, H, W, generator=g, dtype=torch.float64)).float().double()
        x = xn.float().permute(0, 2, 3, 1).contiguous()
    dy = torch.randn(B, OH, OW, CO, generator=g)
    Wt = torch.randn(CO, C, K, K, generator=g) * 0.05
    xd, dyd, Wd = x.to(dev), dy.to(dev), Wt.to(dev)
    dW = torch.zeros(splits, CO, C, K, K, device=dev)
    db = torch.zeros(splits, CO, device=dev)
    if u8:
        d.x_u8 = xd.data_ptr()
    else:
        d.x_f32 = xd.data_ptr()
    d.weight, d.dy, d.dW, d.db, d.splits = Wd.data_ptr(), dyd.data_ptr(), dW.data_ptr(), \
        db.data_ptr(), splits
    for _ in range(200):
        ops.call_desc("d3a_conv_bwd_w", d)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 500
    e0.record()
    for _ in range(n):
        ops.call_desc("d3a_conv_bwd_w", d)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / n
    Wr = Wt.double().requires_grad_(True)
    out = F.conv2d(xn, Wr, None, stride=S)
    out.backward(dy.double().permute(0, 3, 1, 2))
    err = float((dW.double().sum(0).cpu() - Wr.grad).abs().max() / Wr.grad.abs().max())
    dbr = dy.double().sum((0, 1, 2))
    errb = float((db.double().sum(0).cpu() - dbr).abs().max() / dbr.abs().max())
    fl = 2.0 * B * OH * OW * CO * C * K * K
    print(json.dumps({"layer": f"{C}x{H}x{W}->{CO} k{K}s{S}", "u8": u8, "splits": splits,
                      "x6": os.environ.get("D3A_CONV_BWD_X6", "1"), "us": round(us, 2),
                      "tflops": round(fl / us / 1e6, 1), "rel_err_dW": err, "rel_err_db": errb}),
          flush=True)

# the input gradient of layers 2 and 3 (d3a_conv_bwd_x vs the column GEMM + col2im pair)
for (C, H, W, CO, K, S, _) in LAYERS[1:]:
    OH, OW = (H - K) // S + 1, (W - K) // S + 1
    d = N.ConvDesc()
    d.B, d.C, d.H, d.W, d.KH, d.KW, d.S, d.OH, d.OW, d.CO = B, C, H, W, K, K, S, OH, OW, CO
    x = torch.relu(torch.randn(B, H, W, C, generator=g)).to(dev)
    dy = torch.randn(B * OH * OW, CO, generator=g).to(dev)
    Wt = (torch.randn(CO, C, K, K, generator=g) * 0.05).to(dev)
    dx = torch.empty(B * H * W, C, device=dev)
    wpack = torch.empty(CO * C * K * K, device=dev)
    d.x_f32, d.weight, d.dy, d.y, d.relu = x.data_ptr(), Wt.data_ptr(), dy.data_ptr(), \
        dx.data_ptr(), 1
    if os.environ.get("PACKED", "1") == "1":
        d.wpack = wpack.data_ptr()
    for _ in range(100):
        ops.call_desc("d3a_conv_bwd_x", d)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(300):
        ops.call_desc("d3a_conv_bwd_x", d)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 300
    fl = 2.0 * B * OH * OW * CO * C * K * K
    print(json.dumps({"bwd_x": f"{C}x{H}x{W}->{CO} k{K}s{S}", "us": round(us, 2),
                      "tflops_useful": round(fl / us / 1e6, 1)}), flush=True)
