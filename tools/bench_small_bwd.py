"""Timing and phase stamps of d3a_mlp_bwd_small (the small-batch MLP backward
on the fp32 matrix cores) at K3's shapes.

    D3A_SB_STAMPS=1 python tools/bench_small_bwd.py
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from d3rlpy_amd import _native as N  # noqa: E402
from d3rlpy_amd import ops  # noqa: E402


def case(R, C, n_in, n_out, dx):
    dev = torch.device("cuda")
    H = 256
    g = torch.Generator().manual_seed(0)
    mk = lambda *s: (torch.randn(*s, generator=g) * 0.1).to(dev)  # noqa: E731
    x, h1, h2 = mk(R, n_in + 1), mk(C, R, H).relu(), mk(C, R, H).relu()
    dout = mk(C, R, n_out)
    W1, W2, W3 = mk(C, H, n_in), mk(C, H, H), mk(C, n_out, H)
    nrb = (R + 31) // 32
    outs = [torch.empty(nrb, C, H, n_in, device=dev), torch.empty(nrb, C, H, device=dev),
            torch.empty(nrb, C, H, H, device=dev), torch.empty(nrb, C, H, device=dev),
            torch.empty(nrb, C, n_out, H, device=dev), torch.empty(nrb, C, n_out, device=dev)]
    dxb = torch.empty(C, R, n_in, device=dev)
    scratch = torch.zeros(8, C, R, H, device=dev)
    tickets = torch.zeros(C, nrb, dtype=torch.int32, device=dev)
    d = N.MlpBwdSmallDesc()
    d.x, d.ldx, d.sxb = x.data_ptr(), n_in + 1, 0
    d.h1, d.h2, d.sh = h1.data_ptr(), h2.data_ptr(), R * H
    d.dout, d.ld_dout, d.sdout = dout.data_ptr(), n_out, R * n_out
    d.W1, d.W2, d.W3 = W1.data_ptr(), W2.data_ptr(), W3.data_ptr()
    d.sW1, d.sW2, d.sW3 = H * n_in, H * H, n_out * H
    for k, t in zip(("dW1", "db1", "dW2", "db2", "dW3", "db3"), outs):
        setattr(d, k, t.data_ptr())
    d.dx = dxb.data_ptr() if dx else None
    d.scratch, d.tickets = scratch.data_ptr(), tickets.data_ptr()
    d.rows, d.n_in, d.n_out, d.C = R, n_in, n_out, C
    for _ in range(10):
        ops.call_desc("d3a_mlp_bwd_small", d)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(50):
        ops.call_desc("d3a_mlp_bwd_small", d)
    ev[1].record()
    torch.cuda.synchronize()
    us = ev[0].elapsed_time(ev[1]) * 1000 / 50
    out = {"R": R, "C": C, "n_in": n_in, "n_out": n_out, "dx": dx, "us_both_launches": round(us, 2)}
    if os.environ.get("D3A_SB_STAMPS") == "1":
        n = 2 * 1024 * 4
        buf = (ctypes.c_ulonglong * n)()
        assert N.lib().d3a_small_bwd_stamps(buf, n) == 0
        st = np.array(buf, dtype=np.float64).reshape(2, 1024, 4)
        for k, nwg in (("A", 8 * nrb * C), ("B", nrb * C)):
            a = st[0 if k == "A" else 1, :nwg]
            out[f"stage{k}_phase_cycles"] = [round(float(v)) for v in np.diff(a, axis=1).mean(0)]
            out[f"stage{k}_start_spread"] = round(float(a[:, 0].max() - a[:, 0].min()))
    print(json.dumps(out))


if __name__ == "__main__":
    torch.cuda.set_device(0)
    case(256, 1, 29, 6, True)     # VAE decoder
    case(256, 2, 23, 200, False)  # QR critics
