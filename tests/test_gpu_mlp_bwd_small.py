"""d3a_mlp_bwd_small (the whole backward of a small-batch [n_in, 256, 256,
n_out] ReLU MLP in one launch) against an fp64 evaluation of the same
backward from the same fp32 kept activations: weight / bias gradients summed
over the per-32-row-block partials and dx within 2e-6 max-normalised (fp32
fma chains), run-to-run bitwise, and the tickets left at zero."""
import numpy as np
import pytest
import torch

from d3rlpy_amd import _native as N
from d3rlpy_amd import ops

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("R,C,n_in,n_out,shared_x,wg,with_dx", [
    (256, 2, 23, 200, True, True, False),    # K3 QR critics
    (256, 1, 29, 6, True, True, True),       # K3 VAE decoder (+ dx)
    (256, 1, 23, 1, True, False, True),      # actor's critic pass: dx only
    (100, 2, 17, 12, False, True, True),     # ragged rows, per-member x
    (37, 1, 64, 256, True, True, True),      # widest shapes, one partial block
])
def test_mlp_bwd_small_matches_fp64(R, C, n_in, n_out, shared_x, wg, with_dx):
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(R * 7 + n_in + n_out)
    H = 256
    W1 = torch.randn(C, H, n_in, generator=g) / np.sqrt(n_in)
    W2 = torch.randn(C, H, H, generator=g) / np.sqrt(H)
    W3 = torch.randn(C, n_out, H, generator=g) / np.sqrt(H)
    b1 = torch.randn(C, H, generator=g) * 0.1
    b2 = torch.randn(C, H, generator=g) * 0.1
    ldx = n_in + 3
    xs = torch.randn(1 if shared_x else C, R, ldx, generator=g)
    x = xs.expand(C, R, ldx) if shared_x else xs
    h1 = torch.relu(torch.einsum("crk,chk->crh", x[:, :, :n_in], W1) + b1[:, None])
    h2 = torch.relu(torch.einsum("crk,chk->crh", h1, W2) + b2[:, None])
    ldo = n_out + 1
    dout = torch.randn(C, R, ldo, generator=g)
    # fp64 backward from the same fp32 activations
    d3 = dout[:, :, :n_out].double()
    dz2 = (d3 @ W3.double()) * (h2 > 0)
    dz1 = (dz2 @ W2.double()) * (h1 > 0)
    ref = dict(dW3=d3.transpose(1, 2) @ h2.double(), db3=d3.sum(1),
               dW2=dz2.transpose(1, 2) @ h1.double(), db2=dz2.sum(1),
               dW1=dz1.transpose(1, 2) @ x[:, :, :n_in].double(), db1=dz1.sum(1),
               dx=dz1 @ W1.double())
    nrb = (R + 31) // 32
    t = lambda a: a.contiguous().to(dev)  # noqa: E731
    xd, h1d, h2d, dod = t(xs), t(h1), t(h2), t(dout)
    W1d, W2d, W3d = t(W1), t(W2), t(W3)
    out = dict(dW1=torch.full((nrb, C, H, n_in), float("nan"), device=dev),
               db1=torch.full((nrb, C, H), float("nan"), device=dev),
               dW2=torch.full((nrb, C, H, H), float("nan"), device=dev),
               db2=torch.full((nrb, C, H), float("nan"), device=dev),
               dW3=torch.full((nrb, C, n_out, H), float("nan"), device=dev),
               db3=torch.full((nrb, C, n_out), float("nan"), device=dev),
               dx=torch.full((C, R, n_in), float("nan"), device=dev))
    scratch = torch.zeros(8, C, R, H, device=dev)
    tickets = torch.zeros(C, nrb, dtype=torch.int32, device=dev)
    d = N.MlpBwdSmallDesc()
    d.x, d.ldx, d.sxb = xd.data_ptr(), ldx, 0 if shared_x else R * ldx
    d.h1, d.h2, d.sh = h1d.data_ptr(), h2d.data_ptr(), R * H
    d.dout, d.ld_dout, d.sdout = dod.data_ptr(), ldo, R * ldo
    d.W1, d.W2, d.W3 = W1d.data_ptr(), W2d.data_ptr(), W3d.data_ptr()
    d.sW1, d.sW2, d.sW3 = H * n_in, H * H, n_out * H
    if wg:
        for k in ("dW1", "db1", "dW2", "db2", "dW3", "db3"):
            setattr(d, k, out[k].data_ptr())
    d.dx = out["dx"].data_ptr() if with_dx else None
    d.scratch, d.tickets = scratch.data_ptr(), tickets.data_ptr()
    d.rows, d.n_in, d.n_out, d.C = R, n_in, n_out, C

    def run():
        ops.call_desc("d3a_mlp_bwd_small", d)
        torch.cuda.synchronize()
        return {k: v.clone() for k, v in out.items()}

    got = run()
    assert int(tickets.abs().sum()) == 0
    rel = lambda a, b: float((a.double().cpu() - b).abs().max() / b.abs().max())  # noqa: E731
    errs = {}
    if wg:
        for k in ("dW1", "db1", "dW2", "db2", "dW3", "db3"):
            errs[k] = rel(got[k].sum(0), ref[k])
    if with_dx:
        errs["dx"] = rel(got["dx"], ref["dx"])
    print({k: f"{v:.1e}" for k, v in errs.items()})
    assert all(v < 2e-6 for v in errs.values()), errs
    again = run()
    for k in errs:
        assert torch.equal(again[k], got[k]), k
