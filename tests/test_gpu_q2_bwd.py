"""d3a_q2_bwd — the one-launch critic weight-gradient backward (GPU only).

Reference semantics: the autograd backward of VectorEncoderWithAction
[n_in -> 256 -> 256] + ContinuousMeanQFunction._fc (d3rlpy/models/torch/
encoders.py:265-275, 328-339, q_functions/mean_q_function.py:255-256) for
the weight gradients, given dL/dQ per row.  Checked against an fp64 torch
evaluation of the same formulas, per 256-row partial (so the partial layout
the optimiser sums is pinned too), within 1e-5 of each partial's largest
entry (fp32 MFMA accumulation over <= 256 rows); run-to-run bit-identical.
"""
import ctypes as C

import pytest
import torch

from d3rlpy_amd import _native as N
from d3rlpy_amd import ops

pytestmark = pytest.mark.gpu

H = 256


def _run(x, h1, h2, gr, gscale, n_scaled, W2, w3, n_in, rows, Cm):
    P = (rows + 255) // 256
    dev = x.device
    out = {
        "dW1": torch.full((P, Cm, H, n_in), float("nan"), device=dev),
        "db1": torch.full((P, Cm, H), float("nan"), device=dev),
        "dW2": torch.full((P, Cm, H, H), float("nan"), device=dev),
        "db2": torch.full((P, Cm, H), float("nan"), device=dev),
        "dW3": torch.full((P, Cm, H), float("nan"), device=dev),
        "db3": torch.full((P, Cm), float("nan"), device=dev),
    }
    d = N.Q2BwdDesc()
    d.x, d.ldx, d.sxb = x.data_ptr(), x.shape[1], 0
    d.h1, d.h2, d.sh, d.ldh = h1.data_ptr(), h2.data_ptr(), rows * H, H
    d.g, d.sgb = gr.data_ptr(), rows
    if n_scaled:
        d.gscale, d.n_scaled = gscale.data_ptr(), n_scaled
    d.W2, d.sW2 = W2.data_ptr(), H * H
    d.w3, d.sw3 = w3.data_ptr(), H
    for k, v in out.items():
        setattr(d, k, v.data_ptr())
    d.rows, d.n_in, d.C = rows, n_in, Cm
    ops.call_desc("d3a_q2_bwd", d)
    torch.cuda.synchronize()
    return out


def _reference(x, h1, h2, gr, gscale, n_scaled, W2, w3, n_in, rows, Cm):
    """fp64 per-256-row-block partials of the same formulas."""
    P = (rows + 255) // 256
    xd = x[:, :n_in].double()
    ref = {k: [] for k in ("dW1", "db1", "dW2", "db2", "dW3", "db3")}
    gp = gr.double().clone()
    if n_scaled:
        gp[:, :n_scaled] *= float(gscale.item())
    for p in range(P):
        sl = slice(256 * p, min(rows, 256 * p + 256))
        per = {k: [] for k in ref}
        for c in range(Cm):
            g_ = gp[c, sl]
            a2, a1 = h2[c, sl].double(), h1[c, sl].double()
            dz2 = g_[:, None] * w3[c].double()[None, :] * (a2 > 0)
            dz1 = (dz2 @ W2[c].double()) * (a1 > 0)
            per["dW1"].append(dz1.T @ xd[sl])
            per["db1"].append(dz1.sum(0))
            per["dW2"].append(dz2.T @ a1)
            per["db2"].append(dz2.sum(0))
            per["dW3"].append(g_ @ a2)
            per["db3"].append(g_.sum())
        for k in ref:
            ref[k].append(torch.stack(per[k]))
    return {k: torch.stack(v) for k, v in ref.items()}


@pytest.mark.parametrize("rows,n_in,ldx,n_scaled", [
    (7936, 14, 16, 7680),   # K2 CQL critic pass: 3NB importance rows scaled
    (7936, 37, 40, 7680),   # K4 antmaze critic pass
    (300, 14, 16, 100),     # ragged last row block
    (256, 23, 24, 0),       # one block, no scaled rows
    (1000, 48, 48, 999),
])
def test_q2_bwd_partials_match_fp64(rows, n_in, ldx, n_scaled):
    gen = torch.Generator(device="cuda").manual_seed(rows + n_in)
    Cm, dev = 2, "cuda"
    # garbage in x's pad columns must not leak into the real ones
    x = torch.randn(rows, ldx, device=dev, generator=gen)
    h1 = torch.relu(torch.randn(Cm, rows, H, device=dev, generator=gen))
    h2 = torch.relu(torch.randn(Cm, rows, H, device=dev, generator=gen))
    gr = torch.randn(Cm, rows, device=dev, generator=gen) * 1e-2
    gscale = torch.tensor([0.7], device=dev)
    W2 = torch.randn(Cm, H, H, device=dev, generator=gen) * 0.06
    w3 = torch.randn(Cm, H, device=dev, generator=gen) * 0.06
    args = (x, h1, h2, gr, gscale, n_scaled, W2, w3, n_in, rows, Cm)
    out = _run(*args)
    ref = _reference(*args)
    for k in ref:
        got, exp = out[k].double(), ref[k].to(dev)
        assert torch.isfinite(got).all(), k  # every partial entry written
        P = got.shape[0]
        for p in range(P):
            scale = exp[p].abs().max().clamp_min(1e-30)
            err = ((got[p] - exp[p]).abs().max() / scale).item()
            assert err < 1e-5, (k, p, err)
    again = _run(*args)
    for k in out:
        assert torch.equal(out[k], again[k]), k  # run-to-run bit-identical


def test_q2_bwd_rejects_bad_shapes():
    d = N.Q2BwdDesc()
    rc = N.lib().d3a_q2_bwd(C.byref(d), None)
    assert rc < 0 and b"null input" in N.lib().d3a_last_error()


def _run_dz(x, ldx, h1, dz2, W2, n_in, rows, Cm):
    P = (rows + 31) // 32
    dev = x.device
    out = {
        "dW1": torch.full((P, Cm, H, n_in), float("nan"), device=dev),
        "db1": torch.full((P, Cm, H), float("nan"), device=dev),
        "dW2": torch.full((P, Cm, H, H), float("nan"), device=dev),
        "db2": torch.full((P, Cm, H), float("nan"), device=dev),
    }
    d = N.Q2BwdDesc()
    d.x, d.ldx, d.sxb = x.data_ptr(), ldx, 0
    d.h1, d.sh, d.ldh = h1.data_ptr(), rows * H, H
    d.dz2, d.sdz, d.block_rows = dz2.data_ptr(), rows * H, 32
    d.W2, d.sW2 = W2.data_ptr(), H * H
    for k, v in out.items():
        setattr(d, k, v.data_ptr())
    d.rows, d.n_in, d.C = rows, n_in, Cm
    ops.call_desc("d3a_q2_bwd", d)
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("rows,n_in,ldx,Cm", [
    (256, 11, 11, 1),   # K2 policy trunk: [obs; next_obs] rows unpadded (ldx = n_in)
    (256, 29, 29, 1),   # K4 antmaze policy
    (100, 3, 3, 1),     # ragged last 32-row block
    (300, 16, 16, 2),   # aligned rows, two members
    (64, 48, 52, 1),
])
def test_q2_bwd_dz2_trunk_matches_fp64(rows, n_in, ldx, Cm):
    """dz2 given (d3a_sac_actor_head's masked head input gradient): the trunk
    of the policy backward (encoders.py:265-275 under sac_impl.py:164-176), as
    one partial per 32-row block, against fp64."""
    gen = torch.Generator(device="cuda").manual_seed(rows * 7 + n_in)
    dev = "cuda"
    # x as a flat buffer of rows ldx apart, with one row of slack
    xb = torch.randn((rows + 1) * ldx, device=dev, generator=gen)
    x = xb[: rows * ldx].view(rows, ldx)
    h1 = torch.relu(torch.randn(Cm, rows, H, device=dev, generator=gen))
    h2 = torch.randn(Cm, rows, H, device=dev, generator=gen)
    dz2 = torch.randn(Cm, rows, H, device=dev, generator=gen) * 1e-2 * (h2 > 0)
    W2 = torch.randn(Cm, H, H, device=dev, generator=gen) * 0.06
    out = _run_dz(x, ldx, h1, dz2, W2, n_in, rows, Cm)
    xd = x[:, :n_in].double()
    for p in range((rows + 31) // 32):
        sl = slice(32 * p, min(rows, 32 * p + 32))
        for c in range(Cm):
            a1, dz = h1[c, sl].double(), dz2[c, sl].double()
            dz1 = (dz @ W2[c].double()) * (a1 > 0)
            exp = {"dW1": dz1.T @ xd[sl], "db1": dz1.sum(0), "dW2": dz.T @ a1, "db2": dz.sum(0)}
            for k, e in exp.items():
                got = out[k][p, c].double()
                assert torch.isfinite(got).all(), (k, p, c)
                err = ((got - e).abs().max() / e.abs().max().clamp_min(1e-30)).item()
                assert err < 1e-5, (k, p, c, err)
    again = _run_dz(x, ldx, h1, dz2, W2, n_in, rows, Cm)
    for k in out:
        assert torch.equal(out[k], again[k]), k
