"""Generated-A GEMMs (d3a_gemm_desc.agen) against d3a_head1_bwd + the plain
GEMMs (GPU only).

The critic backward of the large passes generates the Q head's masked input
gradient g'[r] * w[j] * [h[r][j] > 0] inside the trunk's weight- and input-
gradient GEMMs instead of writing it with d3a_head1_bwd and reading it back.
The generated operand is the same fp32 product, so both GEMM outputs must be
bit-identical to the two-launch path; the head's weight / bias gradients are
fp64 sums over the same rows in a different split, so their split totals must
agree to fp32 rounding.
"""
import ctypes as C

import pytest
import torch

from d3rlpy_amd import _native as N
from d3rlpy_amd import ops

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rows,n_scaled", [(5000, 1234), (7936, 0)])
def test_head_gradient_generated_in_gemms(rows, n_scaled):
    g = torch.Generator(device="cuda").manual_seed(11)
    Cm, H, Hp, S = 2, 256, 256, 32
    dev = "cuda"
    h2 = torch.relu(torch.randn(Cm, rows, H, device=dev, generator=g))
    h1 = torch.relu(torch.randn(Cm, rows, Hp, device=dev, generator=g))
    gr = torch.randn(Cm, rows, device=dev, generator=g) * 1e-2
    w = torch.randn(Cm, H, device=dev, generator=g) * 0.06
    W2 = torch.randn(Cm, H, Hp, device=dev, generator=g) * 0.06
    gscale = torch.tensor([0.7], device=dev)

    def head_desc(dz=None, dWh=None, dbh=None, splits=S):
        d = N.Head1BwdDesc()
        d.g, d.sgb = gr.data_ptr(), rows
        if n_scaled:
            d.gscale, d.n_scaled = gscale.data_ptr(), n_scaled
        d.h, d.shb, d.ldh = h2.data_ptr(), rows * H, H
        d.w, d.swb = w.data_ptr(), H
        if dz is not None:
            d.dz, d.sdzb, d.lddz = dz.data_ptr(), rows * H, H
        if dWh is not None:
            d.dW, d.sWs = dWh.data_ptr(), Cm * H
            d.db, d.sbs = dbh.data_ptr(), Cm
        d.rows, d.n, d.C, d.splits = rows, H, Cm, splits
        return d

    prev = ops.SBF16_TERMS
    ops.set_sbf16(0)
    try:
        # two-launch reference: d3a_head1_bwd writes dz, the GEMMs read it
        dz = torch.zeros(Cm, rows, H, device=dev)
        dWh_ref = torch.zeros(S, Cm, H, device=dev)
        dbh_ref = torch.zeros(S, Cm, device=dev)
        ops.call_desc("d3a_head1_bwd", head_desc(dz, dWh_ref, dbh_ref))
        dW_ref = torch.zeros(S, Cm, H, Hp, device=dev)
        db_ref = torch.zeros(S, Cm, H, device=dev)
        dx_ref = torch.zeros(Cm, rows, Hp, device=dev)
        ops.linear_bwd_w(dz.data_ptr(), H, rows * H, h1.data_ptr(), Hp, rows * Hp,
                         dW_ref.data_ptr(), Cm, rows, Hp, H, S, db=db_ref.data_ptr())
        ops.linear_bwd_x(dz.data_ptr(), H, rows * H, W2.data_ptr(), dx_ref.data_ptr(), Hp,
                         rows * Hp, Cm, rows, Hp, H, mask=h1.data_ptr(), ldm=Hp, smb=rows * Hp)
        # generated path
        dWh = torch.full((S, Cm, H), float("nan"), device=dev)
        dbh = torch.full((S, Cm), float("nan"), device=dev)
        dW = torch.full((S, Cm, H, Hp), float("nan"), device=dev)
        db = torch.full((S, Cm, H), float("nan"), device=dev)
        dx = torch.full((Cm, rows, Hp), float("nan"), device=dev)
        ag = head_desc(None, dWh, dbh)
        ops.linear_bwd_w(0, H, rows * H, h1.data_ptr(), Hp, rows * Hp, dW.data_ptr(), Cm, rows,
                         Hp, H, S, db=db.data_ptr(), agen=ag)
        ops.linear_bwd_x(0, H, rows * H, W2.data_ptr(), dx.data_ptr(), Hp, rows * Hp, Cm, rows,
                         Hp, H, mask=h1.data_ptr(), ldm=Hp, smb=rows * Hp, agen=head_desc())
        torch.cuda.synchronize()
    finally:
        ops.set_sbf16(prev)
    assert torch.equal(dW, dW_ref)
    assert torch.equal(db, db_ref)
    assert torch.equal(dx, dx_ref)
    # head gradients: fp64 totals over the same rows, split differently
    gs = gr.clone()
    gs[:, :n_scaled] = gr[:, :n_scaled] * gscale  # fp32, as the kernels form g'
    gsf = gs.double()
    ref_w = torch.einsum("cr,crj->cj", gsf, h2.double())
    for tot, ref in ((dWh.double().sum(0), ref_w), (dWh_ref.double().sum(0), ref_w),
                     (dbh.double().sum(0), gsf.sum(1)), (dbh_ref.double().sum(0), gsf.sum(1))):
        e = float((tot - ref).abs().max()) / max(1e-30, float(ref.abs().max()))
        assert e <= 1e-6, e
    assert not torch.isnan(dWh).any() and not torch.isnan(dbh).any()


@pytest.mark.parametrize("generated,n_in,ldx", [(False, 14, 16), (True, 14, 16),
                                                (True, 37, 40), (False, 64, 64)])
def test_first_layer_weight_gradient_epilogue(generated, n_in, ldx):
    """wnext: the layer-0 weight / bias gradient partials formed from the
    layer-1 input-gradient tile (dz1 never written) against dz1 written by the
    plain GEMM and reduced by linear_bwd_w: the 128-row-tile totals agree to
    fp32 rounding (max-normalised 1e-6)."""
    g = torch.Generator(device="cuda").manual_seed(12)
    Cm, rows, H = 2, 7936 - 37, 256
    dev = "cuda"
    x = torch.randn(rows, ldx, device=dev, generator=g)
    x[:, n_in:] = 0
    h1 = torch.relu(torch.randn(Cm, rows, H, device=dev, generator=g))
    h2 = torch.relu(torch.randn(Cm, rows, H, device=dev, generator=g))
    dz2 = torch.randn(Cm, rows, H, device=dev, generator=g) * 1e-3
    W2 = torch.randn(Cm, H, H, device=dev, generator=g) * 0.06
    gr = torch.randn(Cm, rows, device=dev, generator=g) * 1e-2
    w = torch.randn(Cm, H, device=dev, generator=g) * 0.06
    ag = None
    if generated:
        ag = N.Head1BwdDesc()
        ag.g, ag.sgb = gr.data_ptr(), rows
        ag.h, ag.shb, ag.ldh = h2.data_ptr(), rows * H, H
        ag.w, ag.swb = w.data_ptr(), H
        ag.rows, ag.n, ag.C, ag.splits = rows, H, Cm, 1
        dz2 = torch.where(h2 > 0, gr[:, :, None] * w[:, None, :], torch.zeros((), device=dev))
    P = (rows + 127) // 128
    prev = ops.SBF16_TERMS
    ops.set_sbf16(0)
    try:
        dz1 = torch.zeros(Cm, rows, H, device=dev)
        ops.linear_bwd_x(dz2.data_ptr(), H, rows * H, W2.data_ptr(), dz1.data_ptr(), H, rows * H,
                         Cm, rows, H, H, mask=h1.data_ptr(), ldm=H, smb=rows * H)
        dW_ref = torch.zeros(P, Cm, H, n_in, device=dev)
        db_ref = torch.zeros(P, Cm, H, device=dev)
        ops.linear_bwd_w(dz1.data_ptr(), H, rows * H, x.data_ptr(), ldx, 0, dW_ref.data_ptr(), Cm,
                         rows, n_in, H, P, db=db_ref.data_ptr())
        dW = torch.full((P, Cm, H, n_in), float("nan"), device=dev)
        db = torch.full((P, Cm, H), float("nan"), device=dev)
        wn = N.GemmWnext()
        wn.x, wn.ldx, wn.sxb, wn.n_in = x.data_ptr(), ldx, 0, n_in
        wn.dW, wn.db = dW.data_ptr(), db.data_ptr()
        ops.linear_bwd_x(0 if generated else dz2.data_ptr(), H, rows * H, W2.data_ptr(), 0, H,
                         rows * H, Cm, rows, H, H, mask=h1.data_ptr(), ldm=H, smb=rows * H,
                         agen=ag, wnext=wn)
        torch.cuda.synchronize()
    finally:
        ops.set_sbf16(prev)
    assert not torch.isnan(dW).any() and not torch.isnan(db).any()
    ref_w = torch.einsum("crj,rd->cjd", dz1.double(), x[:, :n_in].double())
    ref_b = dz1.double().sum(1)
    for tot, ref in ((dW.double().sum(0), ref_w), (dW_ref.double().sum(0), ref_w),
                     (db.double().sum(0), ref_b), (db_ref.double().sum(0), ref_b)):
        e = float((tot - ref).abs().max()) / float(ref.abs().max())
        assert e <= 1e-6, e
    # per tile: the same 128 rows
    tile_w = torch.stack([torch.einsum("crj,rd->cjd", dz1[:, t * 128:(t + 1) * 128].double(),
                                       x[t * 128:(t + 1) * 128, :n_in].double())
                          for t in range(P)])
    e = float((dW.double() - tile_w).abs().max()) / float(tile_w.abs().max())
    assert e <= 1e-6, e


@pytest.mark.parametrize("C", [2, 5])
def test_head1_min_matches_rowdot_and_argmin_backward(C):
    """d3a_head1_min (the actor phase's Q head + min-over-critics backward in
    one launch) is bit-identical to d3a_rowdot_f32 followed by d3a_head1_bwd
    in argmin mode, ties included."""
    g = torch.Generator(device="cuda").manual_seed(13)
    rows, H = 300, 256
    h = torch.relu(torch.randn(C, rows, H, device="cuda", generator=g))
    w = torch.randn(C, H, device="cuda", generator=g) * 0.06
    b = torch.randn(C, device="cuda", generator=g)
    # ties: member 1 a copy of member 0 on some rows
    h[1, :50] = h[0, :50]
    w[1] = w[0]
    b[1] = b[0]
    q_ref = torch.zeros(C, rows, device="cuda")
    ops.rowdot(h.data_ptr(), rows * H, H, w.data_ptr(), H, b.data_ptr(), 1, q_ref.data_ptr(),
               rows, C, rows, H)
    dz_ref = torch.zeros(C, rows, H, device="cuda")
    gout_ref = torch.zeros(C, rows, device="cuda")
    d = N.Head1BwdDesc()
    d.q_min, d.sqb, d.scale = q_ref.data_ptr(), rows, -1.0 / 256
    d.g_out, d.sgb = gout_ref.data_ptr(), rows
    d.h, d.shb, d.ldh = h.data_ptr(), rows * H, H
    d.w, d.swb = w.data_ptr(), H
    d.dz, d.sdzb, d.lddz = dz_ref.data_ptr(), rows * H, H
    d.rows, d.n, d.C, d.splits = rows, H, C, max(1, rows // 64)
    ops.call_desc("d3a_head1_bwd", d)
    q = torch.full((C, rows), float("nan"), device="cuda")
    dz = torch.full((C, rows, H), float("nan"), device="cuda")
    gout = torch.full((C, rows), float("nan"), device="cuda")
    m = N.Head1MinDesc()
    m.h, m.shb, m.ldh = h.data_ptr(), rows * H, H
    m.w, m.swb = w.data_ptr(), H
    m.b, m.sbb = b.data_ptr(), 1
    m.q, m.sqb = q.data_ptr(), rows
    m.scale = -1.0 / 256
    m.g_out, m.sgb = gout.data_ptr(), rows
    m.dz, m.sdzb, m.lddz = dz.data_ptr(), rows * H, H
    m.rows, m.n, m.C = rows, H, C
    ops.call_desc("d3a_head1_min", m)
    torch.cuda.synchronize()
    assert torch.equal(q, q_ref)
    assert torch.equal(gout, gout_ref)
    assert torch.equal(dz, dz_ref)
    assert torch.equal(torch.signbit(dz), torch.signbit(dz_ref))
