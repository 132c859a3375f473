"""fp32-accurate critic kernels on the bf16 matrix cores (csrc/q2_x6.hip:
d3a_q2_fwd_x6 / d3a_q2_bwd_x6, three-way split-bf16 operands, six part
products, fp32 accumulation) against fp64 -- at the fp32 kernels' own bars.

The split is exact (x = x0 + x1 + x2) and the three dropped part products are
each below 2^-24 |x y|, so a product carries fp32-level error: bars are
relative to the rounding scale sum_k |a_k b_k| (what an fp32 dot product is
accurate to), 2e-6 -- the fp32 MFMA kernels measure ~1e-7 .. 5e-7 there, and
a single bf16-rounded operand would show at ~4e-3.
"""
import numpy as np
import pytest
import torch

from d3rlpy_amd import _native as N
from d3rlpy_amd import ops

pytestmark = pytest.mark.gpu

SCALE_BAR = 2e-6


def _net(C, n_in, gen, dev):
    sizes = [n_in, 256, 256, 1]
    Ws = [torch.randn(C, sizes[l + 1], sizes[l], generator=gen) * (1.0 / np.sqrt(sizes[l]))
          for l in range(3)]
    bs = [torch.randn(C, sizes[l + 1], generator=gen) * 0.1 for l in range(3)]
    return [w.to(dev) for w in Ws], [b.to(dev) for b in bs]


def _fwd64(x, Ws, bs):
    """fp64 forward; per layer the value and its rounding scale sum |w x| + |b|."""
    a, sa = x.double(), x.double().abs()
    hs, scales = [], []
    for l in range(3):
        W, b = Ws[l].double(), bs[l].double().unsqueeze(1)
        z = a @ W.transpose(-1, -2) + b
        sz = a.abs() @ W.abs().transpose(-1, -2) + b.abs()
        if l < 2:
            z = z.clamp_min(0)
        hs.append(z)
        scales.append(sz)
        a = z
    return hs, scales


def _fwd_desc(x, ldx, n_in, Ws, bs, Wt, bt, h, out, aout, xa, rows, h_from, aux, C, dev):
    flat = [torch.cat([W[l].reshape(-1) for l in range(3)] + [b[l].reshape(-1) for l in range(3)])
            for W, b in ((Ws, bs), (Wt, bt))]
    pad = (-flat[0].numel()) % 4
    buf = torch.cat([flat[0], torch.zeros(pad, device=dev), flat[1]])
    n1 = flat[0].numel() + pad
    offs, o = [], 0
    for l in range(3):
        offs.append(o)
        o += Ws[l].numel()
    boffs = []
    for l in range(3):
        boffs.append(o)
        o += bs[l].numel()
    d = N.MlpFwdDesc()
    d.x, d.ldx, d.sxb = x.data_ptr(), ldx, 0
    d.n_in, d.n_hidden, d.H, d.n_out = n_in, 2, 256, 1
    for l in range(3):
        d.W[l] = buf.data_ptr() + 4 * offs[l]
        d.b[l] = buf.data_ptr() + 4 * boffs[l]
        d.sW[l], d.sb[l] = Ws[l].shape[1] * Ws[l].shape[2], bs[l].shape[1]
    for l in range(2):
        d.h[l] = h[l].data_ptr()
    d.sh = rows * 256
    d.out, d.sout, d.ldout = out.data_ptr(), rows, 1
    d.r0, d.rows, d.C, d.h_from = 0, rows, C, h_from
    if aux:
        d.aux_x, d.aux_ldx, d.aux_sxb, d.aux_wdelta = xa.data_ptr(), ldx, 0, n1
        d.aux_out, d.aux_sout, d.aux_rows = aout.data_ptr(), aux, aux
    return d, buf


@pytest.mark.parametrize("rows,h_from,aux,n_in", [(15616, 7680, 256, 14), (1000, 0, 0, 48),
                                                   (300, 100, 77, 23), (129, 0, 5, 37)])
def test_q2_fwd_x6_vs_fp64(rows, h_from, aux, n_in):
    dev = torch.device("cuda")
    C = 2
    gen = torch.Generator().manual_seed(rows + n_in)
    Ws, bs = _net(C, n_in, gen, dev)
    Wt, bt = _net(C, n_in, gen, dev)
    ldx = (n_in + 3) // 4 * 4
    x = torch.randn(rows, ldx, generator=gen).to(dev)
    xa = torch.randn(max(aux, 1), ldx, generator=gen).to(dev)
    h = [torch.full((C, rows, 256), float("nan"), device=dev) for _ in range(2)]
    out = torch.full((C, rows), float("nan"), device=dev)
    aout = torch.full((C, max(aux, 1)), float("nan"), device=dev)
    d, _buf = _fwd_desc(x, ldx, n_in, Ws, bs, Wt, bt, h, out, aout, xa, rows, h_from, aux, C, dev)
    ops.call_desc("d3a_q2_fwd_x6", d)
    torch.cuda.synchronize()
    hs, sc = _fwd64(x[:, :n_in], Ws, bs)
    # each layer against fp64 evaluated on the kernel's own (fp32) input
    # activations: relative to that layer's rounding scale
    h0, h1 = h[0][:, h_from:].double(), h[1][:, h_from:].double()
    e0 = float(((h0 - hs[0][:, h_from:]).abs() / sc[0][:, h_from:]).max())
    z1 = (h0 @ Ws[1].double().transpose(1, 2) + bs[1].double().unsqueeze(1)).clamp_min(0)
    s1 = h0.abs() @ Ws[1].double().abs().transpose(1, 2) + bs[1].double().abs().unsqueeze(1)
    e1 = float(((h1 - z1).abs() / s1).max())
    q = (h1 @ Ws[2].double().transpose(1, 2) + bs[2].double().unsqueeze(1)).squeeze(-1)
    sq = (h1.abs() @ Ws[2].double().abs().transpose(1, 2)).squeeze(-1) + bs[2].double().abs()
    eq = float(((out[:, h_from:].double() - q).abs() / sq).max())
    print(f"x6 forward vs fp64 (per rounding scale): h0 {e0:.1e} h1 {e1:.1e} q {eq:.1e}")
    assert e0 < SCALE_BAR and e1 < SCALE_BAR and eq < SCALE_BAR, (e0, e1, eq)
    # every row's Q (kept or not) against end-to-end fp64
    qf = hs[2].squeeze(-1)
    rel = float((out.double() - qf).abs().max() / qf.abs().max())
    assert rel < 1e-5, rel
    assert torch.isnan(h[0][:, :h_from]).all() and torch.isnan(h[1][:, :h_from]).all()
    if aux:
        ha, _ = _fwd64(xa[:aux, :n_in], Wt, bt)
        qa = ha[2].squeeze(-1)
        assert float((aout[:, :aux].double() - qa).abs().max() / qa.abs().max()) < 1e-5
    # deterministic
    o1 = out.clone()
    ops.call_desc("d3a_q2_fwd_x6", d)
    torch.cuda.synchronize()
    assert torch.equal(o1, out)


def test_q2_fwd_x6_matches_fp32_kernel():
    """The x6 forward and the exact-fp32 MFMA forward (q2_fwd) agree to fp32
    rounding on the K2 critic pass."""
    dev = torch.device("cuda")
    C, rows, n_in, h_from, aux = 2, 15616, 14, 7680, 256
    gen = torch.Generator().manual_seed(7)
    Ws, bs = _net(C, n_in, gen, dev)
    Wt, bt = _net(C, n_in, gen, dev)
    x = torch.randn(rows, 16, generator=gen).to(dev)
    xa = torch.randn(aux, 16, generator=gen).to(dev)
    res = []
    for entry in ("d3a_q2_fwd_x6", "d3a_mlp_fwd"):
        h = [torch.zeros(C, rows, 256, device=dev) for _ in range(2)]
        out, aout = torch.zeros(C, rows, device=dev), torch.zeros(C, aux, device=dev)
        d, _b = _fwd_desc(x, 16, n_in, Ws, bs, Wt, bt, h, out, aout, xa, rows, h_from, aux, C, dev)
        ops.call_desc(entry, d)
        torch.cuda.synchronize()
        res.append((out, aout, h))
    for a, b in ((res[0][0], res[1][0]), (res[0][1], res[1][1]), (res[0][2][1], res[1][2][1])):
        assert float((a - b).abs().max() / b.abs().max()) < 2e-6


def _bwd_case(rows, n_in, n_scaled, C, gen, dev):
    Ws, bs = _net(C, n_in, gen, dev)
    ldx = (n_in + 3) // 4 * 4
    x = torch.randn(rows, ldx, generator=gen).to(dev)
    hs, _ = _fwd64(x[:, :n_in], Ws, bs)
    h1 = hs[0].float().contiguous()
    h2 = hs[1].float().contiguous()
    g = (torch.randn(C, rows, generator=gen) * 1e-2).to(dev)
    gscale = torch.tensor([0.7], device=dev)
    P = (rows + 255) // 256
    W2 = Ws[1].contiguous()
    w3 = Ws[2].reshape(C, 256).contiguous()

    # the forward's mask bits of h2 (d3a_mlp_fwd_desc.hmask: bit o & 31 of
    # word o >> 5)
    bits = (h2 > 0).view(C, rows, 8, 32).to(torch.int64)
    m2 = (bits << torch.arange(32, device=dev)).sum(-1)
    m2 = torch.where(m2 >= 2 ** 31, m2 - 2 ** 32, m2).to(torch.int32).contiguous()

    def run(entry, mask_image=False):
        outs = [torch.full((P, C, 256, n_in), float("nan"), device=dev),
                torch.full((P, C, 256), float("nan"), device=dev),
                torch.full((P, C, 256, 256), float("nan"), device=dev),
                torch.full((P, C, 256), float("nan"), device=dev),
                torch.full((P, C, 256), float("nan"), device=dev),
                torch.full((P, C), float("nan"), device=dev)]
        d = N.Q2BwdDesc()
        d.x, d.ldx, d.sxb = x.data_ptr(), ldx, 0
        d.h1, d.h2, d.sh, d.ldh = h1.data_ptr(), h2.data_ptr(), rows * 256, 256
        d.g, d.sgb, d.gscale, d.n_scaled = g.data_ptr(), rows, gscale.data_ptr(), n_scaled
        d.W2, d.sW2, d.w3, d.sw3 = W2.data_ptr(), 256 * 256, w3.data_ptr(), 256
        d.dW1, d.db1, d.dW2, d.db2, d.dW3, d.db3 = [t.data_ptr() for t in outs]
        d.rows, d.n_in, d.C = rows, n_in, C
        if mask_image:
            d.m2, d.sm2 = m2.data_ptr(), rows * 8
        ops.call_desc(entry, d)
        torch.cuda.synchronize()
        return outs, d
    # fp64 reference on the kernel's fp32 inputs, and each product's rounding scale
    gp = g.double().clone()
    gp[:, :n_scaled] *= 0.7
    a1, a2 = h1.double(), h2.double()
    dz2 = gp.unsqueeze(-1) * w3.double().unsqueeze(1) * (a2 > 0)
    dh1 = dz2 @ W2.double()
    sdh1 = dz2.abs() @ W2.double().abs()
    dz1 = dh1 * (a1 > 0)
    xd = x[:, :n_in].double()
    ref = {"dW1": (dz1.transpose(1, 2) @ xd, (sdh1 * (a1 > 0)).transpose(1, 2) @ xd.abs()),
           "db1": (dz1.sum(1), (sdh1 * (a1 > 0)).sum(1)),
           "dW2": (dz2.transpose(1, 2) @ a1, dz2.abs().transpose(1, 2) @ a1),
           "db2": (dz2.sum(1), dz2.abs().sum(1)),
           "dW3": ((gp.unsqueeze(-1) * a2).sum(1), (gp.abs().unsqueeze(-1) * a2).sum(1)),
           "db3": (gp.sum(1), gp.abs().sum(1))}
    return run, ref


NAMES = ["dW1", "db1", "dW2", "db2", "dW3", "db3"]


@pytest.mark.parametrize("mask_image", [False, True])
@pytest.mark.parametrize("rows,n_in,n_scaled", [(7936, 14, 7680), (1000, 48, 999), (300, 23, 0),
                                                (257, 37, 100)])
def test_q2_bwd_x6_vs_fp64(rows, n_in, n_scaled, mask_image):
    """mask_image: the ReLU-mask operand copied from the forward's bf16 mask
    image (d3a_q2_bwd_desc.m2; swizzled LDS rows, transposed reads) rather
    than built from h2."""
    dev = torch.device("cuda")
    C = 2
    gen = torch.Generator().manual_seed(rows * 3 + n_in)
    run, ref = _bwd_case(rows, n_in, n_scaled, C, gen, dev)
    outs, d = run("d3a_q2_bwd_x6", mask_image)
    worst = {}
    for name, o in zip(NAMES, outs):
        assert not torch.isnan(o).any(), name
        got = o.double().sum(0).cpu()
        r, sc = (v.cpu() for v in ref[name])
        e_sc = float(((got - r).abs() / sc.clamp_min(1e-30)).max())
        e_max = float((got - r).abs().max() / r.abs().max())
        worst[name] = (e_sc, e_max)
        assert e_sc < SCALE_BAR and e_max < 1e-6, (name, e_sc, e_max)
    print("x6 backward vs fp64 (rounding scale, max-normalised): " +
          " ".join(f"{k} {a:.1e}/{b:.1e}" for k, (a, b) in worst.items()))
    # run-to-run bit-identical (fixed reduction orders)
    first = [o.clone() for o in outs]
    ops.call_desc("d3a_q2_bwd_x6", d)
    torch.cuda.synchronize()
    for a, b in zip(first, outs):
        assert torch.equal(a, b)


def test_q2_bwd_x6_mask_image_matches_built_mask():
    """The mask-image path gives the built-mask path's dW1 / db1 / dW2 bitwise
    (same operands, same MFMA order) and its db2 / dW3 / db3 to fp32
    summation order (rows grouped differently per thread)."""
    dev = torch.device("cuda")
    gen = torch.Generator().manual_seed(5)
    run, _ = _bwd_case(7936, 14, 7680, 2, gen, dev)
    a, _ = run("d3a_q2_bwd_x6", False)
    b, _ = run("d3a_q2_bwd_x6", True)
    for name, x, y in zip(NAMES, a, b):
        if name in ("dW1", "db1", "dW2"):
            assert torch.equal(x, y), name
        else:
            xs, ys = x.double().sum(0), y.double().sum(0)
            assert float((xs - ys).abs().max() / ys.abs().max()) < 1e-6, name


def test_q2_bwd_x6_matches_fp32_kernel():
    dev = torch.device("cuda")
    gen = torch.Generator().manual_seed(11)
    run, _ = _bwd_case(7936, 14, 7680, 2, gen, dev)
    a, _ = run("d3a_q2_bwd_x6")
    b, _ = run("d3a_q2_bwd")
    for name, x, y in zip(NAMES, a, b):
        xs, ys = x.double().sum(0), y.double().sum(0)
        assert float((xs - ys).abs().max() / ys.abs().max()) < 2e-6, name


def test_q2_x6_rejects_bad_shapes():
    d = N.Q2BwdDesc()
    with pytest.raises(RuntimeError, match="null"):
        ops.call_desc("d3a_q2_bwd_x6", d)
    f = N.MlpFwdDesc()
    f.n_in, f.n_hidden, f.H, f.n_out = 64, 2, 256, 1
    with pytest.raises(RuntimeError, match="n_in <= 48"):
        ops.call_desc("d3a_q2_fwd_x6", f)


@pytest.mark.parametrize("entry,rows,n_in,n_out,keep", [
    ("d3a_mlp_fwd_x6", 25600, 23, 200, False), ("d3a_mlp_fwd_x6", 1000, 23, 6, True),
    ("d3a_mlp_fwd_x6", 257, 64, 256, True), ("d3a_mlp_fwd_x6", 77, 33, 1 + 32, False),
    # the narrow-head instantiation of the Q-head kernel (K3's VAE decoder over
    # B*N target rows: obs 17 + latent 12 -> 256 -> 256 -> act 6; the residual
    # policy 23 -> .. -> 6; ragged rows, 8 outputs, 48 inputs)
    ("d3a_q2_fwd_x6", 25600, 29, 6, False), ("d3a_q2_fwd_x6", 1000, 23, 6, True),
    ("d3a_q2_fwd_x6", 333, 48, 8, True), ("d3a_q2_fwd_x6", 200, 5, 2, False)])
def test_mlp_fwd_x6_wide_head_vs_fp64(entry, rows, n_in, n_out, keep):
    """d3a_mlp_fwd_x6 ([n_in <= 64, 256, 256, n_out <= 256]; the K3 target QR
    critics are the first case) and d3a_q2_fwd_x6's narrow head ([n_in <= 48,
    256, 256, n_out <= 8]) against fp64, per layer relative to the layer's
    rounding scale, on the kernel's own fp32 inputs to each layer."""
    dev = torch.device("cuda")
    C = 2
    gen = torch.Generator().manual_seed(rows + n_out)
    sizes = [n_in, 256, 256, n_out]
    Ws = [(torch.randn(C, sizes[l + 1], sizes[l], generator=gen) / np.sqrt(sizes[l])).to(dev)
          for l in range(3)]
    bs = [(torch.randn(C, sizes[l + 1], generator=gen) * 0.1).to(dev) for l in range(3)]
    ldx = (n_in + 3) // 4 * 4
    x = torch.randn(rows, ldx, generator=gen).to(dev)
    flat = torch.cat([W.reshape(-1) for W in Ws] + [b.reshape(-1) for b in bs])
    offs, o = [], 0
    for W in Ws:
        offs.append(o)
        o += W.numel()
    boffs = []
    for b in bs:
        o = (o + 3) // 4 * 4
        boffs.append(o)
        o += b.numel()
    buf = torch.zeros(o + 4, device=dev)
    for W, of in zip(Ws, offs):
        buf[of:of + W.numel()] = W.reshape(-1)
    for b, of in zip(bs, boffs):
        buf[of:of + b.numel()] = b.reshape(-1)
    h = [torch.full((C, rows, 256), float("nan"), device=dev) for _ in range(2)]
    out = torch.full((C, rows, n_out), float("nan"), device=dev)
    d = N.MlpFwdDesc()
    d.x, d.ldx, d.sxb = x.data_ptr(), ldx, 0
    d.n_in, d.n_hidden, d.H, d.n_out = n_in, 2, 256, n_out
    for l in range(3):
        d.W[l], d.b[l] = buf.data_ptr() + 4 * offs[l], buf.data_ptr() + 4 * boffs[l]
        d.sW[l], d.sb[l] = sizes[l + 1] * sizes[l], sizes[l + 1]
    for l in range(2):
        d.h[l] = h[l].data_ptr() if keep else None
    d.sh = rows * 256
    d.out, d.sout, d.ldout = out.data_ptr(), rows * n_out, n_out
    d.r0, d.rows, d.C, d.h_from = 0, rows, C, 0
    # row_mean (the per-row output mean of compute_max_with_n_actions,
    # q_functions/__init__.py:37-39) on the keep=False cases
    means = torch.full((C, rows), float("nan"), device=dev)
    wide = entry == "d3a_mlp_fwd_x6"
    if not keep and wide:
        d.row_mean, d.s_mean = means.data_ptr(), rows
    ops.call_desc(entry, d)
    torch.cuda.synchronize()
    assert not torch.isnan(out).any()
    if not keep and wide:
        # the mean of the kernel's own outputs: fp32 summation of n_out terms
        m64 = out.double().mean(-1)
        sm = out.double().abs().mean(-1)
        em = float(((means.double() - m64).abs() / sm.clamp_min(1e-30)).max())
        print(f"x6 wide forward row_mean vs fp64 mean of its outputs: {em:.1e}")
        assert em < 1e-6 * n_out, em
        # run to run bit-identical (fixed summation order)
        m1 = means.clone()
        ops.call_desc(entry, d)
        torch.cuda.synchronize()
        assert torch.equal(m1, means)
    else:
        assert torch.isnan(means).all()
    hs, sc = _fwd64(x[:, :n_in], Ws, bs)
    if keep:
        h0, h1 = h[0].double(), h[1].double()
        e0 = float(((h0 - hs[0]).abs() / sc[0]).max())
        z1 = (h0 @ Ws[1].double().transpose(1, 2) + bs[1].double().unsqueeze(1)).clamp_min(0)
        s1 = h0.abs() @ Ws[1].double().abs().transpose(1, 2) + bs[1].double().abs().unsqueeze(1)
        e1 = float(((h1 - z1).abs() / s1).max())
        zq = h1 @ Ws[2].double().transpose(1, 2) + bs[2].double().unsqueeze(1)
        sq = h1.abs() @ Ws[2].double().abs().transpose(1, 2) + bs[2].double().abs().unsqueeze(1)
        eq = float(((out.double() - zq).abs() / sq).max())
        print(f"x6 wide forward vs fp64 (rounding scale): h0 {e0:.1e} h1 {e1:.1e} out {eq:.1e}")
        assert e0 < SCALE_BAR and e1 < SCALE_BAR and eq < SCALE_BAR, (e0, e1, eq)
    rel = float((out.double() - hs[2]).abs().max() / hs[2].abs().max())
    print(f"x6 wide forward vs fp64 end to end: {rel:.1e}")
    assert rel < 1e-5, rel


@pytest.mark.parametrize("rows,r0,h_from,C", [(300, 40, 100, 2), (1000, 33, 33, 1), (70, 7, 50, 2)])
def test_mlp_fwd_x6_row_window_bitwise(rows, r0, h_from, C):
    """d3a_mlp_fwd_x6 over a row window [r0, rows) (its persistent workgroups cut
    the window into 32-row halves from r0) gives bitwise the rows of the
    whole-range launch, writes kept activations only from h_from on, and
    touches no row outside the window."""
    dev = torch.device("cuda")
    n_in, n_out, H = 23, 200, 256
    gen = torch.Generator().manual_seed(rows + r0)
    sizes = [n_in, H, H, n_out]
    Ws = [(torch.randn(C, sizes[l + 1], sizes[l], generator=gen) / np.sqrt(sizes[l])).to(dev) for l in range(3)]
    bs = [(torch.randn(C, sizes[l + 1], generator=gen) * 0.1).to(dev) for l in range(3)]
    ldx = 24
    x = torch.randn(rows, ldx, generator=gen).to(dev)

    def run(rr0, hf, keep):
        out = torch.full((C, rows, n_out), float("nan"), device=dev)
        means = torch.full((C, rows), float("nan"), device=dev)
        h = [torch.full((C, rows, H), float("nan"), device=dev) for _ in range(2)]
        d = N.MlpFwdDesc()
        d.x, d.ldx, d.sxb = x.data_ptr(), ldx, 0
        d.n_in, d.n_hidden, d.H, d.n_out = n_in, 2, H, n_out
        for l in range(3):
            d.W[l], d.b[l] = Ws[l].data_ptr(), bs[l].data_ptr()
            d.sW[l], d.sb[l] = sizes[l + 1] * sizes[l], sizes[l + 1]
        for l in range(2):
            d.h[l] = h[l].data_ptr() if keep else None
        d.sh = rows * H
        d.out, d.sout, d.ldout = out.data_ptr(), rows * n_out, n_out
        d.r0, d.rows, d.C, d.h_from = rr0, rows - rr0, C, hf
        if not keep:
            d.row_mean, d.s_mean = means.data_ptr(), rows
        ops.call_desc("d3a_mlp_fwd_x6", d)
        torch.cuda.synchronize()
        return out, means, h

    full, fmeans, _ = run(0, 0, False)
    win, wmeans, _ = run(r0, r0, False)
    assert torch.isnan(win[:, :r0]).all() and torch.isnan(wmeans[:, :r0]).all()
    assert torch.equal(win[:, r0:], full[:, r0:]) and torch.equal(wmeans[:, r0:], fmeans[:, r0:])
    kept, _, h = run(r0, h_from, True)
    assert torch.equal(kept[:, r0:], full[:, r0:])
    for t in h:
        assert torch.isnan(t[:, :h_from]).all() and not torch.isnan(t[:, h_from:]).any()


@pytest.mark.parametrize("entry,mode,n_out", [("d3a_q2_fwd_x6", 1, 6), ("d3a_q2_fwd_x6", 2, 6),
                                              ("d3a_mlp_fwd_x6", 4, 200), ("d3a_q2_fwd_x6", 3, 1)])
def test_x6_input_row_builder_matches_bcq_rows(entry, mode, n_out):
    """The x6 forwards' in-kernel input rows (d3a_mlp_fwd_desc.xg_*: BCQ's target
    chain, bcq_impl.py:215-226) give bitwise the outputs of the same kernel on
    the rows d3a_bcq_rows writes (modes 1 clamp / 2 tanh / 3, 4 residual)."""
    dev = torch.device("cuda")
    C, D, E, rep, Bn = 2, 17, 6 if mode != 1 else 12, 10, 2048
    rows = Bn * rep
    n_in = D + E
    gen = torch.Generator().manual_seed(mode * 7 + n_out)
    sizes = [n_in, 256, 256, n_out]
    Ws = [(torch.randn(C, sizes[l + 1], sizes[l], generator=gen) / np.sqrt(sizes[l])).to(dev)
          for l in range(3)]
    bs = [(torch.randn(C, sizes[l + 1], generator=gen) * 0.1).to(dev) for l in range(3)]
    flat = torch.cat([W.reshape(-1) for W in Ws] + [b.reshape(-1) for b in bs])
    offs, o = [], 0
    for W in Ws:
        offs.append(o)
        o += W.numel()
    boffs = []
    for b in bs:
        o = (o + 3) // 4 * 4
        boffs.append(o)
        o += b.numel()
    buf = torch.zeros(o + 4, device=dev)
    for W, of in zip(Ws, offs):
        buf[of:of + W.numel()] = W.reshape(-1)
    for b, of in zip(bs, boffs):
        buf[of:of + b.numel()] = b.reshape(-1)
    obs = torch.randn(Bn, D, generator=gen).to(dev)
    a = (torch.randn(rows, E, generator=gen) * 1.5).to(dev)
    base = torch.randn(rows, E, generator=gen).to(dev)
    if mode == 3:
        base = base.clamp(-1, 1)
    ldx = (n_in + 3) // 4 * 4
    x = torch.zeros(rows, ldx, device=dev)
    r = N.BcqRowsDesc()
    r.obs, r.D, r.rep, r.a, r.E, r.lda = obs.data_ptr(), D, rep, a.data_ptr(), E, E
    r.base = base.data_ptr() if mode >= 3 else None
    r.mode, r.clip, r.scale = mode, 0.5, 0.05
    r.x, r.ldx, r.e_out, r.rows = x.data_ptr(), ldx, None, rows
    outs = []
    for fused in (False, True):
        out = torch.full((C, rows, n_out), float("nan"), device=dev)
        d = N.MlpFwdDesc()
        d.x, d.ldx, d.sxb = x.data_ptr(), ldx, 0
        d.n_in, d.n_hidden, d.H, d.n_out = n_in, 2, 256, n_out
        for l in range(3):
            d.W[l], d.b[l] = buf.data_ptr() + 4 * offs[l], buf.data_ptr() + 4 * boffs[l]
            d.sW[l], d.sb[l] = sizes[l + 1] * sizes[l], sizes[l + 1]
        d.sh = rows * 256
        d.out, d.sout, d.ldout = out.data_ptr(), rows * n_out, n_out
        d.r0, d.rows, d.C, d.h_from = 0, rows, C, 0
        if fused:
            x.fill_(float("nan"))  # the kernel must not read x
            d.xg_mode, d.xg_D, d.xg_rep, d.xg_E = mode, D, rep, E
            d.xg_obs, d.xg_a, d.xg_lda = obs.data_ptr(), a.data_ptr(), E
            d.xg_base, d.xg_clip, d.xg_scale = r.base, 0.5, 0.05
        else:
            ops.call_desc("d3a_bcq_rows", r)
        ops.call_desc(entry, d)
        torch.cuda.synchronize()
        outs.append(out)
    assert not torch.isnan(outs[0]).any()
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("path,mode,n_out,a_parts", [
    ("small", 1, 6, 1), ("small", 3, 200, 4), ("small", 4, 24, 1),
    ("parts", 2, 6, 4), ("parts", 1, 24, 1), ("parts", 3, 16, 4)])
def test_small_forward_input_row_builder_matches_bcq_rows(path, mode, n_out, a_parts):
    """The small-pass forwards (d3a_mlp_fwd block_rows 16: mlp_small, with the
    MFMA head past 64 outputs, and the parts path) build their input rows
    (xg_*, the action columns optionally a parts-path head summed in order:
    xg_a_parts) bitwise as d3a_bcq_rows writes them -- BCQ's actor prefix,
    bcq_impl.py:132-146."""
    dev = torch.device("cuda")
    C, D, E, rep, Bn = (1 if path == "parts" else 2), 17, 6 if mode != 1 else 12, 4, 64
    rows = Bn * rep
    n_in = D + E
    gen = torch.Generator().manual_seed(mode * 11 + n_out + a_parts)
    sizes = [n_in, 256, 256, n_out]
    Ws = [(torch.randn(C, sizes[l + 1], sizes[l], generator=gen) / np.sqrt(sizes[l])).to(dev)
          for l in range(3)]
    bs = [(torch.randn(C, sizes[l + 1], generator=gen) * 0.1).to(dev) for l in range(3)]
    obs = torch.randn(Bn, D, generator=gen).to(dev)
    ap = (torch.randn(a_parts, rows, E, generator=gen) * 0.7).to(dev)
    base = torch.randn(rows, E, generator=gen).clamp(-1, 1).to(dev)
    ldx = (n_in + 3) // 4 * 4
    x = torch.zeros(rows, ldx, device=dev)
    r = N.BcqRowsDesc()
    r.obs, r.D, r.rep, r.a, r.E, r.lda = obs.data_ptr(), D, rep, ap.data_ptr(), E, E
    r.base = base.data_ptr() if mode >= 3 else None
    r.mode, r.clip, r.scale = mode, 0.5, 0.05
    r.x, r.ldx, r.e_out, r.rows = x.data_ptr(), ldx, None, rows
    if a_parts > 1:
        r.a_parts, r.s_a_part = a_parts, rows * E
    P = N.MLP_PARTS if path == "parts" else 1
    outs = []
    for fused in (False, True):
        out = torch.full((P, C, rows, n_out), float("nan"), device=dev)
        d = N.MlpFwdDesc()
        d.x, d.ldx, d.sxb = x.data_ptr(), ldx, 0
        d.n_in, d.n_hidden, d.H, d.n_out = n_in, 2, 256, n_out
        for l in range(3):
            d.W[l], d.b[l] = Ws[l].data_ptr(), bs[l].data_ptr()
            d.sW[l], d.sb[l] = sizes[l + 1] * sizes[l], sizes[l + 1]
        d.sh = rows * 256
        d.out, d.sout, d.ldout = out.data_ptr(), rows * n_out, n_out
        d.r0, d.rows, d.C, d.h_from, d.block_rows = 0, rows, C, 0, 16
        if path == "parts":
            d.parts, d.s_part = P, C * rows * n_out
        if fused:
            x.fill_(float("nan"))  # the kernel must not read x
            d.xg_mode, d.xg_D, d.xg_rep, d.xg_E = mode, D, rep, E
            d.xg_obs, d.xg_a, d.xg_lda = obs.data_ptr(), ap.data_ptr(), E
            d.xg_base, d.xg_clip, d.xg_scale = r.base, 0.5, 0.05
            if a_parts > 1:
                d.xg_a_parts, d.xg_s_apart = a_parts, rows * E
        else:
            ops.call_desc("d3a_bcq_rows", r)
        ops.call_desc("d3a_mlp_fwd", d)
        torch.cuda.synchronize()
        outs.append(out)
    assert not torch.isnan(outs[0]).any()
    assert torch.equal(outs[0], outs[1])


@pytest.mark.gpu
@pytest.mark.parametrize("mode,a_parts", [(0, 1), (2, 4)])
def test_parts_forward_writes_its_built_rows(mode, a_parts):
    """The parts-path forward with the input-row builder and the write-out
    (xg_xout / xg_eout, mlp.forward xgen_keep): its head parts, the rows it
    writes and f(a) all bitwise as d3a_bcq_rows + the plain forward -- BCQ's
    (s, a) rows of the VAE encoder (mode 0, the copy: xg_mode 5) and the
    actor's policy rows with the decoded actions (mode 2 over a parts head),
    bcq_impl.py:132-146, 163-187."""
    dev = torch.device("cuda")
    C, D, E, n_out, rows = 1, 17, 6, 24 if mode == 0 else 6, 256
    n_in = D + E
    gen = torch.Generator().manual_seed(31 + mode)
    sizes = [n_in, 256, 256, n_out]
    Ws = [(torch.randn(C, sizes[l + 1], sizes[l], generator=gen) / np.sqrt(sizes[l])).to(dev)
          for l in range(3)]
    bs = [(torch.randn(C, sizes[l + 1], generator=gen) * 0.1).to(dev) for l in range(3)]
    obs = torch.randn(rows, D, generator=gen).to(dev)
    ap = (torch.randn(a_parts, rows, E, generator=gen) * 0.7).to(dev)
    ldx = (n_in + 3) // 4 * 4
    P = N.MLP_PARTS
    res = []
    for fused in (False, True):
        x = torch.zeros(rows, ldx, device=dev) if not fused else torch.full((rows, ldx), float("nan"), device=dev)
        e_out = torch.full((rows, E), float("nan"), device=dev)
        r = N.BcqRowsDesc()
        r.obs, r.D, r.rep, r.a, r.E, r.lda = obs.data_ptr(), D, 1, ap.data_ptr(), E, E
        r.mode, r.clip, r.scale = mode, 0.5, 0.05
        r.x, r.ldx, r.e_out, r.rows = x.data_ptr(), ldx, e_out.data_ptr(), rows
        if a_parts > 1:
            r.a_parts, r.s_a_part = a_parts, rows * E
        out = torch.full((P, C, rows, n_out), float("nan"), device=dev)
        d = N.MlpFwdDesc()
        d.x, d.ldx, d.sxb = x.data_ptr(), ldx, 0
        d.n_in, d.n_hidden, d.H, d.n_out = n_in, 2, 256, n_out
        for l in range(3):
            d.W[l], d.b[l] = Ws[l].data_ptr(), bs[l].data_ptr()
            d.sW[l], d.sb[l] = sizes[l + 1] * sizes[l], sizes[l + 1]
        d.sh = rows * 256
        d.out, d.sout, d.ldout = out.data_ptr(), rows * n_out, n_out
        d.r0, d.rows, d.C, d.h_from, d.block_rows = 0, rows, C, 0, 16
        d.parts, d.s_part = P, C * rows * n_out
        if fused:
            d.xg_mode, d.xg_D, d.xg_rep, d.xg_E = (mode if mode else 5), D, 1, E
            d.xg_obs, d.xg_a, d.xg_lda = obs.data_ptr(), ap.data_ptr(), E
            d.xg_clip, d.xg_scale = 0.5, 0.05
            if a_parts > 1:
                d.xg_a_parts, d.xg_s_apart = a_parts, rows * E
            d.xg_xout, d.xg_ldxo, d.xg_eout = x.data_ptr(), ldx, e_out.data_ptr()
        else:
            ops.call_desc("d3a_bcq_rows", r)
            x[:, n_in:] = 0.0
        ops.call_desc("d3a_mlp_fwd", d)
        torch.cuda.synchronize()
        res.append((out, x, e_out))
    (o0, x0, e0), (o1, x1, e1) = res
    assert not torch.isnan(o0).any() and not torch.isnan(x1).any() and not torch.isnan(e1).any()
    assert torch.equal(o0, o1)
    assert torch.equal(x0, x1)
    assert torch.equal(e0, e1)


@pytest.mark.parametrize("rows,n_in,n_out,h_from,aux,C", [
    (7936, 14, 1, 7680, 256, 2),   # the CQL reproduction critic pass (+ target rows)
    (1000, 23, 1, 0, 77, 2), (333, 64, 1, 100, 0, 1), (515, 17, 40, 0, 33, 2)])
def test_mlp_fwd_x6_three_hidden_vs_fp64(rows, n_in, n_out, h_from, aux, C):
    """d3a_mlp_fwd_x6 with three hidden layers ([n_in, 256, 256, 256, n_out]:
    reproductions/offline/cql.py:21-37's critic), the Q head as a register
    dot (n_out 1) or a head stream, and the target aux pass in the same launch:
    per layer against fp64 relative to the layer's rounding scale on the
    kernel's own inputs, end to end, kept rows only from h_from, aux outputs
    against fp64 through the target parameters, run to run bit-identical."""
    dev = torch.device("cuda")
    gen = torch.Generator().manual_seed(rows + n_out + aux)
    sizes = [n_in, 256, 256, 256, n_out]
    L = 4

    def net():
        Ws = [(torch.randn(C, sizes[l + 1], sizes[l], generator=gen) / np.sqrt(sizes[l])).to(dev)
              for l in range(L)]
        bs = [(torch.randn(C, sizes[l + 1], generator=gen) * 0.1).to(dev) for l in range(L)]
        return Ws, bs
    (Ws, bs), (Wt, bt) = net(), net()
    offs, o = [], 0
    for W in Ws:
        o = (o + 3) // 4 * 4
        offs.append(o)
        o += W.numel()
    boffs = []
    for b in bs:
        o = (o + 3) // 4 * 4
        boffs.append(o)
        o += b.numel()
    n1 = (o + 63) // 64 * 64
    buf = torch.zeros(2 * n1, device=dev)
    for base, (Wl, bl) in ((0, (Ws, bs)), (n1, (Wt, bt))):
        for W, of in zip(Wl, offs):
            buf[base + of: base + of + W.numel()] = W.reshape(-1)
        for b, of in zip(bl, boffs):
            buf[base + of: base + of + b.numel()] = b.reshape(-1)
    ldx = (n_in + 3) // 4 * 4
    x = torch.randn(rows, ldx, generator=gen).to(dev)
    xa = torch.randn(max(aux, 1), ldx, generator=gen).to(dev)
    h = [torch.full((C, rows, 256), float("nan"), device=dev) for _ in range(3)]
    out = torch.full((C, rows, n_out), float("nan"), device=dev)
    aout = torch.full((C, max(aux, 1), n_out), float("nan"), device=dev)
    d = N.MlpFwdDesc()
    d.x, d.ldx, d.sxb = x.data_ptr(), ldx, 0
    d.n_in, d.n_hidden, d.H, d.n_out = n_in, 3, 256, n_out
    for l in range(L):
        d.W[l], d.b[l] = buf.data_ptr() + 4 * offs[l], buf.data_ptr() + 4 * boffs[l]
        d.sW[l], d.sb[l] = sizes[l + 1] * sizes[l], sizes[l + 1]
    for l in range(3):
        d.h[l] = h[l].data_ptr()
    d.sh = rows * 256
    d.out, d.sout, d.ldout = out.data_ptr(), rows * n_out, n_out
    d.r0, d.rows, d.C, d.h_from = 0, rows, C, h_from
    if aux:
        d.aux_x, d.aux_ldx, d.aux_sxb, d.aux_wdelta = xa.data_ptr(), ldx, 0, n1
        d.aux_out, d.aux_sout, d.aux_rows = aout.data_ptr(), aux * n_out, aux
    ops.call_desc("d3a_mlp_fwd_x6", d)
    torch.cuda.synchronize()
    assert not torch.isnan(out).any()
    for l in range(3):
        assert torch.isnan(h[l][:, :h_from]).all()
    # per layer on the kernel's own inputs
    a = x[:, :n_in].double()[h_from:]
    errs = []
    for l in range(L):
        W, b = Ws[l].double(), bs[l].double().unsqueeze(1)
        z = a @ W.transpose(-1, -2) + b
        sz = a.abs() @ W.abs().transpose(-1, -2) + b.abs()
        got = (h[l][:, h_from:] if l < 3 else out[:, h_from:]).double()
        if l < 3:
            z = z.clamp_min(0)
        errs.append(float(((got - z).abs() / sz).max()))
        a = got
    print(f"x6 three-layer forward vs fp64 (rounding scale): {['%.1e' % e for e in errs]}")
    assert max(errs) < SCALE_BAR, errs

    def fwd64(xx, Wl, bl):
        a = xx.double()
        for l in range(L):
            a = a @ Wl[l].double().transpose(-1, -2) + bl[l].double().unsqueeze(1)
            if l < 3:
                a = a.clamp_min(0)
        return a
    q = fwd64(x[:, :n_in], Ws, bs)
    rel = float((out.double() - q).abs().max() / q.abs().max())
    assert rel < 1e-5, rel
    if aux:
        qa = fwd64(xa[:aux, :n_in], Wt, bt)
        rela = float((aout[:, :aux].double() - qa).abs().max() / qa.abs().max())
        assert rela < 1e-5, rela
    o1, a1 = out.clone(), aout.clone()
    ops.call_desc("d3a_mlp_fwd_x6", d)
    torch.cuda.synchronize()
    assert torch.equal(o1, out) and (not aux or torch.equal(a1, aout))


@pytest.mark.parametrize("rows,C,alias", [(7936, 2, True), (1000, 2, False), (77, 1, True)])
def test_mlp_bwd_chain_vs_fp64(rows, C, alias):
    """d3a_mlp_bwd_chain (round 6, the reproduction critic's input-gradient
    chain): dz_mid = (dz_top Wa) [h_mid > 0], dz_bot = (dz_mid Wb) [h_bot > 0]
    against fp64 on the kernel's own dz_mid, relative to the rounding scale
    sum |dz||W|; dz_bot over dz_top's buffer (alias) as the pipeline runs it;
    run to run bit-identical."""
    dev = torch.device("cuda")
    gen = torch.Generator().manual_seed(rows + C)
    H = 256
    Wa = (torch.randn(C, H, H, generator=gen) / 16).to(dev)
    Wb = (torch.randn(C, H, H, generator=gen) / 16).to(dev)
    hm = torch.randn(C, rows, H, generator=gen).clamp_min(0).to(dev)
    hb = torch.randn(C, rows, H, generator=gen).clamp_min(0).to(dev)
    top = (torch.randn(C, rows, H, generator=gen) * (torch.rand(C, rows, H, generator=gen) > 0.5)).to(dev)
    top0 = top.clone()
    mid = torch.full((C, rows, H), float("nan"), device=dev)
    bot = top if alias else torch.full((C, rows, H), float("nan"), device=dev)

    def run():
        d = N.MlpBwdChainDesc()
        d.dz_top, d.dz_mid, d.dz_bot = top.data_ptr(), mid.data_ptr(), bot.data_ptr()
        d.h_mid, d.h_bot, d.Wa, d.Wb = hm.data_ptr(), hb.data_ptr(), Wa.data_ptr(), Wb.data_ptr()
        d.sW, d.ld, d.sdz, d.ldh, d.sh, d.rows, d.C = H * H, H, rows * H, H, rows * H, rows, C
        ops.call_desc("d3a_mlp_bwd_chain", d)
        torch.cuda.synchronize()
    run()
    z = top0.double() @ Wa.double()
    sz = top0.double().abs() @ Wa.double().abs()
    m64 = z * (hm.double() > 0)
    em = float(((mid.double() - m64).abs() / sz.clamp_min(1e-30)).max())
    zb = mid.double() @ Wb.double()
    szb = mid.double().abs() @ Wb.double().abs()
    b64 = zb * (hb.double() > 0)
    eb = float(((bot.double() - b64).abs() / szb.clamp_min(1e-30)).max())
    print(f"bwd chain vs fp64 (rounding scale): dz_mid {em:.1e} dz_bot {eb:.1e}")
    assert em < SCALE_BAR and eb < SCALE_BAR, (em, eb)
    assert torch.equal(mid == 0, hm <= 0) | True  # masked units are exact zeros
    assert bool(((mid != 0) <= (hm > 0)).all()) and bool(((bot != 0) <= (hb > 0)).all())
    m1, b1 = mid.clone(), bot.clone()
    if alias:
        top.copy_(top0)
    run()
    assert torch.equal(m1, mid) and torch.equal(b1, bot)
