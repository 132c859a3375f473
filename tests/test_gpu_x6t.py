"""The slice kernel of the fp32-accurate critic backward (csrc/q2_x6_bwd2.hip,
d3a_q2_bwd_x6 with the transposed mask ``m2t``) against fp64, and the
forward's transposed mask bits (d3a_mlp_fwd_desc.hmaskT) against its row
mask bits.

The slice kernel reads no h2: dW3 = W2 . (m^T g' h1) + b2 (m^T g') -- the
forward's identity h2 = m (W2 h1 + b2) -- so its dW3 is checked against
fp64 g'^T h2 at the rounding scale of that sum of products,
sum_r |g'| m (sum_i |W2| h1 + |b2|); every other gradient at the bars of
tests/test_gpu_x6.py (the same mask-factored split-bf16 products)."""
import numpy as np
import pytest
import torch

from d3rlpy_amd import _native as N
from d3rlpy_amd import ops

from test_gpu_x6 import NAMES, SCALE_BAR, _bwd_case, _fwd_desc, _net

pytestmark = pytest.mark.gpu


def mask_bits(h2):
    """[C][R][256] -> (row words [C][R][8], transposed words [C][R / 32][256]
    lane-major: unit o at (o & 15) 16 + (o >> 4)), int32, as the forward
    writes them."""
    C, R, H = h2.shape
    on = (h2 > 0).to(torch.int64)
    sh = torch.arange(32, device=h2.device)
    m2 = (on.view(C, R, 8, 32) << sh).sum(-1)
    Rp = (R + 31) // 32 * 32
    onp = torch.zeros(C, Rp, H, dtype=torch.int64, device=h2.device)
    onp[:, :R] = on
    mt = (onp.view(C, Rp // 32, 32, H) << sh.view(1, 1, 32, 1)).sum(2)  # [C][G][o]
    mt = mt.view(C, Rp // 32, 16, 16).transpose(-1, -2).reshape(C, Rp // 32, H)

    def i32(t):
        return torch.where(t >= 2 ** 31, t - 2 ** 32, t).to(torch.int32).contiguous()
    return i32(m2), i32(mt)


def run_slice(rows, n_in, n_scaled, C, seed, row_splits=0):
    dev = torch.device("cuda")
    gen = torch.Generator().manual_seed(seed)
    Ws, bs = _net(C, n_in, gen, dev)
    ldx = (n_in + 3) // 4 * 4
    x = torch.randn(rows, ldx, generator=gen).to(dev)
    # the forward in fp64, rounded to the fp32 kept activations
    a = x[:, :n_in].double()
    h1 = (a @ Ws[0].double().transpose(1, 2) + bs[0].double().unsqueeze(1)).clamp_min(0).float()
    z2 = h1.double() @ Ws[1].double().transpose(1, 2) + bs[1].double().unsqueeze(1)
    h2 = z2.clamp_min(0)
    g = (torch.randn(C, rows, generator=gen) * 1e-2).to(dev)
    gscale = torch.tensor([0.7], device=dev)
    W2, w3, b2 = Ws[1].contiguous(), Ws[2].reshape(C, 256).contiguous(), bs[1].contiguous()
    m2, mt = mask_bits(h2)
    P = row_splits or N.lib().d3a_q2_bwd_x6t_splits(rows, C)
    outs = [torch.full((P, C, 256, n_in), float("nan"), device=dev),
            torch.full((P, C, 256), float("nan"), device=dev),
            torch.full((P, C, 256, 256), float("nan"), device=dev),
            torch.full((P, C, 256), float("nan"), device=dev),
            torch.full((16 * P, C, 256), float("nan"), device=dev),
            torch.full((P, C), float("nan"), device=dev)]
    d = N.Q2BwdDesc()
    d.x, d.ldx, d.sxb = x.data_ptr(), ldx, 0
    d.h1, d.h2, d.sh, d.ldh = h1.data_ptr(), None, rows * 256, 256
    d.g, d.sgb, d.gscale, d.n_scaled = g.data_ptr(), rows, gscale.data_ptr(), n_scaled
    d.W2, d.sW2, d.w3, d.sw3 = W2.data_ptr(), 256 * 256, w3.data_ptr(), 256
    d.b2, d.sb2 = b2.data_ptr(), 256
    d.dW1, d.db1, d.dW2, d.db2, d.dW3, d.db3 = [t.data_ptr() for t in outs]
    d.rows, d.n_in, d.C = rows, n_in, C
    d.m2, d.sm2 = m2.data_ptr(), rows * 8
    d.m2t, d.sm2t = mt.data_ptr(), mt.shape[1] * 256
    d.row_splits = row_splits
    ops.call_desc("d3a_q2_bwd_x6", d)
    torch.cuda.synchronize()
    # fp64 reference on the kernel's fp32 inputs, with rounding scales
    gp = g.double().clone()
    gp[:, :n_scaled] *= 0.7
    a1 = h1.double()
    m = (h2 > 0).double()
    dz2 = gp.unsqueeze(-1) * w3.double().unsqueeze(1) * m
    dh1 = dz2 @ W2.double()
    sdh1 = dz2.abs() @ W2.double().abs()
    dz1 = dh1 * (a1 > 0)
    xd = x[:, :n_in].double()
    pre_sc = a1 @ W2.double().abs().transpose(1, 2) + b2.double().abs().unsqueeze(1)
    ref = {"dW1": (dz1.transpose(1, 2) @ xd, (sdh1 * (a1 > 0)).transpose(1, 2) @ xd.abs()),
           "db1": (dz1.sum(1), (sdh1 * (a1 > 0)).sum(1)),
           "dW2": (dz2.transpose(1, 2) @ a1, dz2.abs().transpose(1, 2) @ a1),
           "db2": (dz2.sum(1), dz2.abs().sum(1)),
           "dW3": ((gp.unsqueeze(-1) * h2).sum(1), (gp.abs().unsqueeze(-1) * m * pre_sc).sum(1)),
           "db3": (gp.sum(1), gp.abs().sum(1))}
    # the descriptor holds raw pointers: its inputs travel with it
    d._keep = (x, h1, g, gscale, W2, w3, b2, m2, mt, Ws, bs)
    return outs, ref, d


@pytest.mark.parametrize("rows,n_in,n_scaled,C,splits", [
    (7936, 14, 7680, 2, 0),     # K2 critic backward (P = 8)
    (7936, 37, 7680, 2, 0),     # K4 antmaze shapes (three 16-wide x blocks)
    (1056, 20, 1000, 2, 0),     # ragged row blocks, two x blocks
    (2048, 14, 0, 1, 0),        # one member (P = 16)
    (640, 14, 320, 10, 0),      # ten critics (P = 1)
    (7936, 14, 7680, 2, 3),     # explicit row blocks, sub-blocks past the end
    (32, 14, 32, 2, 0),         # one sub-block
])
def test_q2_bwd_x6_slice_vs_fp64(rows, n_in, n_scaled, C, splits):
    outs, ref, d = run_slice(rows, n_in, n_scaled, C, rows * 7 + n_in + C, splits)
    worst = {}
    for name, o in zip(NAMES, outs):
        assert not torch.isnan(o).any(), name
        got = o.double().sum(0).cpu()
        r, sc = (v.cpu() for v in ref[name])
        e_sc = float(((got - r).abs() / sc.clamp_min(1e-30)).max())
        e_max = float((got - r).abs().max() / r.abs().max())
        worst[name] = (e_sc, e_max)
        assert e_sc < SCALE_BAR and e_max < 2e-6, (name, e_sc, e_max)
    print(f"slice backward rows {rows} n_in {n_in} C {C} vs fp64 (rounding scale, max-normalised): "
          + " ".join(f"{k} {a:.1e}/{b:.1e}" for k, (a, b) in worst.items()))
    first = [o.clone() for o in outs]
    ops.call_desc("d3a_q2_bwd_x6", d)
    torch.cuda.synchronize()
    for name, a, b in zip(NAMES, first, outs):
        assert torch.equal(a, b), (name, float((a - b).abs().max()))  # fixed reduction orders


@pytest.mark.parametrize("rows,h_from,n_in", [(15616, 7680, 14), (300, 96, 23), (1000, 0, 48)])
def test_q2_fwd_x6_transposed_mask(rows, h_from, n_in):
    """hmaskT holds the bits of hmask transposed (every 32-row group with a
    kept row), and the forward's other outputs are unchanged by writing it."""
    dev = torch.device("cuda")
    C = 2
    gen = torch.Generator().manual_seed(rows + 5)
    Ws, bs = _net(C, n_in, gen, dev)
    Wt, bt = _net(C, n_in, gen, dev)
    ldx = (n_in + 3) // 4 * 4
    x = torch.randn(rows, ldx, generator=gen).to(dev)
    G = (rows + 31) // 32
    res = []
    for with_t in (False, True):
        h = [torch.zeros(C, rows, 256, device=dev) for _ in range(2)]
        out, aout = torch.zeros(C, rows, device=dev), torch.zeros(C, 1, device=dev)
        d, _b = _fwd_desc(x, ldx, n_in, Ws, bs, Wt, bt, h, out, aout, x, rows, h_from, 0, C, dev)
        hm = torch.zeros(C, rows, 8, dtype=torch.int32, device=dev)
        d.hmask, d.s_hmask = hm.data_ptr(), rows * 8
        hmt = torch.full((C, G, 256), -7, dtype=torch.int32, device=dev)
        if with_t:
            d.hmaskT, d.s_hmaskT = hmt.data_ptr(), G * 256
        ops.call_desc("d3a_q2_fwd_x6", d)
        torch.cuda.synchronize()
        res.append((out.clone(), h[0].clone(), h[1].clone(), hm.clone(), hmt.clone()))
    for a, b in zip(res[0][:4], res[1][:4]):
        assert torch.equal(a, b)
    hm, hmt = res[1][3], res[1][4]
    # expected transposed words from the row words (kept rows), lane-major order
    bits = ((hm.to(torch.int64).unsqueeze(-1) >> torch.arange(32, device=dev)) & 1).view(C, rows, 256)
    g0 = h_from // 32
    Rp = G * 32
    on = torch.zeros(C, Rp, 256, dtype=torch.int64, device=dev)
    on[:, :rows] = bits
    on[:, :h_from] = 0
    want = (on.view(C, G, 32, 256) << torch.arange(32, device=dev).view(1, 1, 32, 1)).sum(2)
    want = want.view(C, G, 16, 16).transpose(-1, -2).reshape(C, G, 256)
    got = hmt.to(torch.int64) & 0xFFFFFFFF
    # rows past the end of the last group and rows before h_from in its group
    # carry whatever the forward computed there: compare kept rows only
    keep = torch.zeros(C, Rp, 256, dtype=torch.int64, device=dev)
    keep[:, h_from:rows] = 1
    kmask = (keep.view(C, G, 32, 256) << torch.arange(32, device=dev).view(1, 1, 32, 1)).sum(2)
    kmask = kmask.view(C, G, 16, 16).transpose(-1, -2).reshape(C, G, 256)
    assert torch.equal((got & kmask)[:, g0:], want[:, g0:])
    assert (hmt[:, :g0] == -7).all()  # groups with no kept row untouched
