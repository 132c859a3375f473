"""Implicit-GEMM convolution kernels (d3a_conv_fwd / d3a_conv_bwd_w) against
torch fp64 conv2d and its autograd (GPU only).

The kernels replace nn.Conv2d in PixelEncoder._conv_encode
(d3rlpy/models/torch/encoders.py:130-162) with the PixelScaler
(preprocessing/scalers.py:109-110) fused into the first layer's loads.
Tolerance: 2e-5 of the output's max |value| (fp32 MFMA accumulation over up to
576 taps; the reference's CPU conv has its own summation order).
"""
import ctypes

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    from d3rlpy_amd import _native
    _native.lib()
    return torch.device("cuda:0")


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / max(1e-30, float(b.abs().max())))


# (B, C, H, W, CO, K, S, u8): the three Nature-DQN layers (conv1 also at 16
# frames: several 16-row steps a wave in conv1_bwd_w_u8s4_kernel; and C = 2,
# CO = 64: Kc = 128, two column blocks), ragged row counts
# (B*OH*OW not a multiple of 128), the unaligned uint8 path (S = 2), K*K*C not
# a multiple of 32 (C = 4, K = 3)
CASES = [(3, 4, 84, 84, 32, 8, 4, True), (16, 4, 84, 84, 32, 8, 4, True),
         (2, 2, 36, 84, 64, 8, 4, True), (5, 32, 20, 20, 64, 4, 2, False),
         (7, 64, 9, 9, 64, 3, 1, False), (2, 4, 18, 18, 32, 4, 2, True),
         (3, 4, 11, 13, 64, 3, 1, False), (1, 8, 9, 9, 32, 5, 2, False)]


def _inputs(g, B, C, H, W, CO, K, u8):
    if u8:
        xq = torch.randint(0, 256, (B, C, H, W), generator=g, dtype=torch.uint8)
        x_nchw = xq.double() / 255.0
    else:
        x_nchw = torch.randn(B, C, H, W, generator=g, dtype=torch.float64).float().double()
        xq = x_nchw.float().permute(0, 2, 3, 1).contiguous()  # NHWC
    Wt = (torch.randn(CO, C, K, K, generator=g) * (1.0 / (C * K * K) ** 0.5))
    bias = torch.randn(CO, generator=g) * 0.1
    return xq, x_nchw, Wt, bias


def _desc(N, B, C, H, W, CO, K, S):
    d = N.ConvDesc()
    d.B, d.C, d.H, d.W, d.KH, d.KW, d.S = B, C, H, W, K, K, S
    d.OH, d.OW, d.CO = (H - K) // S + 1, (W - K) // S + 1, CO
    return d


@pytest.mark.parametrize("B,C,H,W,CO,K,S,u8", CASES)
def test_conv_fwd_matches_torch(dev, B, C, H, W, CO, K, S, u8):
    from d3rlpy_amd import _native as N, ops
    g = torch.Generator().manual_seed(B * 131 + C * 7 + K)
    xq, x_nchw, Wt, bias = _inputs(g, B, C, H, W, CO, K, u8)
    ref = torch.relu(F.conv2d(x_nchw, Wt.double(), bias.double(), stride=S))  # NCHW
    ref = ref.permute(0, 2, 3, 1).reshape(-1, CO)
    d = _desc(N, B, C, H, W, CO, K, S)
    xd, Wd, bd = xq.to(dev), Wt.to(dev), bias.to(dev)
    y = torch.full((ref.shape[0], CO), float("nan"), device=dev)
    wpack = torch.full((CO * C * K * K,), float("nan"), device=dev)
    if u8:
        d.x_u8 = xd.data_ptr()
    else:
        d.x_f32, d.wpack = xd.data_ptr(), wpack.data_ptr()
    d.weight, d.bias, d.y, d.relu = Wd.data_ptr(), bd.data_ptr(), y.data_ptr(), 1
    ops.call_desc("d3a_conv_fwd", d)
    torch.cuda.synchronize()
    assert torch.isfinite(y).all()
    assert _rel(y, ref) < 2e-5


@pytest.mark.parametrize("B,C,H,W,CO,K,S,u8", CASES)
@pytest.mark.parametrize("splits", [1, 3, 32])
def test_conv_bwd_w_matches_autograd(dev, B, C, H, W, CO, K, S, u8, splits):
    from d3rlpy_amd import _native as N, ops
    g = torch.Generator().manual_seed(B * 17 + C + K + splits)
    xq, x_nchw, Wt, bias = _inputs(g, B, C, H, W, CO, K, u8)
    OH, OW = (H - K) // S + 1, (W - K) // S + 1
    dy = torch.randn(B, OH, OW, CO, generator=g)           # NHWC, pre-activation grad
    Wr = Wt.double().requires_grad_(True)
    br = bias.double().requires_grad_(True)
    out = F.conv2d(x_nchw, Wr, br, stride=S)
    out.backward(dy.double().permute(0, 3, 1, 2))
    d = _desc(N, B, C, H, W, CO, K, S)
    xd, Wd, dyd = xq.to(dev), Wt.to(dev), dy.to(dev).contiguous()
    dW = torch.full((splits, CO, C, K, K), float("nan"), device=dev)
    db = torch.full((splits, CO), float("nan"), device=dev)
    if u8:
        d.x_u8 = xd.data_ptr()
    else:
        d.x_f32 = xd.data_ptr()
    d.weight, d.dy, d.dW, d.db, d.splits = Wd.data_ptr(), dyd.data_ptr(), dW.data_ptr(), \
        db.data_ptr(), splits
    ops.call_desc("d3a_conv_bwd_w", d)
    torch.cuda.synchronize()
    assert torch.isfinite(dW).all() and torch.isfinite(db).all()
    assert _rel(dW.double().sum(0), Wr.grad) < 2e-5
    assert _rel(db.double().sum(0), br.grad) < 2e-5


def test_conv_fwd_pixel_scale_bit_exact(dev):
    """A one-hot kernel (tap (c, kh, kw) = 1, bias 0, no ReLU) copies x / 255:
    equal bit for bit to torch's x.float() / 255.0 for every byte value."""
    from d3rlpy_amd import _native as N, ops
    B, C, H, W, CO, K, S = 4, 4, 32, 32, 32, 8, 4
    x = torch.arange(B * C * H * W, dtype=torch.int64).remainder(256).to(torch.uint8)
    x = x.view(B, C, H, W)
    Wt = torch.zeros(CO, C, K, K)
    for co in range(CO):
        Wt[co, co % C, (co // C) % K, co % K] = 1.0
    d = _desc(N, B, C, H, W, CO, K, S)
    y = torch.full((B * d.OH * d.OW, CO), float("nan"), device=dev)
    xd, Wd, bd = x.to(dev), Wt.to(dev), torch.zeros(CO, device=dev)
    d.x_u8, d.weight, d.bias, d.y, d.relu = xd.data_ptr(), Wd.data_ptr(), bd.data_ptr(), \
        y.data_ptr(), 0
    ops.call_desc("d3a_conv_fwd", d)
    torch.cuda.synchronize()
    xs = x.float() / 255.0
    ref = torch.empty(B, d.OH, d.OW, CO)
    for co in range(CO):
        c, kh, kw = co % C, (co // C) % K, co % K
        ref[..., co] = xs[:, c, kh:kh + S * (d.OH - 1) + 1:S, kw:kw + S * (d.OW - 1) + 1:S]
    assert torch.equal(y.cpu(), ref.reshape(-1, CO))
    assert len(torch.unique(x)) == 256


def test_conv_rejects_bad_geometry(dev):
    from d3rlpy_amd import _native as N
    lib = N.lib()
    d = _desc(N, 1, 4, 84, 84, 48, 8, 4)          # CO must be 32 or 64
    d.x_u8, d.weight, d.y = 1, 1, 1
    assert lib.d3a_conv_fwd(ctypes.byref(d), None) < 0
    d = _desc(N, 1, 3, 84, 84, 32, 8, 4)          # fp32 NHWC needs C % 4 == 0
    d.x_f32, d.weight, d.y = 16, 16, 16
    assert lib.d3a_conv_fwd(ctypes.byref(d), None) < 0
    d = _desc(N, 1, 4, 84, 84, 32, 8, 4)
    d.OH = 21                                    # inconsistent output size
    d.x_u8, d.weight, d.y = 1, 1, 1
    assert lib.d3a_conv_fwd(ctypes.byref(d), None) < 0


# (B, C, H, W, CO, K, S): the K5 layers 2 and 3, uneven stride phases (H, W
# not multiples of S), a stride whose phases take different tap counts (K 4,
# S 3), CO 32
BWD_X_CASES = [(5, 32, 20, 20, 64, 4, 2), (7, 64, 9, 9, 64, 3, 1), (2, 32, 11, 13, 64, 3, 2),
               (3, 64, 10, 10, 32, 4, 3), (1, 32, 8, 8, 64, 8, 4)]


@pytest.mark.parametrize("B,C,H,W,CO,K,S", BWD_X_CASES)
@pytest.mark.parametrize("relu", [1, 0])
@pytest.mark.parametrize("packed", [True, False])
def test_conv_bwd_x_matches_autograd(dev, B, C, H, W, CO, K, S, relu, packed):
    """d3a_conv_bwd_x against autograd's input gradient of conv2d (fp64),
    times [x > 0] (the ReLU of the layer that produced x) when relu."""
    from d3rlpy_amd import _native as N, ops
    g = torch.Generator().manual_seed(B * 23 + C + K * 5 + S)
    x = torch.randn(B, C, H, W, generator=g, dtype=torch.float64).float().double()
    Wt = (torch.randn(CO, C, K, K, generator=g) * (1.0 / (C * K * K) ** 0.5))
    OH, OW = (H - K) // S + 1, (W - K) // S + 1
    dy = torch.randn(B, OH, OW, CO, generator=g)
    xr = x.clone().requires_grad_(True)
    F.conv2d(xr, Wt.double(), None, stride=S).backward(dy.double().permute(0, 3, 1, 2))
    ref = xr.grad * (x > 0) if relu else xr.grad
    ref = ref.permute(0, 2, 3, 1).reshape(-1, C)
    d = _desc(N, B, C, H, W, CO, K, S)
    xd = x.float().permute(0, 2, 3, 1).contiguous().to(dev)
    Wd, dyd = Wt.to(dev), dy.to(dev).contiguous()
    dx = torch.full((B * H * W, C), float("nan"), device=dev)
    d.x_f32, d.weight, d.dy, d.y, d.relu = xd.data_ptr(), Wd.data_ptr(), dyd.data_ptr(), \
        dx.data_ptr(), relu
    wpack = torch.full((CO * C * K * K,), float("nan"), device=dev)
    if packed:  # the re-laid weight path (CO % 32 == 0; else the gather path)
        d.wpack = wpack.data_ptr()
    ops.call_desc("d3a_conv_bwd_x", d)
    torch.cuda.synchronize()
    assert torch.isfinite(dx).all()
    assert _rel(dx, ref) < 2e-5
    if relu:
        assert bool((dx.cpu()[ref == 0] == 0).all())
