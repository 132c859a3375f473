"""Split-bf16 GEMM (d3a_gemm_sbf16) on the bf16 matrix cores (GPU only).

1. Lane maps: operands exactly representable in bf16 (small integers x 2^-k)
   give the exact fp64 result with either split (every part but the first is
   zero), bias and ReLU included.
2. Accuracy at the K2 critic layer-1 shape (2 x 15616 rows x 256 x 256,
   K2-like magnitudes), max-normalised against fp64:
     terms 6 (hi/mid/lo): within 1e-6 — the fp32 MFMA GEMM's own level
     terms 3 (hi/lo):     within 3e-5 — not fp32-exact (printed beside fp32)
"""
import pytest
import torch

from d3rlpy_amd import ops

pytestmark = pytest.mark.gpu


def _ref(x, W, b, relu):
    y = torch.einsum("ri,coi->cro", x.double(), W.double()) + b.double()[:, None]
    return torch.relu(y) if relu else y


@pytest.mark.parametrize("terms", [3, 6])
def test_sbf16_exact_on_bf16_representable_data(terms):
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randint(-8, 9, (300, 64), device="cuda", generator=g).float() / 8
    W = torch.randint(-8, 9, (2, 96, 64), device="cuda", generator=g).float() / 16
    b = torch.randint(-8, 9, (2, 96), device="cuda", generator=g).float() / 4
    y = torch.empty(2, 300, 96, device="cuda")
    ops.gemm_sbf16(x, W, b, y, terms=terms, relu=True)
    torch.cuda.synchronize()
    assert torch.equal(y.double(), _ref(x, W, b, True))


def test_sbf16_accuracy_k2_layer():
    g = torch.Generator(device="cuda").manual_seed(1)
    R, H = 15616, 256
    x = torch.relu(torch.randn(R, H, device="cuda", generator=g))
    W = torch.randn(2, H, H, device="cuda", generator=g) * 0.0625
    b = torch.randn(2, H, device="cuda", generator=g) * 0.0625
    ref = _ref(x, W, b, False)
    scale = float(ref.abs().max())
    errs = {}
    for terms in (3, 6):
        y = torch.empty(2, R, H, device="cuda")
        ops.gemm_sbf16(x, W, b, y, terms=terms)
        torch.cuda.synchronize()
        errs[terms] = float((y.double() - ref).abs().max()) / scale
    y32 = torch.empty(2, R, H, device="cuda")
    ops.linear_fwd(x.data_ptr(), True, H, W.data_ptr(), b.data_ptr(), y32.data_ptr(), 2, R, H, H,
                   relu=False, ldy=H, sxb=0, syb=R * H)
    torch.cuda.synchronize()
    e32 = float((y32.double() - ref).abs().max()) / scale
    print(f"max-normalised error vs fp64: split-bf16 x3 {errs[3]:.2e}, x6 {errs[6]:.2e}, "
          f"fp32 MFMA {e32:.2e}")
    assert errs[6] <= 1e-6
    assert errs[3] <= 3e-5
