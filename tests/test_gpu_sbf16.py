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


@pytest.mark.parametrize("terms", [3, 6])
def test_sbf16_input_gradient_gemm(terms):
    """dx = (dz @ W) * [h > 0] with W [out][in] (n-contiguous B, transposed
    while staging): exact on bf16-representable data, fp32-level otherwise."""
    g = torch.Generator(device="cuda").manual_seed(3)
    C, R, O, I = 2, 4100, 256, 256
    dz = torch.randint(-8, 9, (C, R, O), device="cuda", generator=g).float() / 8
    W = torch.randint(-8, 9, (C, O, I), device="cuda", generator=g).float() / 16
    h = torch.randn(C, R, I, device="cuda", generator=g)
    ref = torch.einsum("cro,coi->cri", dz.double(), W.double()) * (h > 0)
    out = torch.empty(C, R, I, device="cuda")
    prev = ops.SBF16_TERMS
    ops.set_sbf16(terms)
    try:
        ops.linear_bwd_x(dz.data_ptr(), O, R * O, W.data_ptr(), out.data_ptr(), I, R * I, C, R,
                         I, O, mask=h.data_ptr(), ldm=I, smb=R * I)
        torch.cuda.synchronize()
        assert torch.equal(out.double(), ref)
        dz2 = torch.randn(C, R, O, device="cuda", generator=g) * 1e-3
        W2 = torch.randn(C, O, I, device="cuda", generator=g) * 0.06
        ops.linear_bwd_x(dz2.data_ptr(), O, R * O, W2.data_ptr(), out.data_ptr(), I, R * I, C, R,
                         I, O, mask=h.data_ptr(), ldm=I, smb=R * I)
        torch.cuda.synchronize()
    finally:
        ops.set_sbf16(prev)
    ref2 = torch.einsum("cro,coi->cri", dz2.double(), W2.double()) * (h > 0)
    e = float((out.double() - ref2).abs().max()) / float(ref2.abs().max())
    print(f"terms {terms}: input-gradient GEMM max-normalised error {e:.2e}")
    assert e <= (1e-6 if terms == 6 else 3e-5)


@pytest.mark.parametrize("terms", [3, 6])
def test_sbf16_weight_gradient_gemm(terms):
    """dW partials [S][C][out][in] = dz^T h over each row slice and the bias
    partials db[S][C][out] = sum_r dz (m-contiguous A and n-contiguous B, both
    transposed while staging; ragged last slice): exact on bf16-representable
    data, fp32-level otherwise; db is the fp64-accumulated fp32 row sum."""
    g = torch.Generator(device="cuda").manual_seed(5)
    C, R, O, I, S = 2, 5000, 256, 192, 7
    kchunk = -(-(-(-R // S)) // 32) * 32
    bounds = [(s * kchunk, min(R, (s + 1) * kchunk)) for s in range(S)]

    def ref(dz, h):
        dW = torch.stack([torch.einsum("cro,cri->coi", dz[:, a:e].double(), h[:, a:e].double())
                          for a, e in bounds])
        db = torch.stack([dz[:, a:e].double().sum(1) for a, e in bounds])
        return dW, db

    dW = torch.empty(S, C, O, I, device="cuda")
    db = torch.empty(S, C, O, device="cuda")

    def run(dz, h):
        ops.linear_bwd_w(dz.data_ptr(), O, R * O, h.data_ptr(), I, R * I, dW.data_ptr(), C, R,
                         I, O, S, db=db.data_ptr())
        torch.cuda.synchronize()

    dz = torch.randint(-8, 9, (C, R, O), device="cuda", generator=g).float() / 8
    h = torch.randint(0, 9, (C, R, I), device="cuda", generator=g).float() / 16
    prev = ops.SBF16_TERMS
    ops.set_sbf16(terms)
    try:
        run(dz, h)
        rW, rb = ref(dz, h)
        assert torch.equal(dW.double(), rW)
        assert torch.equal(db.double(), rb)
        dz2 = torch.randn(C, R, O, device="cuda", generator=g) * 1e-3
        h2 = torch.relu(torch.randn(C, R, I, device="cuda", generator=g))
        run(dz2, h2)
    finally:
        ops.set_sbf16(prev)
    rW, rb = ref(dz2, h2)
    e = float((dW.double() - rW).abs().max()) / float(rW.abs().max())
    eb = float((db.double() - rb).abs().max()) / float(rb.abs().max())
    print(f"terms {terms}: weight-gradient GEMM max-normalised error {e:.2e}, db {eb:.2e}")
    assert e <= (1e-6 if terms == 6 else 3e-5)
    assert eb <= 1e-7


def test_cql_sbf16x6_update_vs_fp64():
    """The K2 update with the large input-gradient GEMMs on split-bf16 x6
    (ops.set_sbf16(6), the opt-in throughput mode of bench.py --precision
    sbf16x6) meets the same fp64 arbiter bar as the fp32 path."""
    import test_gpu_cql_parity as t
    prev = ops.SBF16_TERMS
    ops.set_sbf16(6)
    try:
        t.test_cql_grad_accuracy_vs_fp64((11, 3))
    finally:
        ops.set_sbf16(prev)


@pytest.mark.parametrize("R,splits", [(1024, 8), (512, 16), (300, 3), (64, 1)])
def test_linear_fwd_splitk_matches_fp64(R, splits):
    """The K5 encoder fc (3,136 -> 512, ReLU) as split-K split-bf16 slices +
    the in-order epilogue (ops.linear_fwd_splitk): within 2e-6 of fp64,
    max-normalised (fp32-accurate six-product split; slices past K add zero
    partials)."""
    g = torch.Generator(device="cuda").manual_seed(R + splits)
    K, F = 3136, 512
    x = torch.relu(torch.randn(R, K, device="cuda", generator=g))
    W = torch.randn(F, K, device="cuda", generator=g) * (1.0 / K ** 0.5)
    b = torch.randn(F, device="cuda", generator=g) * 0.1
    y = torch.full((R, F), float("nan"), device="cuda")
    part = torch.full((splits, R, F), float("nan"), device="cuda")
    ops.linear_fwd_splitk(x.data_ptr(), K, W.data_ptr(), b.data_ptr(), y.data_ptr(), R, K, F,
                          True, part, splits)
    torch.cuda.synchronize()
    ref = torch.relu(x.double() @ W.double().T + b.double())
    err = float((y.double() - ref).abs().max() / ref.abs().max())
    print(f"R={R} splits={splits}: max err {err:.2e}")
    assert torch.isfinite(y).all() and err < 2e-6
