"""Thin Python wrappers around the C-ABI: torch tensors -> raw pointers.

Every wrapper enqueues on torch's *current* HIP stream and never
synchronises, so a sequence of calls can be captured into a HIP graph with
``torch.cuda.graph``.  Tensors must be fp32 (or the stated dtype), on the GPU
and contiguous where a row-major layout is implied.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import gc
import os
import warnings
from typing import Optional, Sequence

import torch

from . import _native as N

_F32 = 4
_TRACE = os.environ.get("D3A_GEMM_TRACE") == "1"  # print GEMM shapes as they are enqueued


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t: Optional[torch.Tensor], offset: int = 0) -> Optional[int]:
    """Device address of ``t`` plus ``offset`` elements (None for None)."""
    if t is None:
        return None
    return t.data_ptr() + offset * t.element_size()


def _need_gpu(*ts: Optional[torch.Tensor]) -> None:
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("d3rlpy_amd ops require device tensors (no CPU fallback)")


def gemm(A: int, B: int, Cp: int, M: int, Nn: int, K: int, *, batch: int = 1,
         sA: Sequence[int], sB: Sequence[int], sC: Sequence[int],
         bias: Optional[int] = None, sbias: int = 0,
         mask: Optional[int] = None, sM: Sequence[int] = (0, 0, 0),
         relu: bool = False, accumulate: bool = False, splits: int = 1, sCs: int = 0,
         alpha: float = 1.0, rowsum: Optional[int] = None, sR: Sequence[int] = (0, 0),
         variant: int = -1, pair: Optional[Sequence[int]] = None,
         agen: Optional[C.Structure] = None, wnext: Optional[C.Structure] = None) -> None:
    """C_b,s(m,n) = epi(alpha * sum_k A_b(m,k) B_b(k,n)); strides (batch, row, col).
    ``agen`` (a Head1BwdDesc): A is generated as that head's masked input
    gradient instead of read (d3a_gemm_desc.agen).
    ``pair = (dA, dB, dC, dbias)``: a second pass of the same shape at those
    element offsets in the same launch (d3a_gemm_desc.batch2 = 2)."""
    d = N.GemmDesc()
    d.A, d.B, d.C, d.bias, d.mask = A, B, Cp, bias, mask
    d.rowsum = rowsum
    d.sRb, d.sRs = sR
    d.variant = variant
    d.M, d.N, d.K, d.batch = M, Nn, K, batch
    d.sAb, d.sAm, d.sAk = sA
    d.sBb, d.sBk, d.sBn = sB
    d.sCb, d.sCm, d.sCn = sC
    d.sbias_b = sbias
    d.sMb, d.sMm, d.sMn = sM
    d.splits, d.sCs = splits, sCs
    d.alpha, d.relu, d.accumulate = alpha, int(relu), int(accumulate)
    if pair is not None:
        d.batch2 = 2
        d.sAb2, d.sBb2, d.sCb2, d.sbias_b2 = pair
    if agen is not None:
        d.agen = C.addressof(agen)
    if wnext is not None:
        d.wnext = C.addressof(wnext)
    if _TRACE:
        print(f"gemm M={M} N={Nn} K={K} batch={batch} splits={splits} sA={tuple(sA)} "
              f"sB={tuple(sB)} sC={tuple(sC)} mask={mask is not None} relu={relu} "
              f"rowsum={rowsum is not None} variant={variant}", flush=True)
    if _CAPTURE is not None:  # inside gemm_pair: submitted together
        _CAPTURE.append((d, agen, wnext))
        return
    N.check(N.lib().d3a_gemm_f32(C.byref(d), _stream()), "d3a_gemm_f32")


_CAPTURE = None  # descriptors collected by gemm_pair
PAIR = os.environ.get("D3A_GEMM_PAIR", "1") != "0"


def gemm_pair(first, second) -> None:
    """Enqueue two independent GEMM wrapper calls (``first()``, ``second()``,
    e.g. one backward layer's weight- and input-gradient GEMMs): when each
    enqueues one d3a_gemm_f32, both go to d3a_gemm_f32_pair (one launch where
    both take the register-direct kernel, else two launches)."""
    global _CAPTURE
    if not PAIR:
        first()
        second()
        return
    _CAPTURE = []
    try:
        first()
        second()
        caps = _CAPTURE
    finally:
        _CAPTURE = None
    if len(caps) == 2:
        N.check(N.lib().d3a_gemm_f32_pair(C.byref(caps[0][0]), C.byref(caps[1][0]), _stream()),
                "d3a_gemm_f32_pair")
    else:
        for d, _, _ in caps:
            N.check(N.lib().d3a_gemm_f32(C.byref(d), _stream()), "d3a_gemm_f32")


def rowdot(X: int, sXb: int, sXr: int, w: int, swb: int, bias: Optional[int], sbb: int,
           out: int, sOb: int, batch: int, rows: int, n: int,
           pair: Optional[Sequence[int]] = None, J: int = 1) -> None:
    """``J`` outputs per row (w [J][n], out rows of stride J); ``pair = (dX, dw,
    dbias, dout)``: a second pass at those element offsets."""
    if pair is None and J == 1:
        N.check(N.lib().d3a_rowdot_f32(X, sXb, sXr, w, swb, bias, sbb, out, sOb, batch, rows, n,
                                       _stream()), "d3a_rowdot_f32")
        return
    p = (1, 0, 0, 0, 0) if pair is None else (2,) + tuple(pair)
    N.check(N.lib().d3a_rowdot2_f32(X, sXb, sXr, w, swb, bias, sbb, out, sOb, batch, rows, n, J,
                                    *p, _stream()), "d3a_rowdot2_f32")


def colreduce(X: int, sXb: int, sXr: int, w: Optional[int], swb: int, out: int, sOb: int,
              sOs: int, batch: int, rows: int, n: int, splits: int) -> None:
    N.check(N.lib().d3a_colreduce_f32(X, sXb, sXr, w, swb, out, sOb, sOs, batch, rows, n,
                                      splits, _stream()), "d3a_colreduce_f32")


def outer_mask(g: int, sgb: int, w: int, swb: int, h: int, shb: int, out: int, sob: int,
               batch: int, rows: int, n: int) -> None:
    N.check(N.lib().d3a_outer_mask_f32(g, sgb, w, swb, h, shb, out, sob, batch, rows, n,
                                       _stream()), "d3a_outer_mask_f32")


def adam(segs: torch.Tensor, n_seg: int, n_blocks: int, step: torch.Tensor, lr: float,
         beta1: float, beta2: float, eps: float, grad_scale: float = 1.0) -> None:
    N.check(N.lib().d3a_adam_f32(ptr(segs), n_seg, n_blocks, ptr(step), lr, beta1, beta2, eps,
                                 grad_scale, _stream()), "d3a_adam_f32")


def adam_step(segs: torch.Tensor, n_seg: int, n_blocks: int, step: torch.Tensor, lr: float,
              beta1: float, beta2: float, eps: float, grad_scale: float = 1.0,
              step_add: int = 1, targ_delta: int = 0, tau: float = 0.0,
              counters: Optional[torch.Tensor] = None, inc_mask: int = 0,
              metrics: Optional[torch.Tensor] = None, ring: Optional[torch.Tensor] = None,
              ring_ctr: Optional[torch.Tensor] = None, metric_scale: float = 1.0,
              blocks: Optional[torch.Tensor] = None, commit_src: Optional[torch.Tensor] = None,
              commit_dst: Sequence[torch.Tensor] = (),
              commit_step: Sequence[Optional[torch.Tensor]] = (),
              one_elem: bool = False) -> None:
    """d3a_adam_step: Adam with the soft target update (``targ_delta`` != 0:
    the target copy ``targ_delta`` elements from each parameter) and the
    step's counter / metric-ring bookkeeping in one launch.  ``one_elem``: no
    segment takes four elements a thread (AdamGroup.one_elem)."""
    d = N.AdamDesc()
    d.segs, d.n_seg, d.n_blocks = ptr(segs), n_seg, n_blocks
    d.step, d.step_add = ptr(step), step_add
    d.lr, d.beta1, d.beta2, d.eps, d.grad_scale = lr, beta1, beta2, eps, grad_scale
    d.soft, d.targ_delta, d.tau = int(targ_delta != 0), targ_delta, tau
    d.counters, d.inc_mask = ptr(counters), inc_mask
    if ring is not None:
        d.metrics, d.n_metrics = ptr(metrics), metrics.numel()
        d.ring, d.ring_cap, d.ring_ctr = ptr(ring), ring.shape[0], ptr(ring_ctr)
    d.metric_scale = metric_scale
    d.blocks = ptr(blocks)  # per-block segment table (AdamGroup), or None
    d.one_elem = int(one_elem)
    if commit_src is not None:
        # a scalar optimiser state staged by an earlier launch of the update
        assert len(commit_dst) <= 8 and commit_src.numel() >= len(commit_dst)
        d.commit_src, d.n_commit = ptr(commit_src), len(commit_dst)
        for i, t in enumerate(commit_dst):
            d.commit_dst[i] = ptr(t)
        for i, t in enumerate(commit_step):
            d.commit_step[i] = ptr(t)
    N.check(N.lib().d3a_adam_step(C.byref(d), _stream()), "d3a_adam_step")


def grad_reduce(segs: torch.Tensor, n_seg: int, n_blocks: int) -> None:
    N.check(N.lib().d3a_grad_reduce_f32(ptr(segs), n_seg, n_blocks, _stream()),
            "d3a_grad_reduce_f32")


def step_end(counters: Optional[torch.Tensor], inc_mask: int, metrics: Optional[torch.Tensor] = None,
             ring: Optional[torch.Tensor] = None, ring_ctr: Optional[torch.Tensor] = None,
             targ: Optional[torch.Tensor] = None, src: Optional[torch.Tensor] = None,
             tau: float = 0.0, metric_scale: float = 1.0) -> None:
    """Soft target update (optional) + metric ring push + step counters, one launch."""
    n = metrics.numel() if metrics is not None else 0
    cap = ring.shape[0] if ring is not None else 0
    ns = targ.numel() if targ is not None else 0
    if targ is not None:
        assert src is not None and src.numel() == ns
    N.check(N.lib().d3a_step_end(ptr(metrics), n, ptr(ring), cap, ptr(ring_ctr), ptr(counters),
                                 inc_mask, ptr(targ), ptr(src), ns, float(tau),
                                 float(metric_scale), _stream()),
            "d3a_step_end")


def standardize(x: torch.Tensor, y: torch.Tensor, mean: torch.Tensor, std: torch.Tensor,
                eps: float) -> None:
    """y = (x - mean) / (std + eps) row-wise (StandardScaler.transform)."""
    _need_gpu(x, y, mean, std)
    assert x.shape == y.shape and x.dim() == 2 and x.stride(1) == 1 and y.stride() == x.stride()
    N.check(N.lib().d3a_standardize_f32(ptr(x), ptr(y), x.shape[0], x.shape[1], x.stride(0),
                                        ptr(mean), ptr(std), float(eps), _stream()),
            "d3a_standardize_f32")


def soft_update(targ: torch.Tensor, src: torch.Tensor, tau: float) -> None:
    _need_gpu(targ, src)
    assert targ.numel() == src.numel() and targ.dtype == src.dtype == torch.float32
    N.check(N.lib().d3a_soft_update_f32(ptr(targ), ptr(src), targ.numel(), float(tau),
                                        _stream()), "d3a_soft_update_f32")


def gemm_sbf16(x: torch.Tensor, W: torch.Tensor, b: Optional[torch.Tensor], y: torch.Tensor,
               terms: int = 6, relu: bool = False) -> None:
    """y[c] = epi(x[c] @ W[c]^T + b[c]) on the bf16 matrix cores with split-bf16
    operands (d3a_gemm_sbf16): x [C, R, in] (or [R, in] shared), W [C, out, in],
    b [C, out], y [C, R, out]."""
    _need_gpu(x, W, b, y)
    C_, out, n_in = W.shape
    shared = x.dim() == 2
    R = x.shape[0] if shared else x.shape[1]
    d = N.GemmDesc()
    d.A, d.B, d.C = ptr(x), ptr(W), ptr(y)
    d.bias = ptr(b)
    d.M, d.N, d.K, d.batch = R, out, n_in, C_
    d.sAb, d.sAm, d.sAk = (0 if shared else R * n_in), n_in, 1
    d.sBb, d.sBk, d.sBn = out * n_in, 1, n_in
    d.sCb, d.sCm, d.sCn = R * out, out, 1
    d.sbias_b = out
    d.splits, d.alpha, d.relu, d.variant, d.batch2 = 1, 1.0, int(relu), -1, 1
    N.check(N.lib().d3a_gemm_sbf16(C.byref(d), terms, _stream()), "d3a_gemm_sbf16")


def linear_fwd_sbf16(x: int, ldx: int, W: int, b: Optional[int], y: int, C_: int, R: int,
                     n_in: int, n_out: int, relu: bool, ldy: int, sxb: int, syb: int,
                     terms: int = 6) -> None:
    """y[c] = act(x[c] @ W[c]^T + b[c]) on d3a_gemm_sbf16 (split-bf16 operands,
    ``terms`` 6: fp32-accurate); pointer form of ``gemm_sbf16``."""
    d = N.GemmDesc()
    d.A, d.B, d.C = x, W, y
    d.bias = b
    d.M, d.N, d.K, d.batch = R, n_out, n_in, C_
    d.sAb, d.sAm, d.sAk = sxb, ldx, 1
    d.sBb, d.sBk, d.sBn = n_out * n_in, 1, n_in
    d.sCb, d.sCm, d.sCn = syb, ldy, 1
    d.sbias_b = n_out
    d.splits, d.alpha, d.relu, d.variant, d.batch2 = 1, 1.0, int(relu), -1, 1
    N.check(N.lib().d3a_gemm_sbf16(C.byref(d), terms, _stream()), "d3a_gemm_sbf16")


def linear_fwd_splitk(x: int, ldx: int, W: int, b: Optional[int], y: int, R: int, n_in: int,
                      n_out: int, relu: bool, part: torch.Tensor, splits: int) -> None:
    """y = act(x @ W^T + b) for one long-K Linear (K5's encoder fc, 3,136 -> 512)
    on the bf16 matrix cores with fp32-accurate split-bf16 operands (six
    products): ``splits`` K slices into ``part`` [splits][R][n_out], then
    d3a_splitk_epilogue_f32 adds them in order with the bias and ReLU."""
    assert part.numel() >= splits * R * n_out and part.is_cuda
    d = N.GemmDesc()
    d.A, d.B, d.C = x, W, part.data_ptr()
    d.M, d.N, d.K, d.batch = R, n_out, n_in, 1
    d.sAb, d.sAm, d.sAk = 0, ldx, 1
    d.sBb, d.sBk, d.sBn = 0, 1, n_in
    d.sCb, d.sCm, d.sCn = 0, n_out, 1
    d.splits, d.sCs = splits, R * n_out
    d.alpha, d.relu, d.variant, d.batch2 = 1.0, 0, -1, 1
    N.check(N.lib().d3a_gemm_sbf16(C.byref(d), 6, _stream()), "d3a_gemm_sbf16")
    N.check(N.lib().d3a_splitk_epilogue_f32(part.data_ptr(), splits, R * n_out, y, b, R, n_out,
                                            int(relu), _stream()), "d3a_splitk_epilogue_f32")


def conv_pack_weights(descs, layouts, philox=None) -> None:
    """d3a_conv_pack_weights over up to 8 ConvDescs (weight -> wpack in layout
    0: the forward's walk order, 1: the input gradient's tap-major order);
    ``philox`` (a PhiloxJob): d3a_conv_pack_weights_philox, the fill on the
    same launch's appended workgroups."""
    n = len(descs)
    arr = (N.ConvDesc * n)(*descs)
    lays = (C.c_int32 * n)(*layouts)
    if philox is not None:
        N.check(N.lib().d3a_conv_pack_weights_philox(arr, lays, n, C.byref(philox), _stream()),
                "d3a_conv_pack_weights_philox")
        return
    N.check(N.lib().d3a_conv_pack_weights(arr, lays, n, _stream()), "d3a_conv_pack_weights")


def philox_fill(out: torch.Tensor, n_normal: int, n_uniform: int, lo: float, hi: float,
                seed: int, ctr: torch.Tensor, ticket: torch.Tensor) -> None:
    _need_gpu(out, ctr, ticket)
    assert out.numel() >= n_normal + n_uniform
    N.check(N.lib().d3a_philox_fill(ptr(out), n_normal, n_uniform, lo, hi,
                                    C.c_uint64(seed & 0xFFFFFFFFFFFFFFFF), ptr(ctr), ptr(ticket),
                                    _stream()), "d3a_philox_fill")


def call_desc(fn_name: str, desc: C.Structure, desc2: Optional[C.Structure] = None) -> None:
    fn = getattr(N.lib(), fn_name)
    if desc2 is None:
        N.check(fn(C.byref(desc), _stream()), fn_name)
    else:
        N.check(fn(C.byref(desc), C.byref(desc2), _stream()), fn_name)


# ---------------------------------------------------------------------------
# nn.Linear helpers over an ensemble of C members stored [C][out][in]
# ---------------------------------------------------------------------------
def linear_fwd(x: int, x_shared: bool, ldx: int, W: int, b: int, y: int, C_: int, R: int,
               n_in: int, n_out: int, relu: bool, ldy: Optional[int] = None,
               sxb: Optional[int] = None, syb: Optional[int] = None, variant: int = -1,
               pair: Optional[Sequence[int]] = None) -> None:
    """y[c] = act(x[c] @ W[c]^T + b[c]); x rows have stride ldx; y is [C][R][n_out].
    ``pair = (dx, dW, dy)`` element offsets of a second pass of the same shape
    (its bias at b + dW) in the same launch."""
    ldy = n_out if ldy is None else ldy
    sxb = (0 if x_shared else R * ldx) if sxb is None else sxb
    syb = R * ldy if syb is None else syb
    gemm(x, W, y, R, n_out, n_in, batch=C_, sA=(sxb, ldx, 1), sB=(n_out * n_in, 1, n_in),
         sC=(syb, ldy, 1), bias=b, sbias=n_out, relu=relu, variant=variant,
         pair=None if pair is None else (pair[0], pair[1], pair[2], pair[1]))


# split-bf16 precision mode for the large input-gradient GEMMs (0 = fp32 MFMA,
# the default and the parity / headline path; 6 = hi/mid/lo split-bf16, fp32-
# accurate; 3 = hi/lo): set with set_sbf16() before the update graphs are captured
SBF16_TERMS = int(os.environ.get("D3A_SBF16", "0"))
SBF16_MIN_ROWS = 4096
SBF16_W = os.environ.get("D3A_SBF16_W", "1") == "1"  # also the weight-gradient GEMMs


# critic-ensemble precision of the large CQL critic passes: "fp32" (the
# reference's; parity path), "bf16" (throughput line: the forward's operands
# rounded to one bf16 part, d3a_q2_fwd_x1, fp32 kept activations; the backward
# the mask-factored split-bf16 d3a_q2_bwd_x6, whose non-mask operands keep
# three parts) or "bf16h" (round 3's line: d3a_q2_fwd_bf16 / d3a_q2_bwd_bf16,
# every operand one bf16 part, bf16 kept activations).  Read when an Impl
# builds its pipeline workspace and at each launch.  NOTE: until round 4
# "bf16" named what is now "bf16h"; round-3 bf16 bench lines correspond to
# "bf16h" and are not comparable with "bf16" lines (bench.py tags each line
# with its kernel pair).
CRITIC_PRECISION = os.environ.get("D3A_CRITIC_PRECISION", "fp32")
_BF16_RENAMED = ("critic precision 'bf16' selects the x1 forward + the split-bf16 x6 "
                 "backward with fp32 kept activations since round 4; round 3's all-bf16 "
                 "line (d3a_q2_fwd_bf16 / d3a_q2_bwd_bf16) is now 'bf16h'")


def set_critic_precision(p: str) -> None:
    global CRITIC_PRECISION
    if p not in ("fp32", "bf16", "bf16h"):
        raise ValueError(f"critic precision must be fp32, bf16 or bf16h, got {p!r}")
    if p == "bf16":
        warnings.warn(_BF16_RENAMED, stacklevel=2)
    CRITIC_PRECISION = p


if CRITIC_PRECISION == "bf16":
    warnings.warn(_BF16_RENAMED + " (D3A_CRITIC_PRECISION)", stacklevel=1)


# GEMM arithmetic of the [n_in <= 48, 256, 256, 1] critic passes at fp32
# precision: "fp32" (v_mfma_f32_32x32x2_f32, exact fp32 fma chains: q2_fwd /
# q2_bwd) or "x6" (exact three-way split-bf16 operands on the bf16 matrix
# cores, fp32-accurate: d3a_q2_fwd_x6 / d3a_q2_bwd_x6, csrc/q2_x6*.hip; the
# default since round 4: it holds the same parity bars, tests/test_gpu_x6.py,
# test_gpu_cql_parity.py, and runs the K2 critic forward in 31.6 us against
# 46.8).  Read at each launch, so set it before an update graph is captured.
CRITIC_GEMM = os.environ.get("D3A_CRITIC_GEMM", "x6")


def set_critic_gemm(mode: str) -> None:
    global CRITIC_GEMM
    if mode not in ("fp32", "x6"):
        raise ValueError(f"critic GEMM mode must be fp32 or x6, got {mode!r}")
    CRITIC_GEMM = mode


def set_sbf16(terms: int) -> None:
    global SBF16_TERMS
    assert terms in (0, 3, 6)
    SBF16_TERMS = terms


def linear_bwd_x(dy: int, ldy: int, sdyb: int, W: int, dx: int, ldx: int, sdxb: int, C_: int,
                 R: int, n_in: int, n_out: int, mask: Optional[int] = None,
                 ldm: int = 0, smb: int = 0, agen: Optional[C.Structure] = None,
                 wnext: Optional[C.Structure] = None, sbf16: int = 0) -> None:
    """dx[c] = (dy[c] @ W[c]) * [mask[c] > 0]; with ``agen`` dy is generated
    from that single-output head (d3a_gemm_desc.agen) and not read; with
    ``wnext`` (a GemmWnext) dx is not written but the layer below's weight /
    bias gradient partials per 128-row tile (d3a_gemm_desc.wnext).  ``sbf16``
    (3 / 6): this GEMM on d3a_gemm_sbf16 at any row count (else SBF16_TERMS
    from SBF16_MIN_ROWS rows)."""
    if wnext is not None:
        if agen is not None and agen.dW:
            agen = type(agen).from_buffer_copy(agen)
            agen.dW = agen.db = None
        gemm(None if agen is not None else dy, W, None, R, n_in, n_out, batch=C_,
             sA=(0 if agen is not None else sdyb, n_out if agen is not None else ldy, 1),
             sB=(n_out * n_in, n_in, 1), sC=(0, 0, 0), mask=mask, sM=(smb, ldm, 1),
             agen=agen, wnext=wnext)
        return
    if agen is not None:
        if agen.dW:  # the head's weight gradients come from the dW launch only
            agen = type(agen).from_buffer_copy(agen)
            agen.dW = agen.db = None
        gemm(None, W, dx, R, n_in, n_out, batch=C_, sA=(0, n_out, 1),
             sB=(n_out * n_in, n_in, 1), sC=(sdxb, ldx, 1), mask=mask, sM=(smb, ldm, 1),
             agen=agen)
        return
    terms = sbf16 or (SBF16_TERMS if R * C_ >= SBF16_MIN_ROWS else 0)
    if terms and n_out % 4 == 0 and n_in % 4 == 0 \
            and ldy % 4 == 0 and dy % 16 == 0 and W % 16 == 0:
        d = N.GemmDesc()
        d.A, d.B, d.C, d.mask = dy, W, dx, mask
        d.M, d.N, d.K, d.batch = R, n_in, n_out, C_
        d.sAb, d.sAm, d.sAk = sdyb, ldy, 1
        d.sBb, d.sBk, d.sBn = n_out * n_in, n_in, 1
        d.sCb, d.sCm, d.sCn = sdxb, ldx, 1
        d.sMb, d.sMm, d.sMn = smb, ldm, 1
        d.splits, d.alpha, d.variant, d.batch2 = 1, 1.0, -1, 1
        N.check(N.lib().d3a_gemm_sbf16(C.byref(d), terms, _stream()), "d3a_gemm_sbf16")
        return
    gemm(dy, W, dx, R, n_in, n_out, batch=C_, sA=(sdyb, ldy, 1), sB=(n_out * n_in, n_in, 1),
         sC=(sdxb, ldx, 1), mask=mask, sM=(smb, ldm, 1))


def linear_bwd_w(dy: int, ldy: int, sdyb: int, x: int, ldx: int, sxb: int, dW: int, C_: int,
                 R: int, n_in: int, n_out: int, splits: int, db: Optional[int] = None,
                 variant: int = -1, agen: Optional[C.Structure] = None,
                 sbf16: int = 0) -> None:
    """dW[s][c] = sum_{r in split s} dy[c][r]^T x[c][r]  -> partials [splits][C][out][in];
    if ``db`` is given, also the bias-gradient partials db[s][c][out] = sum_r dy[c][r].
    With ``agen`` dy is generated from that single-output head, whose weight /
    bias gradient partials the same launch writes (d3a_gemm_desc.agen)."""
    if agen is not None:
        gemm(None, x, dW, n_out, n_in, R, batch=C_, sA=(0, 1, n_out), sB=(sxb, ldx, 1),
             sC=(n_out * n_in, n_in, 1), splits=splits, sCs=C_ * n_out * n_in,
             rowsum=db, sR=(n_out, C_ * n_out), variant=variant, agen=agen)
        return
    terms = sbf16 or (SBF16_TERMS if SBF16_W and R * C_ >= SBF16_MIN_ROWS else 0)
    if terms and n_out >= 128 and n_in >= 128 \
            and n_out % 4 == 0 and n_in % 4 == 0 and ldy % 4 == 0 and ldx % 4 == 0 \
            and dy % 16 == 0 and x % 16 == 0:
        d = N.GemmDesc()
        d.A, d.B, d.C = dy, x, dW
        d.rowsum = db
        d.sRb, d.sRs = n_out, C_ * n_out
        d.M, d.N, d.K, d.batch = n_out, n_in, R, C_
        d.sAb, d.sAm, d.sAk = sdyb, 1, ldy
        d.sBb, d.sBk, d.sBn = sxb, ldx, 1
        d.sCb, d.sCm, d.sCn = n_out * n_in, n_in, 1
        d.splits, d.sCs = splits, C_ * n_out * n_in
        d.alpha, d.variant, d.batch2 = 1.0, -1, 1
        N.check(N.lib().d3a_gemm_sbf16(C.byref(d), terms, _stream()), "d3a_gemm_sbf16")
        return
    gemm(dy, x, dW, n_out, n_in, R, batch=C_, sA=(sdyb, 1, ldy), sB=(sxb, ldx, 1),
         sC=(n_out * n_in, n_in, 1), splits=splits, sCs=C_ * n_out * n_in,
         rowsum=db, sR=(n_out, C_ * n_out), variant=variant)


# D3A_OP_REPLAY=0: replay the update graphs with CUDAGraph.replay instead of
# the update-step custom op (A/B of the two host paths)
_OP_REPLAY = os.environ.get("D3A_OP_REPLAY", "1") == "1"


def update_state(*objs) -> list:
    """The device tensors an update step mutates, for the update-step op's
    ``Tensor(a!)[] state``: every GPU tensor attribute of the given objects
    (an Impl and its workspace), the flat buffers of their ParamStores and
    OptimStates, one tensor per storage."""
    from .nets import OptimState, ParamStore
    out, seen = [], set()

    def add(t):
        if torch.is_tensor(t) and t.is_cuda:
            k = t.untyped_storage().data_ptr()
            if k not in seen:
                seen.add(k)
                out.append(t)
    for o in objs:
        for v in vars(o).values():
            if isinstance(v, ParamStore):
                add(v.data)
            elif isinstance(v, OptimState):
                add(v.exp_avg.data)
                add(v.exp_avg_sq.data)
                add(v.step)
            else:
                add(v)
    return out


def replay_update(g, state: list, cql: bool = False) -> None:
    """Launch a captured update pipeline through the PyTorch custom op
    (``torch.ops.d3rlpy_amd.cql_update_step`` / ``update_step``,
    csrc/torch_ops.cpp): the graph's exec handle on the current stream, the
    mutated tensors declared.  No fallback: the op library must be built."""
    if not _OP_REPLAY:
        g.replay()  # (A/B: torch.cuda.CUDAGraph.replay)
        return
    from . import torch_ops
    ns = torch_ops.load()
    (ns.cql_update_step if cql else ns.update_step)(g.raw_cuda_graph_exec(), state)


@contextlib.contextmanager
def graph_capture(g):
    """``torch.cuda.graph(g)`` with Python's cyclic garbage collector paused for
    the capture: a collection triggered by an allocation inside the capture runs
    the finalizers of unreachable objects from earlier work (freeing device
    memory, destroying another HIP graph), which is not legal while the stream
    is capturing -- measured as an abort in the GPU suite.  (torch.cuda.graph
    already collects once before the capture starts.)"""
    was = gc.isenabled()
    gc.disable()
    try:
        with torch.cuda.graph(g):
            yield
    finally:
        if was:
            gc.enable()
