"""Forward / backward schedules of a ReLU MLP ensemble on the HIP kernels.

The reference evaluates each critic of an ensemble sequentially through
autograd (ensemble_q_function.py:95-105, 167-170); here the C members of an
ensemble are one batched launch per layer, and backward is written out by
hand (no autograd):

  forward   h_l = relu(h_{l-1} W_l^T + b_l)  (last layer linear, or a row-dot
            when it has a single output)
  backward  head:  dW = dy^T h, db = sum dy, dz = dy W * [h > 0]
            trunk: dW_l = dz_l^T h_{l-1}, db_l = sum dz_l,
                   dz_{l-1} = dz_l W_l * [h_{l-1} > 0]
            input: dx = dz_0 W_0 (only when requested)

Weight gradients are written as split-K partial sums (summed in a fixed
order inside the Adam kernel), so every reduction is deterministic.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import List, Optional

import torch

from . import _native as N
from . import ops
from .nets import EnsembleMLP, GradSpace, ParamStore


def n_splits(rows: int, min_rows: int = 32, max_splits: int = 32) -> int:
    """Split-K slices for weight gradients: >= min_rows rows per slice, at most
    max_splits slices (the Adam kernel sums the slices in a fixed order)."""
    return max(1, min(max_splits, rows // min_rows))


@dataclass
class Acts:
    """Activation buffers of one forward pass: h[l] is [C][R][H_l] (trunk);
    ``hmask`` (optional, ``with_mask``): the last hidden layer's ReLU mask as
    bits, int32 [C][R][H / 32], written by the split-bf16 x6 Q forward for the
    kept rows and read by its backward (d3a_mlp_fwd_desc.hmask / d3a_q2_bwd_
    desc.m2)."""

    h: List[torch.Tensor]
    out: torch.Tensor  # [C][R] (single output) or [C][R][out]
    R: int
    hmask: Optional[torch.Tensor] = None
    # first row of the mask image the last forward wrote (None: not written;
    # the backward then builds the mask from h2)
    hmask_from: Optional[int] = None
    # one past the last row it wrote (the forward's r1): a backward uses the
    # image only for rows inside [hmask_from, hmask_to)
    hmask_to: Optional[int] = None
    # the same mask transposed ([C][ceil(R / 32)][256] int32, d3a_mlp_fwd_desc.
    # hmaskT), written with hmask where the forward's rows start on a 32-row
    # group; read by the slice backward (d3a_q2_bwd_desc.m2t)
    hmaskT: Optional[torch.Tensor] = None
    hmaskT_from: Optional[int] = None
    # the slice backward reads no h2: the x6 forward then keeps only h[0] and
    # the mask bits (set by the owner of the backward space, BackwardSpace.slice)
    no_last_h: bool = False

    @staticmethod
    def alloc(net: EnsembleMLP, R: int, device, dtype=torch.float32,
              with_mask: bool = False) -> "Acts":
        """``dtype`` bfloat16: kept activations for the bf16 critic kernels
        (d3a_q2_fwd_bf16 / d3a_q2_bwd_bf16 are then selected by forward /
        backward); outputs stay fp32."""
        hs = [torch.zeros(net.C, R, net.sizes[l + 1], device=device, dtype=dtype)
              for l in range(net.n_layers - 1)]
        out_dim = net.sizes[-1]
        out = torch.zeros((net.C, R) if out_dim == 1 else (net.C, R, out_dim), device=device)
        hm = hmt = None
        if with_mask and net.n_layers >= 2 and net.sizes[-2] % 32 == 0:
            hm = torch.zeros(net.C, R, net.sizes[-2] // 32, device=device, dtype=torch.int32)
            if net.sizes[-2] == 256:
                hmt = torch.zeros(net.C, (R + 31) // 32, 256, device=device, dtype=torch.int32)
        return Acts(hs, out, R, hm, hmaskT=hmt)

    def relu_decisions(self, c: int, r0: int, r1: int) -> List[torch.Tensor]:
        """[h_l > 0] of member c, rows [r0, r1), for every hidden layer: from
        the kept activations, the last one from the mask bits when it is not
        kept (no_last_h)."""
        out = [(h[c, r0:r1] > 0) for h in self.h]
        if self.no_last_h:
            assert (self.hmask is not None and self.hmask_from is not None
                    and self.hmask_from <= r0 and r1 <= self.hmask_to)
            w = self.hmask[c, r0:r1].to(torch.int64)
            bits = (w.unsqueeze(-1) >> torch.arange(32, device=w.device)) & 1
            out[-1] = bits.reshape(r1 - r0, -1).bool()
        return out


# one-launch forward (d3a_mlp_fwd) unless D3A_FUSED_MLP=0 (per-layer GEMMs,
# kept for A/B measurement and as the path for shapes the fused kernel rejects)
_FUSED = os.environ.get("D3A_FUSED_MLP", "1") != "0"


# below this many rows x members the per-layer GEMMs win: a fused workgroup
# computes every output column of its rows on one CU, so small passes leave
# most CUs idle (measured: 100-512-row passes 10-60 % slower fused, the
# 2 x 15616-row critic pass 12 % faster: 72 vs 82 us)
FUSED_MIN_ROWS = int(os.environ.get("D3A_FUSED_MIN_ROWS", "4096"))
# the fused backward-data kernel is opt-in: its weight operand is read across
# rows (four loads per lane per 8 k) and it measured 67 us against 52 us for
# the per-layer head backward + input-gradient GEMM on the K2 critic pass
_FUSED_BWD = os.environ.get("D3A_FUSED_BWD", "0") == "1"
# head backward generated inside the trunk GEMMs (see backward); measured on
# the K2 critic backward (7,936 rows x 2 members), off for small passes where
# the register-direct GEMM + d3a_head1_bwd is faster
_HEAD_GEN = os.environ.get("D3A_HEAD_GEN", "1") == "1"
_HEAD_GEN_MIN_ROWS = 4096
# the first layer's weight gradient formed in the epilogue of the second
# layer's input-gradient GEMM (d3a_gemm_desc.wnext): same size gate
_FIRST_LAYER_EPI = os.environ.get("D3A_W0_EPI", "1") == "1"
# rows per fused workgroup (32 or 64; 0 = the library's choice)
_FUSED_BM = int(os.environ.get("D3A_FUSED_BM", "0"))
# the whole weight-gradient backward of a [n_in -> 256 -> 256 -> 1] Q ensemble
# in one launch (d3a_q2_bwd) for large critic passes (the K2 / K4 CQL critic:
# 7,936 rows x 2 members); D3A_Q2_BWD=0 keeps the per-layer GEMM path
_Q2 = os.environ.get("D3A_Q2_BWD", "1") == "1"
# input rows built inside the x6 forwards (mlp.forward xgen); D3A_XGEN=0 keeps
# the separate d3a_bcq_rows launch (A/B)
_XGEN = os.environ.get("D3A_XGEN", "1") == "1"
# the x6 critic backward reads the forward's bf16 mask image of h2 instead of
# building it from h2 (D3A_MASK_IMAGE=0: build it, A/B)
_MASK_IMAGE = os.environ.get("D3A_MASK_IMAGE", "1") == "1"
# the SAC / CQL actor head in the policy trunk backward's prologue
# (d3a_q2_bwd_actor_head: one launch fewer per actor update)
# -- off by default: measured slower on K2 (the fused launch 32.9 us against
# 8.6 + 10.6 for the pair; every quarter workgroup re-forms its rows' dz2 inside
# the trunk's row pipeline), kept bitwise-tested for the record
_HEAD_IN_TRUNK = os.environ.get("D3A_HEAD_IN_TRUNK", "0") == "1"


def q2_shape(net: EnsembleMLP) -> bool:
    """[n_in <= 48, 256, 256, 1]: the shape of the q2 critic kernels."""
    s = net.sizes
    return net.n_layers == 3 and s[1] == 256 and s[2] == 256 and s[3] == 1 and s[0] <= 48


def x6_narrow_shape(net: EnsembleMLP) -> bool:
    """[n_in <= 48, 256, 256, 1 < n_out <= 8]: d3a_q2_fwd_x6's narrow-head
    instantiation (BCQ's VAE decoder / residual policy over the target rows)."""
    s = net.sizes
    return (net.n_layers == 3 and s[1] == 256 and s[2] == 256 and 1 < s[3] <= 8
            and s[0] <= 48)


def small_bwd_ok(net: EnsembleMLP, rows: int) -> bool:
    """[n_in <= 64, 256, 256, n_out <= 256] over at most 2,048 rows: the shape
    of d3a_mlp_bwd_small (one launch for the whole backward)."""
    s = net.sizes
    return (_SMALL_BWD and net.n_layers == 3 and s[1] == 256 and s[2] == 256 and s[0] <= 64
            and s[3] <= 256 and rows <= 2048)


# the two-launch small-batch backward (d3a_mlp_bwd_small) replaces the four or
# five per-layer GEMM launches of each K3 network's backward.  Its first
# version (VALU fma chains, 33-43 us) lost to them (K3 1,673 against 1,824
# steps/s, profiles/r05_bcq_timeline_smallbwd.txt); on the fp32 matrix cores it
# wins (K3 2,047 -> 2,134).  D3A_SMALL_BWD=0 keeps the per-layer GEMMs (A/B).
_SMALL_BWD = os.environ.get("D3A_SMALL_BWD", "1") == "1"
# the small-pass forward also takes heads of 65-256 outputs (as an MFMA layer;
# BCQ's QR critics over their batch rows); D3A_SMALL_WIDE=0 keeps those on the
# per-layer GEMMs (A/B)
_SMALL_WIDE = os.environ.get("D3A_SMALL_WIDE", "1") == "1"


# the x6 Q forward streams W0 / W1 as split-bf16 operand images formed once
# per step by an earlier launch (d3a_mlp_fwd_desc.wp; in the CQL step the
# sampler's launch forms them) instead of splitting the fp32 weights in every
# workgroup; D3A_X6_PRESPLIT=0 keeps the in-kernel split (A/B)
_PRESPLIT = os.environ.get("D3A_X6_PRESPLIT", "1") == "1"


def presplit_ok(net: EnsembleMLP) -> bool:
    """The shape and arithmetic of the pre-split x6 Q forward: [n_in <= 32,
    256, 256, 1] critics on the fp32-accurate split-bf16 kernels."""
    return (_PRESPLIT and q2_shape(net) and net.sizes[0] <= 32 and ops.CRITIC_GEMM == "x6"
            and ops.CRITIC_PRECISION not in ("bf16", "bf16h"))


# d3a_mlp_fwd_x6 streaming pre-split images (D3A_X6_WIDE_PRESPLIT=1): off --
# measured slower at the reproduction config (forward 40.5 against 34.9 us in
# the step: the three 16-byte part loads a k step, three steps ahead, leave the
# products waiting on L2 where the fp32 words' split filled the gaps)
_WIDE_PRESPLIT = os.environ.get("D3A_X6_WIDE_PRESPLIT", "0") == "1"


def wide_presplit_ok(net: EnsembleMLP) -> bool:
    """d3a_mlp_fwd_x6's pre-split stream images apply: n_in <= 32 and
    [.., 256, 256, 256, 1] or [.., 256, 256, 1 < n_out <= 256] (x6 GEMMs)."""
    s = net.sizes
    return (_PRESPLIT and _WIDE_PRESPLIT and ops.CRITIC_GEMM == "x6" and ops.CRITIC_PRECISION not in ("bf16", "bf16h")
            and s[0] <= 32 and ((x6_deep3_shape(net) and s[-1] == 1) or x6_wide_shape(net)))


class WeightImages:
    """Split-bf16 operand images (d3a_x6_split's layout) of two of a critic's
    weight matrices, one pair per parameter store (e.g. the online critics
    and their targets): a q2 critic's W0 and W1 (the pre-split x6 Q forward),
    or the 256-wide stream matrices of d3a_mlp_fwd_x6 -- W1 and W2 of a
    three-hidden-layer critic, W1 and the wide head of a two-layer one
    (``streams``).  ``jobs()`` is the d3a_x6_split descriptor that forms them
    from the stores' current weights, ``wparts(i, j)`` the images of stores i
    (main pass) and j (aux pass) for ``forward(..., wparts=...)``.  The images
    are valid only after the jobs ran on the weights the forward reads."""

    def __init__(self, net: EnsembleMLP, stores, device, streams: bool = False):
        assert wide_presplit_ok(net) if streams else presplit_ok(net)
        self.net = net
        self.layers = (1, 2) if streams else (0, 1)
        self.kpad = [(net.sizes[l] + 15) // 16 * 16 for l in self.layers]
        self.xl = (net.sizes[0] + 15) // 16 * 16  # (W0's padded k)
        C = net.C
        self.imgs = [(st,) + tuple(torch.zeros(C * net.sizes[l + 1] * kp * 3, dtype=torch.bfloat16,
                                               device=device)
                                   for l, kp in zip(self.layers, self.kpad))
                     for st in stores]

    def jobs(self) -> "N.X6SplitDesc":
        net, C = self.net, self.net.C
        d = N.X6SplitDesc()
        i = 0
        for st, ia, ib in self.imgs:
            for l, img, kpad in zip(self.layers, (ia, ib), self.kpad):
                j = d.job[i]
                j.src, j.dst = net.W(l, st), img.data_ptr()
                j.rows, j.k, j.kpad = C * net.sizes[l + 1], net.sizes[l], kpad
                i += 1
        d.n_jobs = i
        return d

    def wparts(self, main: int, aux: Optional[int] = None) -> tuple:
        m = self.imgs[main]
        a = self.imgs[aux] if aux is not None else None
        return (m[1].data_ptr(), m[2].data_ptr(),
                a[1].data_ptr() if a else None, a[2].data_ptr() if a else None)


def x6_deep_shape(net: EnsembleMLP) -> bool:
    """>= 3 hidden layers, all 256 wide (the CQL reproduction critic, [obs +
    act, 256, 256, 256, 1]: reproductions/offline/cql.py:21-37): under
    CRITIC_GEMM "x6" its large backward GEMMs (>= 128 wide both ways) run on
    d3a_gemm_sbf16 with six-product split-bf16 operands (fp32-accurate)."""
    return net.n_layers >= 4 and all(h == 256 for h in net.sizes[1:-1])


# D3A_X6_DEEP=0 keeps the deep critics' backward on the fp32 GEMMs (A/B);
# the forward stays on the one-launch fp32 kernel with the target aux pass
# unless D3A_X6_DEEP_FWD=1 (per-layer split-bf16 launches: measured slower at
# the reproduction config, 60.7 + 21.6 us against 56.5 us, round 5)
_X6_DEEP = os.environ.get("D3A_X6_DEEP", "1") == "1"
_X6_DEEP_FWD = os.environ.get("D3A_X6_DEEP_FWD", "0") == "1"
# the three-hidden-layer critic's forward (+ its target aux pass) in one
# d3a_mlp_fwd_x6 launch (round 6; D3A_X6_DEEP3=0: the fp32 fused kernel)
_X6_DEEP3 = os.environ.get("D3A_X6_DEEP3", "1") == "1"
# its backward's input-gradient chain in one d3a_mlp_bwd_chain launch (round 6)
_X6_BWD_CHAIN = os.environ.get("D3A_X6_BWD_CHAIN", "1") == "1"


def x6_deep3_shape(net: EnsembleMLP) -> bool:
    """[n_in <= 64, 256, 256, 256, n_out <= 256]: d3a_mlp_fwd_x6's three-layer
    instantiation (the CQL reproduction critic)."""
    s = net.sizes
    return net.n_layers == 4 and s[1] == s[2] == s[3] == 256 and s[0] <= 64 and 1 <= s[4] <= 256


def x6_wide_shape(net: EnsembleMLP) -> bool:
    """[n_in <= 64, 256, 256, 1 < n_out <= 256] (not a narrow shape):
    d3a_mlp_fwd_x6's shape."""
    s = net.sizes
    return (net.n_layers == 3 and s[1] == 256 and s[2] == 256 and 1 < s[3] <= 256
            and s[0] <= 64 and not x6_narrow_shape(net))


def q2_ok(net: EnsembleMLP, rows: int) -> bool:
    """d3a_q2_bwd applies: two hidden layers of 256, one output, <= 48 inputs,
    a large pass (per-layer GEMMs win on the 100-512-row passes)."""
    s = net.sizes
    return (_Q2 and not _FUSED_BWD and not ops.SBF16_TERMS and net.n_layers == 3
            and s[1] == 256 and s[2] == 256 and s[3] == 1 and s[0] <= 48
            and rows * net.C >= _HEAD_GEN_MIN_ROWS)


# trunk backward of a [n_in <= 48, 256, 256, J] net whose head a caller's
# kernel differentiated (the SAC / CQL actor phase's policy, d3a_sac_actor_head
# writes dz2 and the head partials): d3a_q2_bwd with dz2 given and 32-row
# partials -- one launch instead of the paired layer-2 launch + the layer-1
# weight-gradient launch
_Q2P = os.environ.get("D3A_Q2P", "1") == "1"


# the critic weight-gradient backward on the slice kernel (csrc/q2_x6_bwd2.hip:
# transposed mask bits, no kept h2, P = d3a_q2_bwd_x6t_splits row blocks);
# D3A_BWD_SLICE=0 keeps the 256-row-block kernel (A/B)
_SLICE = os.environ.get("D3A_BWD_SLICE", "1") == "1"


def slice_ok(net: EnsembleMLP, rows: int, r0: int) -> bool:
    """The slice backward applies to a q2 backward space of ``rows`` rows read
    from row ``r0`` of the x6 forward's activations: x6 critic GEMMs with
    fp32 kept activations and both on 32-row groups."""
    # (the bf16 line's x1 forward writes the same mask bits: round 6)
    return (_SLICE and q2_ok(net, rows) and ops.CRITIC_GEMM == "x6"
            and ops.CRITIC_PRECISION != "bf16h" and rows % 32 == 0 and r0 % 32 == 0)


def q2p_ok(net: EnsembleMLP, rows: int) -> bool:
    s = net.sizes
    return (_Q2P and not _FUSED_BWD and not ops.SBF16_TERMS and net.n_layers == 3
            and s[1] == 256 and s[2] == 256 and s[0] <= 48 and 0 < rows <= 4096)


# small passes (policy over [obs; next_obs], actor / target passes of a few
# hundred rows): 16-row workgroups, the whole MLP in one launch
# (d3a_mlp_fwd block_rows 16, csrc/mlp_small.hip)
_SMALL = os.environ.get("D3A_MLP_SMALL", "1") == "1"
SMALL_MAX_ROWS = 2048
# few-hundred-row passes of [n_in, 256, 256, n_out <= 16] MLPs whose consumer
# sums head parts (the CQL / SAC policy over [obs; next_obs]): the second
# hidden layer split over four times the workgroups (d3a_mlp_fwd parts)
_PARTS = os.environ.get("D3A_MLP_PARTS", "1") == "1"


def small_ok(net: EnsembleMLP, rows: int) -> bool:
    hidden = net.sizes[1:-1]
    # (a head wider than 64 runs as an MFMA layer: two hidden layers only)
    return (_SMALL and 1 <= len(hidden) <= N.MLP_MAX_HIDDEN and set(hidden) == {256}
            and net.sizes[0] <= 256 and rows * net.C <= SMALL_MAX_ROWS
            and (net.sizes[-1] <= 64 or (_SMALL_WIDE and net.sizes[-1] <= 256 and len(hidden) == 2)))


def parts_ok(net: EnsembleMLP) -> bool:
    """Shape of d3a_mlp_fwd's parts path (two hidden layers of 256, the
    second split into D3A_MLP_PARTS unit parts; n_in <= 64, n_out <= 32)."""
    return (_PARTS and list(net.sizes[1:-1]) == [256, 256] and net.sizes[0] <= 64
            and net.sizes[-1] <= 32)


def fused_ok(net: EnsembleMLP, rows: Optional[int] = None, backward: bool = False) -> bool:
    hidden = net.sizes[1:-1]
    return (_FUSED and 1 <= len(hidden) <= N.MLP_MAX_HIDDEN and len(set(hidden)) == 1
            and hidden[0] % 32 == 0 and 32 <= hidden[0] <= 256 and net.sizes[0] <= 256
            and net.sizes[-1] <= (64 if backward else 1024)
            and (rows is None or rows * net.C >= FUSED_MIN_ROWS))


def forward(net: EnsembleMLP, store: ParamStore, x: int, x_shared: bool, ldx: int, acts: Acts,
            r0: int = 0, r1: Optional[int] = None, sxb: Optional[int] = None,
            members: Optional[int] = None, keep_h: bool = True,
            h_from: Optional[int] = None, aux: Optional[tuple] = None,
            skip_head: bool = False, out_parts: Optional[torch.Tensor] = None,
            row_mean: Optional[torch.Tensor] = None, xgen=None, xgen_keep: bool = False,
            wparts: Optional[tuple] = None, presplit=None, philox=None) -> bool:
    """Forward rows [r0, r1) of x (row stride ldx) through the ensemble
    (through its first ``members`` members only, when given).  ``keep_h``:
    store the hidden activations in ``acts.h`` (needed by a backward pass),
    for rows >= ``h_from`` only when given (the fused kernel skips the rest;
    the per-layer path stores every row).

    ``aux = (store2, x2, ldx2, acts2)``: a second, independent forward of the
    same network with the parameters of ``store2`` (same layout, e.g. the
    targets) over all acts2.R rows of x2 (shared by the members), no
    activations kept.  On the fused path it rides in the same launch (its
    workgroups use the CUs the main pass leaves idle); on the per-layer path
    each layer's launch carries it as a second batch dimension when its shape
    equals the main pass's (acts2.R == acts.R rows, same ldx); otherwise it is
    a separate forward.

    ``xgen`` (a d3a_bcq_rows descriptor whose x is this pass's input ``x``):
    the input rows are that builder's; the x6 kernels form them while staging
    (d3a_mlp_fwd_desc.xg_*), any other path launches d3a_bcq_rows first.
    ``xgen_keep``: the rows (and the builder's e_out) must also be written, as
    d3a_bcq_rows writes them, for a later reader; the parts path forms and
    writes them in-kernel (xg_xout / xg_eout), any other path launches
    d3a_bcq_rows first.

    ``wparts`` (WeightImages.wparts): where the launch is the pre-split x6 Q
    forward, its W0 / W1 (and the aux pass's) are read from those images
    (formed from the current weights by an earlier launch of the step).

    ``presplit`` (an X6SplitDesc, with ``out_parts``): the parts-path launch
    also runs those d3a_x6_split jobs on extra workgroups; ``philox`` (a
    PhiloxJob, with ``out_parts``) likewise a d3a_philox_fill.

    ``row_mean`` ([C][R] fp32): also the mean of each row's outputs, where the
    launch is d3a_mlp_fwd_x6 (its epilogue forms it); returns whether it was
    written (False: the caller forms it).

    ``out_parts`` ([D3A_MLP_PARTS][C][R][n_out], ``parts_ok`` shapes): the
    head is written there as partial sums over the second hidden layer's unit
    parts (d3a_mlp_fwd_desc.parts; consumers sum them in order), not to
    acts.out."""
    R = acts.R
    r1 = R if r1 is None else r1
    n = r1 - r0
    if acts.hmask is not None:
        acts.hmask_from = acts.hmask_to = None  # set below where this forward writes the mask image
        acts.hmaskT_from = None
    if n <= 0:
        return False
    C = net.C if members is None else members
    sizes = net.sizes
    bf16 = bool(acts.h) and acts.h[0].dtype == torch.bfloat16
    if bf16 and not (q2_shape(net) and keep_h and members is None and not skip_head):
        raise NotImplementedError("bf16 activations: [n_in <= 48, 256, 256, 1] critics, "
                                  "all members, activations kept")
    small = not bf16 and not skip_head and small_ok(net, n * C // net.C)
    # deep 256-wide critics under CRITIC_GEMM "x6": per-layer launches with the
    # 256 x 256 layers on the split-bf16 GEMM (six products, fp32-accurate)
    deep6 = (not bf16 and out_parts is None and ops.CRITIC_GEMM == "x6" and _X6_DEEP
             and _X6_DEEP_FWD and x6_deep_shape(net) and n * C >= 8192 and xgen is None)
    assert philox is None or out_parts is not None, "a philox job rides on the parts path only"
    if out_parts is not None:
        assert parts_ok(net) and not bf16 and not skip_head and aux is None
        assert tuple(out_parts.shape) == (N.MLP_PARTS, C, R, sizes[-1])
        small = True
    if not deep6 and (bf16 or small or fused_ok(net, n * C // net.C)):
        d = N.MlpFwdDesc()
        d.block_rows = 16 if small else _FUSED_BM
        d.x, d.ldx = x, ldx
        d.sxb = (0 if x_shared else R * ldx) if sxb is None else sxb
        L = net.n_layers
        d.n_in, d.n_hidden, d.H, d.n_out = sizes[0], L - 1, sizes[1], sizes[-1]
        for l in range(L):
            d.W[l], d.b[l] = net.W(l, store), net.b(l, store)
            d.sW[l], d.sb[l] = sizes[l + 1] * sizes[l], sizes[l + 1]
        for l in range(L - 1):
            d.h[l] = acts.h[l].data_ptr() if keep_h else None
        d.sh = R * sizes[1]
        d.out = acts.out.data_ptr()
        d.sout, d.ldout = R * sizes[-1], sizes[-1]
        if out_parts is not None:
            d.out, d.parts, d.s_part = out_parts.data_ptr(), N.MLP_PARTS, C * R * sizes[-1]
            if presplit is not None:
                d.presplit = presplit
            if philox is not None:
                d.philox = philox
        d.r0, d.rows, d.C = r0, n, C
        d.h_from = r0 if h_from is None else max(r0, h_from)
        if aux is not None and members is None:
            ast, ax, aldx, aacts = aux
            assert ast.size == store.size and list(ast.specs) == list(store.specs)
            d.aux_x, d.aux_ldx, d.aux_sxb = ax, aldx, 0
            d.aux_wdelta = (ast.data.data_ptr() - store.data.data_ptr()) // 4
            d.aux_out, d.aux_sout, d.aux_rows = aacts.out.data_ptr(), aacts.R * sizes[-1], aacts.R
            aux = None
        entry = "d3a_q2_fwd_bf16" if bf16 else "d3a_mlp_fwd"
        big = (not bf16 and not small and out_parts is None
               and (n + (d.aux_rows if d.aux_rows else 0)) * C >= 8192)
        if big and q2_shape(net) and ops.CRITIC_PRECISION == "bf16":
            entry = "d3a_q2_fwd_x1"  # the bf16 line: one bf16 part per operand
        elif big and (q2_shape(net) or x6_narrow_shape(net)) and ops.CRITIC_GEMM == "x6":
            entry = "d3a_q2_fwd_x6"  # fp32-accurate split-bf16 (Q head or <= 8 outputs)
        elif (not bf16 and not small and ops.CRITIC_GEMM == "x6" and x6_wide_shape(net)
              and out_parts is None and not d.aux_rows and n * C >= 8192):
            entry = "d3a_mlp_fwd_x6"  # wide head (e.g. BCQ's target QR critics)
        elif big and _X6_DEEP3 and ops.CRITIC_GEMM == "x6" and x6_deep3_shape(net) \
                and members is None and (xgen is None or not d.aux_rows):
            entry = "d3a_mlp_fwd_x6"  # three hidden layers (+ the aux pass, same launch)
        if xgen is not None:
            # the builder rides in the x6 forwards and the small-pass ones
            # (block_rows 16); a builder with a side output (e_out) keeps its
            # own launch
            xg_ok = (entry in ("d3a_q2_fwd_x6", "d3a_mlp_fwd_x6")
                     or (entry == "d3a_mlp_fwd" and d.block_rows == 16))
            # (writing the rows out: the parts path only)
            parts_path = entry == "d3a_mlp_fwd" and out_parts is not None
            outs = xgen_keep or bool(xgen.e_out)
            if (_XGEN and xg_ok and not d.aux_rows and r0 == 0 and (not outs or (xgen_keep and parts_path))):
                # (d3a_bcq_rows mode 0, the copy, is the builder's mode 5)
                d.xg_mode = xgen.mode if xgen.mode != 0 else 5
                d.xg_D, d.xg_rep, d.xg_E = xgen.D, xgen.rep, xgen.E
                d.xg_obs, d.xg_a, d.xg_lda = xgen.obs, xgen.a, xgen.lda
                d.xg_base, d.xg_clip, d.xg_scale = xgen.base, xgen.clip, xgen.scale
                if xgen.a_parts > 1:
                    d.xg_a_parts, d.xg_s_apart = xgen.a_parts, xgen.s_a_part
                if xgen_keep:
                    d.xg_xout, d.xg_ldxo, d.xg_eout = xgen.x, xgen.ldx, xgen.e_out
            else:
                ops.call_desc("d3a_bcq_rows", xgen)
            xgen = None
        if acts.hmask is not None:
            if (entry in ("d3a_q2_fwd_x6", "d3a_q2_fwd_x1") and keep_h and members is None
                    and sizes[-1] == 1):
                d.hmask, d.s_hmask = acts.hmask.data_ptr(), R * (sizes[-2] // 32)
                acts.hmask_from, acts.hmask_to = d.h_from, r1
                if acts.hmaskT is not None and r0 % 32 == 0:
                    d.hmaskT, d.s_hmaskT = acts.hmaskT.data_ptr(), acts.hmaskT[0].numel()
                    acts.hmaskT_from = d.h_from
                    if acts.no_last_h:
                        d.h[L - 2] = None  # the slice backward reads no h2
            elif acts.no_last_h:
                raise RuntimeError("Acts.no_last_h: the forward must be the x6 Q forward "
                                   "that writes the mask bits")
        if (wparts is not None and entry == "d3a_q2_fwd_x6" and presplit_ok(net)
                and members is None and d.xg_mode == 0):
            d.wp[0], d.wp[1] = wparts[0], wparts[1]
            if d.aux_rows:
                assert wparts[2] is not None and wparts[3] is not None
                d.aux_wp[0], d.aux_wp[1] = wparts[2], wparts[3]
        elif wparts is not None and entry == "d3a_mlp_fwd_x6" and wide_presplit_ok(net) \
                and members is None:
            d.wp[0], d.wp[1] = wparts[0], wparts[1]  # the stream matrices' images
            if d.aux_rows:
                assert wparts[2] is not None and wparts[3] is not None
                d.aux_wp[0], d.aux_wp[1] = wparts[2], wparts[3]
        means = row_mean is not None and entry == "d3a_mlp_fwd_x6"
        if means:
            assert tuple(row_mean.shape) == (C, R) and row_mean.dtype == torch.float32
            d.row_mean, d.s_mean = row_mean.data_ptr(), R
        ops.call_desc(entry, d)
        if aux is not None:
            forward(net, aux[0], aux[1], True, aux[2], aux[3], keep_h=False)
        return means
    if xgen is not None:
        ops.call_desc("d3a_bcq_rows", xgen)  # the per-layer path reads built rows
    L = net.n_layers
    inp, ld_in = x + 4 * r0 * ldx, ldx
    sxb_ = (0 if x_shared else R * ldx) if sxb is None else sxb
    # the aux pass rides in the same launches (second batch dimension, element
    # offsets from the main pass's operands) when it has the main pass's shape
    pair = aux is not None and members is None and x_shared and sxb is None and r0 == 0 \
        and n == R and aux[3].R == R and aux[2] == ldx and not deep6
    if pair:
        ast, ax, _, aacts = aux
        assert ast.size == store.size and list(ast.specs) == list(store.specs)
        dW = (ast.data.data_ptr() - store.data.data_ptr()) // 4
        dx = (ax - inp) // 4
    for l in range(L - 1):
        h = acts.h[l]
        H = sizes[l + 1]
        dy = (aacts.h[l].data_ptr() - h.data_ptr()) // 4 if pair else 0
        if deep6 and l >= 1:
            ops.linear_fwd_sbf16(inp, ld_in, net.W(l, store), net.b(l, store),
                                 h.data_ptr() + 4 * r0 * H, C, n, sizes[l], H, relu=True, ldy=H,
                                 sxb=R * ld_in, syb=R * H)
        else:
            ops.linear_fwd(inp, False, ld_in, net.W(l, store), net.b(l, store),
                           h.data_ptr() + 4 * r0 * H, C, n, sizes[l], H, relu=True, ldy=H,
                           sxb=sxb_ if l == 0 else R * ld_in, syb=R * H,
                           pair=(dx, dW, dy) if pair else None)
        inp, ld_in = h.data_ptr() + 4 * r0 * H, H
        dx = dy
    out_dim = sizes[-1]
    Hl = sizes[-2]
    dout = (aacts.out.data_ptr() - acts.out.data_ptr()) // 4 if pair else 0
    if skip_head:  # the caller's kernel evaluates the head (head1_min)
        assert not pair
        return False
    if out_dim <= 16:
        # narrow heads (Q values, policy mu|logstd): one wave per row beats a
        # 32-wide MFMA tile that is mostly padding
        ops.rowdot(inp, R * Hl if L > 1 else sxb_, ld_in, net.W(L - 1, store), Hl * out_dim,
                   net.b(L - 1, store), out_dim, acts.out.data_ptr() + 4 * r0 * out_dim,
                   R * out_dim, C, n, Hl, pair=(dx, dW, dW, dout) if pair else None, J=out_dim)
    else:
        ops.linear_fwd(inp, False, ld_in, net.W(L - 1, store), net.b(L - 1, store),
                       acts.out.data_ptr() + 4 * r0 * out_dim, C, n, Hl, out_dim, relu=False,
                       ldy=out_dim, sxb=R * Hl if L > 1 else sxb_, syb=R * out_dim,
                       pair=(dx, dW, dout) if pair else None)
    if aux is not None and not pair:
        forward(net, aux[0], aux[1], True, aux[2], aux[3], keep_h=False)
    return False


class BackwardSpace:
    """dz ping-pong buffers + weight-gradient partial workspaces for one net."""

    def __init__(self, net: EnsembleMLP, rows: int, grads: Optional[GradSpace], device,
                 splits: Optional[int] = None, head_partials: Optional[int] = None,
                 slice_r0: Optional[int] = None, small: bool = False):
        """``head_partials``: partial count of the head layer's weight / bias
        gradients when a caller's kernel writes them (one per row, say)
        instead of the split-K GEMM (``backward(..., head_ready=True)``).
        ``slice_r0``: the backward will read the forward's activations from
        this row on; where ``slice_ok`` the weight gradients come from the
        slice kernel (``self.slice``: its partial layout, and the caller's
        Acts must set ``no_last_h``).  ``small``: where ``small_bwd_ok`` the
        whole backward is one d3a_mlp_bwd_small launch (``self.small``: one
        partial per 32-row block for every layer)."""
        self.net = net
        self.rows = rows
        hidden = net.sizes[1:-1]
        if len(set(hidden)) > 1:
            raise NotImplementedError("hidden layers of unequal width are not supported")
        Hmax = hidden[0] if hidden else 1
        self.fused = _FUSED_BWD and fused_ok(net, rows, backward=True)
        # fused path: one dz buffer per hidden layer (written by d3a_mlp_bwd,
        # read by the weight-gradient GEMMs) + the effective head gradient;
        # per-layer path: two ping-pong buffers
        n_dz = len(hidden) if self.fused else 2
        self.dz = [torch.zeros(net.C, rows, Hmax, device=device) for _ in range(max(2, n_dz))]
        self.g_eff = torch.zeros(net.C, rows, device=device) if self.fused else None
        self.splits = n_splits(rows) if splits is None else splits
        self.grads = grads
        # every weight gradient from d3a_q2_bwd: one partial per 256-row block
        self.q2 = grads is not None and head_partials is None and q2_ok(net, rows)
        # the trunk from a caller-formed dz2 (head_ready), 32-row partials
        self.q2p = (grads is not None and head_partials is not None and not self.fused
                    and q2p_ok(net, rows))
        self.slice = (self.q2 and slice_r0 is not None and slice_ok(net, rows, slice_r0))
        self.slice_P = N.lib().d3a_q2_bwd_x6t_splits(rows, net.C) if self.slice else 0
        self.small = (small and not self.fused and not self.q2 and not self.q2p
                      and small_bwd_ok(net, rows))
        if self.small:
            nrb = (rows + 31) // 32
            self.sb_scratch = torch.zeros(8, net.C, rows, 256, device=device)
            self.sb_tickets = torch.zeros(net.C, nrb, dtype=torch.int32, device=device)
        # first-layer weight gradients as one partial per 128-row tile, from
        # the second layer's input-gradient GEMM (backward's wnext path; it
        # needs a layer above the first one, i.e. >= 2 hidden layers)
        self.l0_tiles = None
        if (grads is not None and _FIRST_LAYER_EPI and not self.fused and not self.q2
                and net.n_layers >= 3 and net.sizes[0] <= 64
                and rows * net.C >= _HEAD_GEN_MIN_ROWS):
            self.l0_tiles = (rows + 127) // 128
        if grads is not None:
            for l in range(net.n_layers):
                o, i = net.sizes[l + 1], net.sizes[l]
                parts = head_partials if (head_partials and l == net.n_layers - 1) \
                    else (self.l0_tiles if (l == 0 and self.l0_tiles) else self.splits)
                wparts = None
                if self.small:
                    parts = (rows + 31) // 32
                elif self.slice:
                    # one per row block; the head weight one per row block and
                    # 16-unit slice of layer 1
                    parts = self.slice_P
                    if l == net.n_layers - 1:
                        wparts = 16 * self.slice_P
                elif self.q2:
                    parts = (rows + 255) // 256
                elif self.q2p and l < net.n_layers - 1:
                    parts = (rows + 31) // 32
                grads.add(net.wname(l), (net.C, o, i), wparts or parts)
                grads.add(net.bname(l), (net.C, o), parts)


def backward(bs: BackwardSpace, store: ParamStore, x: int, x_shared: bool, ldx: int,
             acts: Acts, dout: int, ld_dout: int, sdout_b: int, r0: int, n: int,
             weight_grads: bool = True, dx: Optional[torch.Tensor] = None,
             sxb: Optional[int] = None, q_min: Optional[int] = None, sq_b: int = 0,
             q_scale: float = 0.0, g_out: Optional[int] = None,
             g_scale: Optional[int] = None, n_scaled: int = 0,
             members: Optional[int] = None, head_ready: bool = False,
             head_desc=None, cql_loss=None) -> Optional[torch.Tensor]:
    """Backward of rows [r0, r0+n) given dL/d(output) (``dout`` points at row r0).
    Returns (per-layer path) the dz buffer holding the first layer's
    pre-activation gradient [C][rows][ld] once the trunk has run.

    ``cql_loss`` (a split d3a_cql_loss_desc): the slice kernel with the CQL
    loss stage in its prologue (d3a_q2_bwd_x6_cql; g_scale is then not read).

    dout layout: [C] x rows, member stride sdout_b, row stride ld_dout (1 for a
    single-output head).  ``dx`` (if given) receives dL/dx as [C][n][in].
    With ``q_min`` (single-output heads only) the row gradient is ``q_scale`` on
    the argmin member of q_min[.][r] (backward of a min over the ensemble).
    ``head_ready``: the caller's head kernel already wrote the head's input
    gradient into ``bs.dz[0]`` and its weight / bias gradient partials (per-
    layer path only); the backward starts at the trunk.
    ``head_desc`` (with ``head_ready``, the one-launch trunk of a 2x256 policy):
    the d3a_sac_actor_head descriptor (dq_min form) whose work runs in the
    trunk launch's prologue instead (d3a_q2_bwd_actor_head); returns False
    when the shape does not take it (the caller launches the head first).
    """
    net = bs.net
    C, L, sizes, R = net.C, net.n_layers, net.sizes, acts.R
    if members is not None:
        assert not weight_grads, "member subsets are for input gradients only"
        C = members
    S = bs.splits
    assert n <= bs.rows
    sxb_ = (0 if x_shared else R * ldx) if sxb is None else sxb
    gs = bs.grads
    if bs.fused:
        assert not head_ready
        _backward_fused(bs, store, x, ldx, sxb_, acts, dout, ld_dout, sdout_b, r0, n,
                        weight_grads, dx, q_min, sq_b, q_scale, g_out, g_scale, n_scaled, C)
        return
    if bs.q2 and weight_grads:
        if (dx is not None or q_min is not None or head_ready or members is not None
                or n != bs.rows or ld_dout != 1):
            raise NotImplementedError("d3a_q2_bwd space: weight gradients of all rows only")
        d = N.Q2BwdDesc()
        H = sizes[1]
        esz = acts.h[0].element_size()  # 2: bf16 activations (d3a_q2_bwd_bf16)
        d.x, d.ldx, d.sxb = x + 4 * r0 * ldx, ldx, sxb_
        d.h1 = acts.h[0].data_ptr() + esz * r0 * H
        d.h2 = acts.h[1].data_ptr() + esz * r0 * H
        if bs.slice:
            # the slice kernel: row + transposed mask bits of the forward, b2,
            # no h2 (the space's partials are laid out for it)
            if not (acts.hmaskT_from is not None and acts.hmaskT_from <= r0 and r0 % 32 == 0
                    and acts.hmask_from is not None and acts.hmask_from <= r0
                    and r0 + n <= acts.hmask_to):
                raise RuntimeError("slice backward: the forward did not write the mask bits "
                                   f"of rows [{r0}, {r0 + n})")
            d.h2 = None
            d.m2, d.sm2 = acts.hmask.data_ptr() + 4 * r0 * (H // 32), R * (H // 32)
            d.m2t, d.sm2t = (acts.hmaskT.data_ptr() + 4 * (r0 // 32) * H, acts.hmaskT[0].numel())
            d.b2, d.sb2 = net.b(1, store), H
            d.row_splits = bs.slice_P
        d.sh, d.ldh = R * H, H
        d.g, d.sgb = dout, sdout_b
        if g_scale is not None:
            d.gscale, d.n_scaled = g_scale, n_scaled
        d.W2, d.sW2 = net.W(1, store), H * H
        d.w3, d.sw3 = net.W(2, store), H
        d.dW1, d.db1 = gs.get(net.wname(0)).data_ptr(), gs.get(net.bname(0)).data_ptr()
        d.dW2, d.db2 = gs.get(net.wname(1)).data_ptr(), gs.get(net.bname(1)).data_ptr()
        d.dW3, d.db3 = gs.get(net.wname(2)).data_ptr(), gs.get(net.bname(2)).data_ptr()
        d.rows, d.n_in, d.C = n, sizes[0], C
        entry = "d3a_q2_bwd_bf16" if esz == 2 else "d3a_q2_bwd"
        if esz == 4 and (ops.CRITIC_GEMM == "x6" or ops.CRITIC_PRECISION == "bf16"):
            entry = "d3a_q2_bwd_x6"  # fp32-accurate split-bf16 (mask-factored)
            if (not bs.slice and acts.hmask is not None and acts.hmask_from is not None
                    and acts.hmask_from <= r0 and r0 + n <= acts.hmask_to and _MASK_IMAGE):
                # the forward's mask image of h2 (same rows as h1 / h2)
                d.m2, d.sm2 = acts.hmask.data_ptr() + 4 * r0 * (H // 32), R * (H // 32)
        if cql_loss is not None:
            assert entry == "d3a_q2_bwd_x6" and bs.slice
            ops.call_desc("d3a_q2_bwd_x6_cql", d, cql_loss)
            return None
        ops.call_desc(entry, d)
        return None

    if (bs.q2p and weight_grads and head_ready and dx is None and members is None
            and n == bs.rows):
        # trunk backward in one launch from the head kernel's dz2 (bs.dz[0])
        d = N.Q2BwdDesc()
        H = sizes[1]
        d.x, d.ldx, d.sxb = x + 4 * r0 * ldx, ldx, sxb_
        d.h1 = acts.h[0].data_ptr() + 4 * r0 * H
        d.sh, d.ldh = R * H, H
        d.dz2, d.sdz = bs.dz[0].data_ptr(), bs.rows * bs.dz[0].shape[2]
        assert bs.dz[0].shape[2] == H
        d.block_rows = 32
        d.W2, d.sW2 = net.W(1, store), H * H
        d.dW1, d.db1 = gs.get(net.wname(0)).data_ptr(), gs.get(net.bname(0)).data_ptr()
        d.dW2, d.db2 = gs.get(net.wname(1)).data_ptr(), gs.get(net.bname(1)).data_ptr()
        d.rows, d.n_in, d.C = n, sizes[0], C
        if head_desc is not None:
            if not (_HEAD_IN_TRUNK and C == 1 and head_desc.dq_min and not head_desc.dq_dz
                    and head_desc.H == H and head_desc.B == n):
                return False
            d.dz2 = None  # formed per workgroup from dhead
            ops.call_desc("d3a_q2_bwd_actor_head", d, head_desc)
            return True
        ops.call_desc("d3a_q2_bwd", d)
        return None
    if head_desc is not None:
        return False

    if (bs.small and q_min is None and g_out is None and g_scale is None and not head_ready
            and (n == bs.rows or not weight_grads)):
        # the whole backward in one launch (d3a_mlp_bwd_small)
        d = N.MlpBwdSmallDesc()
        H = sizes[1]
        d.x, d.ldx, d.sxb = x + 4 * r0 * ldx, ldx, sxb_
        d.h1 = acts.h[0].data_ptr() + 4 * r0 * H
        d.h2 = acts.h[1].data_ptr() + 4 * r0 * H
        d.sh = R * H
        d.dout, d.ld_dout, d.sdout = dout, ld_dout, sdout_b
        d.W1, d.W2, d.W3 = net.W(0, store), net.W(1, store), net.W(2, store)
        d.sW1, d.sW2, d.sW3 = H * sizes[0], H * H, sizes[3] * H
        if weight_grads:
            d.dW1, d.db1 = gs.get(net.wname(0)).data_ptr(), gs.get(net.bname(0)).data_ptr()
            d.dW2, d.db2 = gs.get(net.wname(1)).data_ptr(), gs.get(net.bname(1)).data_ptr()
            d.dW3, d.db3 = gs.get(net.wname(2)).data_ptr(), gs.get(net.bname(2)).data_ptr()
        d.dx = dx.data_ptr() if dx is not None else None
        d.scratch, d.tickets = bs.sb_scratch.data_ptr(), bs.sb_tickets.data_ptr()
        d.rows, d.n_in, d.n_out, d.C = n, sizes[0], sizes[3], C
        ops.call_desc("d3a_mlp_bwd_small", d)
        return None

    def h_ptr(l):  # input activation of layer l at row r0
        if l == 0:
            return x + 4 * r0 * ldx, ldx, sxb_
        H = sizes[l]
        return acts.h[l - 1].data_ptr() + 4 * r0 * H, H, R * H

    # ---- head layer L-1
    hin, ld_h, sh = h_ptr(L - 1)
    Hin = sizes[L - 1]
    out_dim = sizes[L]
    cur = bs.dz[0]
    if L == 1:
        if weight_grads:
            gW, gb = gs.get(net.wname(0)), gs.get(net.bname(0))
            ops.linear_bwd_w(dout, ld_dout, sdout_b, hin, ld_h, sh, gW.data_ptr(), C, n, Hin,
                             out_dim, S, db=gb.data_ptr())
        if dx is not None:
            ops.linear_bwd_x(dout, ld_dout, sdout_b, net.W(0, store), dx.data_ptr(), sizes[0],
                             n * sizes[0], C, n, sizes[0], out_dim)
        return
    ld_cur = bs.dz[0].shape[2]
    scur = bs.rows * ld_cur
    # deep 256-wide critics under CRITIC_GEMM "x6": the 256 x 256 layers'
    # weight and input gradients on the split-bf16 GEMM (six products); the
    # head's dz then comes from d3a_head1_bwd (agen is an fp32-GEMM feature)
    t6 = 6 if (ops.CRITIC_GEMM == "x6" and _X6_DEEP and x6_deep_shape(net)
               and n * C >= 8192) else 0
    # large critic backward: the head's masked input gradient is generated
    # inside the trunk's two GEMMs (d3a_gemm_desc.agen) instead of written by
    # d3a_head1_bwd and read back; the weight-gradient GEMM also writes the
    # head's weight / bias gradient partials
    agen = None
    if out_dim == 1 and q_min is None and weight_grads and _HEAD_GEN and not ops.SBF16_TERMS \
            and not t6 and n * C >= _HEAD_GEN_MIN_ROWS:
        agen = N.Head1BwdDesc()
        agen.g, agen.sgb = dout, sdout_b
        if g_scale is not None:
            agen.gscale, agen.n_scaled = g_scale, n_scaled
        agen.h, agen.shb, agen.ldh = hin, sh, ld_h
        agen.w, agen.swb = net.W(L - 1, store), Hin
        gW, gb = gs.get(net.wname(L - 1)), gs.get(net.bname(L - 1))
        agen.dW, agen.sWs = gW.data_ptr(), C * Hin
        agen.db, agen.sbs = gb.data_ptr(), C
        agen.rows, agen.n, agen.C, agen.splits = n, Hin, C, S
    if agen is not None or head_ready:
        pass
    elif out_dim == 1:
        # fused: masked input gradient + head weight/bias gradients, h read once
        d = N.Head1BwdDesc()
        if q_min is not None:
            d.q_min, d.sqb, d.scale = q_min, sq_b, q_scale
            d.g_out, d.sgb = g_out, sdout_b
        else:
            d.g, d.sgb = dout, sdout_b
            if g_scale is not None:
                d.gscale, d.n_scaled = g_scale, n_scaled
        d.h, d.shb, d.ldh = hin, sh, ld_h
        d.w, d.swb = net.W(L - 1, store), Hin
        d.dz, d.sdzb, d.lddz = cur.data_ptr(), scur, ld_cur
        if weight_grads:
            gW, gb = gs.get(net.wname(L - 1)), gs.get(net.bname(L - 1))
            d.dW, d.sWs = gW.data_ptr(), C * Hin
            d.db, d.sbs = gb.data_ptr(), C
        d.rows, d.n, d.C = n, Hin, C
        d.splits = S if weight_grads else max(1, n // 64)
        ops.call_desc("d3a_head1_bwd", d)
    else:
        assert q_min is None
        if weight_grads and not head_ready:
            gW, gb = gs.get(net.wname(L - 1)), gs.get(net.bname(L - 1))
            ops.linear_bwd_w(dout, ld_dout, sdout_b, hin, ld_h, sh, gW.data_ptr(), C, n, Hin,
                             out_dim, S, db=gb.data_ptr())
        if not head_ready:
            ops.linear_bwd_x(dout, ld_dout, sdout_b, net.W(L - 1, store), cur.data_ptr(), ld_cur,
                             scur, C, n, Hin, out_dim, mask=hin, ldm=ld_h, smb=sh)
    # ---- the three-hidden-layer critic (round 6): the two 256-wide layers'
    # input gradients in one d3a_mlp_bwd_chain launch (dz3 -> dz2 -> dz1 on
    # split-bf16 streams over W^T), the weight gradients on their GEMMs
    if (t6 and _X6_BWD_CHAIN and L == 4 and weight_grads and dx is None and not head_ready
            and agen is None and members is None and bs.dz[0].shape[2] == sizes[1]):
        dz3, other = cur, (bs.dz[1] if cur is bs.dz[0] else bs.dz[0])
        H = sizes[1]
        gW, gb = gs.get(net.wname(2)), gs.get(net.bname(2))
        h2p, ld2, s2 = h_ptr(2)
        ops.linear_bwd_w(dz3.data_ptr(), ld_cur, scur, h2p, ld2, s2, gW.data_ptr(), C, n, H, H, S,
                         db=gb.data_ptr(), sbf16=t6)
        ch = N.MlpBwdChainDesc()
        ch.dz_top, ch.dz_mid, ch.dz_bot = dz3.data_ptr(), other.data_ptr(), dz3.data_ptr()
        ch.h_mid, ch.h_bot = h_ptr(2)[0], h_ptr(1)[0]
        ch.Wa, ch.Wb, ch.sW = net.W(2, store), net.W(1, store), H * H
        ch.ld, ch.sdz, ch.ldh, ch.sh, ch.rows, ch.C = ld_cur, scur, H, R * H, n, C
        ops.call_desc("d3a_mlp_bwd_chain", ch)
        gW, gb = gs.get(net.wname(1)), gs.get(net.bname(1))
        h1p, ld1, s1 = h_ptr(1)
        ops.linear_bwd_w(other.data_ptr(), ld_cur, scur, h1p, ld1, s1, gW.data_ptr(), C, n, H, H, S,
                         db=gb.data_ptr(), sbf16=t6)
        gW, gb = gs.get(net.wname(0)), gs.get(net.bname(0))
        x0, ldx0, sx0 = h_ptr(0)
        S0 = bs.l0_tiles if bs.l0_tiles else S
        ops.linear_bwd_w(dz3.data_ptr(), ld_cur, scur, x0, ldx0, sx0, gW.data_ptr(), C, n, sizes[0],
                         H, S0, db=gb.data_ptr(), sbf16=t6)
        return None
    # ---- trunk layers L-2 .. 0
    # first layer's weight gradients from the second layer's dX epilogue
    ew = (bs.l0_tiles is not None and weight_grads and dx is None and n == bs.rows
          and not ops.SBF16_TERMS and not t6)
    for l in range(L - 2, -1, -1):
        Hout = sizes[l + 1]
        Hin = sizes[l]
        hin, ld_h, sh = h_ptr(l)
        dz = cur
        ag = agen if l == L - 2 else None  # the head's dz, generated
        if l == 0 and ew:
            break  # written by the l == 1 launch
        if weight_grads and l > 0 and not (l == 1 and ew):
            # this layer's weight and input gradients are independent: one
            # paired submission (a single launch on the register-direct kernel)
            gW, gb = gs.get(net.wname(l)), gs.get(net.bname(l))
            nxt = bs.dz[1] if cur is bs.dz[0] else bs.dz[0]
            ops.gemm_pair(
                lambda: ops.linear_bwd_w(dz.data_ptr(), ld_cur, scur, hin, ld_h, sh,
                                         gW.data_ptr(), C, n, Hin, Hout, S, db=gb.data_ptr(),
                                         agen=ag, sbf16=t6),
                lambda: ops.linear_bwd_x(dz.data_ptr(), ld_cur, scur, net.W(l, store),
                                         nxt.data_ptr(), ld_cur, scur, C, n, Hin, Hout,
                                         mask=hin, ldm=ld_h, smb=sh, agen=ag, sbf16=t6))
            cur = nxt
            continue
        if weight_grads:
            gW, gb = gs.get(net.wname(l)), gs.get(net.bname(l))
            S_l = bs.l0_tiles if (l == 0 and bs.l0_tiles) else S
            ops.linear_bwd_w(dz.data_ptr(), ld_cur, scur, hin, ld_h, sh, gW.data_ptr(), C, n, Hin,
                             Hout, S_l, db=gb.data_ptr(), agen=ag, sbf16=t6)
        if l == 1 and ew:
            x0, ldx0, sx0 = h_ptr(0)
            wn = N.GemmWnext()
            wn.x, wn.ldx, wn.sxb, wn.n_in = x0, ldx0, sx0, sizes[0]
            wn.dW = gs.get(net.wname(0)).data_ptr()
            wn.db = gs.get(net.bname(0)).data_ptr()
            ops.linear_bwd_x(dz.data_ptr(), ld_cur, scur, net.W(1, store), 0, ld_cur, scur, C, n,
                             Hin, Hout, mask=hin, ldm=ld_h, smb=sh, agen=ag, wnext=wn)
            continue
        if l > 0:
            nxt = bs.dz[1] if cur is bs.dz[0] else bs.dz[0]
            ops.linear_bwd_x(dz.data_ptr(), ld_cur, scur, net.W(l, store), nxt.data_ptr(), ld_cur,
                             scur, C, n, Hin, Hout, mask=hin, ldm=ld_h, smb=sh, agen=ag, sbf16=t6)
            cur = nxt
        elif dx is not None:
            ops.linear_bwd_x(dz.data_ptr(), ld_cur, scur, net.W(0, store), dx.data_ptr(), Hin,
                             n * Hin, C, n, Hin, Hout, agen=ag)
    return cur



def _backward_fused(bs: BackwardSpace, store: ParamStore, x: int, ldx: int, sxb: int, acts: Acts,
                    dout: int, ld_dout: int, sdout_b: int, r0: int, n: int, weight_grads: bool,
                    dx: Optional[torch.Tensor], q_min: Optional[int], sq_b: int, q_scale: float,
                    g_out: Optional[int], g_scale: Optional[int], n_scaled: int, C: int) -> None:
    """d3a_mlp_bwd (the dz chain and dx in one launch) + one split-K weight
    gradient GEMM per layer (with the bias gradient as its row sums)."""
    net = bs.net
    L, sizes, R = net.n_layers, net.sizes, acts.R
    H, J = sizes[1], sizes[-1]
    rows = bs.rows
    d = N.MlpBwdDesc()
    d.n_in, d.n_hidden, d.H, d.n_out, d.C = sizes[0], L - 1, H, J, C
    for l in range(L):
        d.W[l], d.sW[l] = net.W(l, store), sizes[l + 1] * sizes[l]
    for l in range(L - 1):
        d.h[l] = acts.h[l].data_ptr() + 4 * r0 * H
        d.dz[l] = bs.dz[l].data_ptr()
    d.sh, d.ldh, d.sdz = R * H, H, rows * H
    if J == 1:
        if q_min is not None:
            d.q_min, d.sqb, d.scale = q_min, sq_b, q_scale
        else:
            d.g, d.sgb = dout, sdout_b
            if g_scale is not None:
                d.gscale, d.n_scaled = g_scale, n_scaled
        if g_out is not None:  # caller wants the effective row gradient (e.g. argmin mask)
            assert not weight_grads
            d.g_eff, d.sgeb = g_out, sdout_b
        else:
            d.g_eff, d.sgeb = bs.g_eff.data_ptr(), rows
    else:
        d.dhead, d.sdhb, d.lddh = dout, sdout_b, ld_dout
    if dx is not None:
        d.dx, d.sdxb, d.lddx = dx.data_ptr(), n * sizes[0], sizes[0]
    d.rows = n
    ops.call_desc("d3a_mlp_bwd", d)
    if not weight_grads:
        return
    gs, S = bs.grads, bs.splits
    hin_last = acts.h[L - 2].data_ptr() + 4 * r0 * H
    gW, gb = gs.get(net.wname(L - 1)), gs.get(net.bname(L - 1))
    if J == 1:
        ops.linear_bwd_w(bs.g_eff.data_ptr(), 1, rows, hin_last, H, R * H, gW.data_ptr(), C, n,
                         H, 1, S, db=gb.data_ptr())
    else:
        ops.linear_bwd_w(dout, ld_dout, sdout_b, hin_last, H, R * H, gW.data_ptr(), C, n, H, J,
                         S, db=gb.data_ptr())
    for l in range(L - 2, -1, -1):
        if l == 0:
            hin, ld_h, sh = x + 4 * r0 * ldx, ldx, sxb
        else:
            hin, ld_h, sh = acts.h[l - 1].data_ptr() + 4 * r0 * H, H, R * H
        gW, gb = gs.get(net.wname(l)), gs.get(net.bname(l))
        ops.linear_bwd_w(bs.dz[l].data_ptr(), H, rows * H, hin, ld_h, sh, gW.data_ptr(), C, n,
                         sizes[l], H, S, db=gb.data_ptr())
