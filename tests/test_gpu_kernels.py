"""Kernel-level parity of the HIP library against plain PyTorch fp32 (GPU only).

Each test calls the C-ABI through d3rlpy_amd.ops on device tensors and
compares with the same op in torch (computed in fp64 where the tolerance is
about accumulation order).  Tolerances are stated per test.
"""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    from d3rlpy_amd import _native
    _native.lib()
    return torch.device("cuda:0")


def _rel_err(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return float((a - b).abs().max() / max(1e-30, float(b.abs().max())))


@pytest.mark.parametrize("M,N,K,C,relu", [(64, 64, 16, 1, False), (200, 256, 14, 2, True),
                                          (7936, 256, 256, 2, True), (37, 6, 256, 1, False),
                                          (1, 1, 1, 1, False), (130, 70, 33, 3, True)])
def test_linear_forward(dev, M, N, K, C, relu):
    from d3rlpy_amd import ops
    g = torch.Generator().manual_seed(M * 7 + N)
    x = torch.randn(M, K, generator=g).to(dev)
    W = torch.randn(C, N, K, generator=g).to(dev)
    b = torch.randn(C, N, generator=g).to(dev)
    y = torch.full((C, M, N), float("nan"), device=dev)
    ops.linear_fwd(x.data_ptr(), True, K, W.data_ptr(), b.data_ptr(), y.data_ptr(), C, M, K, N,
                   relu)
    torch.cuda.synchronize()
    ref = torch.einsum("mk,cnk->cmn", x.double(), W.double()) + b.double()[:, None, :]
    if relu:
        ref = ref.clamp_min(0)
    # exact-f32 MFMA chain: error <= K * 2^-24 * sum|a*b| ~ 1e-6 relative at K=256
    assert _rel_err(y, ref) < 2e-6


@pytest.mark.parametrize("R,Nin,Nout,C,splits", [(7936, 256, 256, 2, 31), (256, 14, 256, 2, 1),
                                                 (100, 3, 7, 1, 3), (513, 256, 6, 1, 2)])
def test_linear_backward(dev, R, Nin, Nout, C, splits):
    from d3rlpy_amd import ops
    g = torch.Generator().manual_seed(R + Nin)
    x = torch.randn(C, R, Nin, generator=g).to(dev)
    dy = torch.randn(C, R, Nout, generator=g).to(dev)
    W = torch.randn(C, Nout, Nin, generator=g).to(dev)
    h = torch.randn(C, R, Nin, generator=g).to(dev).clamp_min(0)
    dW = torch.zeros(splits, C, Nout, Nin, device=dev)
    ops.linear_bwd_w(dy.data_ptr(), Nout, R * Nout, x.data_ptr(), Nin, R * Nin, dW.data_ptr(), C,
                     R, Nin, Nout, splits)
    dx = torch.zeros(C, R, Nin, device=dev)
    ops.linear_bwd_x(dy.data_ptr(), Nout, R * Nout, W.data_ptr(), dx.data_ptr(), Nin, R * Nin, C,
                     R, Nin, Nout, mask=h.data_ptr(), ldm=Nin, smb=R * Nin)
    torch.cuda.synchronize()
    ref_dW = torch.einsum("crn,cri->cni", dy.double(), x.double())
    ref_dx = torch.einsum("crn,cni->cri", dy.double(), W.double()) * (h.double() > 0)
    assert _rel_err(dW.sum(0), ref_dW) < 5e-6
    assert _rel_err(dx, ref_dx) < 5e-6


@pytest.mark.parametrize("variant", list(range(11)))
def test_gemm_every_variant(dev, variant):
    """Every tile variant (LDS-tiled 0-8, register-direct 9-10) on all four
    operand-layout combinations with row sums, bias, relu, mask and
    accumulate; fp64 reference, tolerance 5e-6 relative (exact-f32 chains)."""
    from d3rlpy_amd import ops
    g = torch.Generator().manual_seed(variant)
    splits = 1
    for (M, N, K, batch) in [(256, 256, 256, 2), (37, 70, 300, 1), (130, 6, 11, 3),
                             (256, 14, 1000, 2)]:
        for a_k, b_k in [(True, True), (True, False), (False, True), (False, False)]:
            A = torch.randn(batch, M, K, generator=g).to(dev)
            Bm = torch.randn(batch, K, N, generator=g).to(dev)
            # storage: k-contiguous or x-contiguous copies of the same operand
            As = A.contiguous() if a_k else A.transpose(1, 2).contiguous()
            Bs = Bm.transpose(1, 2).contiguous() if b_k else Bm.contiguous()
            sA = (M * K, K, 1) if a_k else (M * K, 1, M)
            sB = (K * N, 1, K) if b_k else (K * N, N, 1)
            bias = torch.randn(batch, N, generator=g).to(dev)
            mask = torch.randn(batch, M, N, generator=g).to(dev)
            Cb = torch.randn(splits, batch, M, N, generator=g).to(dev)
            C0 = Cb.clone()
            rs = torch.zeros(splits, batch, M, device=dev)
            ops.gemm(As.data_ptr(), Bs.data_ptr(), Cb.data_ptr(), M, N, K, batch=batch, sA=sA,
                     sB=sB, sC=(M * N, N, 1), splits=splits, sCs=batch * M * N,
                     bias=bias.data_ptr(), sbias=N, relu=True, mask=mask.data_ptr(),
                     sM=(M * N, N, 1), accumulate=True, rowsum=rs.data_ptr(), sR=(M, batch * M),
                     variant=variant)
            torch.cuda.synchronize()
            tot = (Cb - C0).double().sum(0)
            ref = torch.einsum("bmk,bkn->bmn", A.double(), Bm.double()) + bias.double()[:, None]
            ref = ref.clamp_min(0) * (mask.double() > 0)
            assert _rel_err(tot, ref) < 5e-6, (variant, M, N, K, a_k, b_k)
            assert _rel_err(rs[0], A.double().sum(2)) < 5e-6, (variant, M, N, K, a_k, b_k)


@pytest.mark.parametrize("variant", list(range(11)))
def test_gemm_split_k_sum(dev, variant):
    """Split-K partials (no epilogue) sum to the full product for every variant."""
    from d3rlpy_amd import ops
    g = torch.Generator().manual_seed(100 + variant)
    M, N, K, batch, splits = 256, 256, 7936 // 4, 2, 8
    A = torch.randn(batch, K, M, generator=g).to(dev)  # dY^T layout: A[m][k] = dY[k][m]
    X = torch.randn(batch, K, N, generator=g).to(dev)
    out = torch.zeros(splits, batch, M, N, device=dev)
    rs = torch.zeros(splits, batch, M, device=dev)
    ops.gemm(A.data_ptr(), X.data_ptr(), out.data_ptr(), M, N, K, batch=batch,
             sA=(K * M, 1, M), sB=(K * N, N, 1), sC=(M * N, N, 1), splits=splits,
             sCs=batch * M * N, rowsum=rs.data_ptr(), sR=(M, batch * M), variant=variant)
    torch.cuda.synchronize()
    ref = torch.einsum("bkm,bkn->bmn", A.double(), X.double())
    assert _rel_err(out.double().sum(0), ref) < 5e-6
    assert _rel_err(rs.double().sum(0), A.double().sum(1)) < 5e-6


def test_rowdot_colreduce_outer(dev):
    from d3rlpy_amd import ops
    g = torch.Generator().manual_seed(3)
    C, R, H = 2, 1000, 256
    X = torch.randn(C, R, H, generator=g).to(dev)
    w = torch.randn(C, H, generator=g).to(dev)
    bias = torch.randn(C, 1, generator=g).to(dev)
    out = torch.zeros(C, R, device=dev)
    ops.rowdot(X.data_ptr(), R * H, H, w.data_ptr(), H, bias.data_ptr(), 1, out.data_ptr(), R, C,
               R, H)
    gq = torch.randn(C, R, generator=g).to(dev)
    S = 4
    cr = torch.zeros(S, C, H, device=dev)
    ops.colreduce(X.data_ptr(), R * H, H, gq.data_ptr(), R, cr.data_ptr(), H, C * H, C, R, H, S)
    om = torch.zeros(C, R, H, device=dev)
    ops.outer_mask(gq.data_ptr(), R, w.data_ptr(), H, X.data_ptr(), R * H, om.data_ptr(), R * H,
                   C, R, H)
    torch.cuda.synchronize()
    ref = torch.einsum("crh,ch->cr", X.double(), w.double()) + bias.double()
    assert _rel_err(out, ref) < 2e-6
    ref_cr = torch.einsum("cr,crh->ch", gq.double(), X.double())
    assert _rel_err(cr.sum(0), ref_cr) < 2e-6
    ref_om = gq.double()[:, :, None] * w.double()[:, None, :] * (X.double() > 0)
    assert torch.equal(om.cpu(), ref_om.float().cpu())


def test_soft_update_bit_exact(dev):
    """soft_sync (torch_utility.py:27-33): three separately rounded fp32 ops."""
    from d3rlpy_amd import ops
    g = torch.Generator().manual_seed(4)
    src = torch.randn(100003, generator=g)
    targ = torch.randn(100003, generator=g)
    tau = 0.005
    ref = targ.clone()
    ref.mul_(1 - tau)
    ref.add_(tau * src)
    t = targ.to(dev)
    ops.soft_update(t, src.to(dev), tau)
    assert torch.equal(t.cpu(), ref)


def test_adam_matches_torch(dev):
    """torch.optim.Adam single-tensor step (the oracle's CPU Adam), 3 steps;
    11 split-K partials (one batch of 32 clamped loads) over a multi-block
    segment followed by a one-block segment (flat grid)."""
    from d3rlpy_amd.nets import AdamGroup, GradSpace, ParamStore
    store = ParamStore()
    store.add("w", (300, 7))
    store.add("b", (5,))
    store.allocate(dev)
    g = torch.Generator().manual_seed(5)
    w0 = torch.randn(300, 7, generator=g)
    b0 = torch.randn(5, generator=g)
    store.view("w").copy_(w0)
    store.view("b").copy_(b0)
    gs = GradSpace(dev)
    gw = gs.add("w", (300, 7), 11)
    gb = gs.add("b", (5,), 1)
    from d3rlpy_amd import ops
    from d3rlpy_amd.nets import OptimState
    opt = AdamGroup(OptimState(store, ["w", "b"], lr=3e-4), gs)
    pw = torch.nn.Parameter(w0.clone())
    pb = torch.nn.Parameter(b0.clone())
    topt = torch.optim.Adam([pw, pb], lr=3e-4)
    for it in range(3):
        parts = torch.randn(11, 300, 7, generator=g) * 10 ** (-it)
        gbv = torch.randn(5, generator=g)
        gw.copy_(parts)
        gb.copy_(gbv.view(1, 5))
        opt.launch()
        ops.step_end(opt.step, 1)
        # the kernel sums split-K partials in fp64 (then rounds once)
        pw.grad = parts.double().sum(0).float()
        pb.grad = gbv.clone()
        topt.step()
    torch.cuda.synchronize()
    assert int(opt.step.item()) == 3
    # identical formula; only the partial-sum order / lerp fma differ (<= few ulp)
    torch.testing.assert_close(store.view("w").cpu(), pw.detach(), rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(store.view("b").cpu(), pb.detach(), rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(opt.exp_avg_sq.view("w").cpu(), topt.state[pw]["exp_avg_sq"],
                               rtol=1e-6, atol=1e-12)


def test_adam_many_partials_matches_torch(dev):
    """A segment with >= 64 partials (one per batch row, e.g. the IQN head's
    weight gradient) is summed by 16-lane groups in a fixed order: 3 Adam
    steps vs torch.optim.Adam on the fp64 sum of the partials."""
    from d3rlpy_amd import ops
    from d3rlpy_amd.nets import AdamGroup, GradSpace, OptimState, ParamStore
    store = ParamStore()
    store.add("w", (4, 517))
    store.add("b", (3,))
    store.allocate(dev)
    g = torch.Generator().manual_seed(9)
    w0, b0 = torch.randn(4, 517, generator=g), torch.randn(3, generator=g)
    store.view("w").copy_(w0)
    store.view("b").copy_(b0)
    gs = GradSpace(dev)
    gw = gs.add("w", (4, 517), 203)
    gb = gs.add("b", (3,), 70)
    opt = AdamGroup(OptimState(store, ["w", "b"], lr=1e-3), gs)
    pw, pb = torch.nn.Parameter(w0.clone()), torch.nn.Parameter(b0.clone())
    topt = torch.optim.Adam([pw, pb], lr=1e-3)
    for it in range(3):
        parts = torch.randn(203, 4, 517, generator=g)
        pbv = torch.randn(70, 3, generator=g)
        gw.copy_(parts)
        gb.copy_(pbv)
        opt.launch()
        ops.step_end(opt.step, 1)
        pw.grad = parts.double().sum(0).float()
        pb.grad = pbv.double().sum(0).float()
        topt.step()
    torch.cuda.synchronize()
    torch.testing.assert_close(store.view("w").cpu(), pw.detach(), rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(store.view("b").cpu(), pb.detach(), rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(opt.grad("w").cpu(), pw.grad, rtol=1e-6, atol=1e-6)


def test_adam_many_segments_matches_torch(dev):
    """150 segments (the block -> segment search runs over three 64-lane
    chunks of the table) of 1 .. 700 elements with 1, 11, 40 (two load
    batches) or 70 (16-lane groups) split-K partials: 2 Adam steps vs
    torch.optim.Adam on the fp64 sums of the partials."""
    from d3rlpy_amd import ops
    from d3rlpy_amd.nets import AdamGroup, GradSpace, OptimState, ParamStore
    g = torch.Generator().manual_seed(21)
    n_seg = 150
    sizes = [int(x) for x in torch.randint(1, 700, (n_seg,), generator=g)]
    sizes[3], sizes[77] = 1, 257  # a one-element segment, a block edge
    parts_of = [(1, 11, 40, 70)[k % 4] for k in range(n_seg)]
    store = ParamStore()
    for k, n in enumerate(sizes):
        store.add(f"p{k}", (n,))
    store.allocate(dev)
    gs = GradSpace(dev)
    views, tparams = [], []
    for k, n in enumerate(sizes):
        x0 = torch.randn(n, generator=g)
        store.view(f"p{k}").copy_(x0)
        views.append(gs.add(f"p{k}", (n,), parts_of[k]))
        tparams.append(torch.nn.Parameter(x0.clone()))
    names = [f"p{k}" for k in range(n_seg)]
    opt = AdamGroup(OptimState(store, names, lr=1e-3), gs)
    topt = torch.optim.Adam(tparams, lr=1e-3)
    for it in range(2):
        for k, n in enumerate(sizes):
            parts = torch.randn(parts_of[k], n, generator=g)
            views[k].copy_(parts.view(views[k].shape))
            tparams[k].grad = parts.double().sum(0).float()
        opt.launch()
        ops.step_end(opt.step, 1)
        topt.step()
    torch.cuda.synchronize()
    for k in range(n_seg):
        torch.testing.assert_close(store.view(f"p{k}").cpu(), tparams[k].detach(),
                                   rtol=1e-6, atol=1e-7, msg=f"segment {k}")
    # the data-parallel path's partial reduction walks the same segment table
    opt.grad_store.data.zero_()
    opt.reduce()
    torch.cuda.synchronize()
    for k in (0, 3, 64, 77, 128, 149):
        torch.testing.assert_close(opt.grad(f"p{k}").cpu(), tparams[k].grad, rtol=2e-7, atol=1e-9,
                                   msg=f"reduced segment {k}")


def test_adam_block_table_bit_identical(dev):
    """d3a_adam_step with the per-block segment table (AdamGroup.block_table,
    the production launch) against the in-kernel segment search on the same
    150-segment layout (1 / 11 / 40 / 70 partials): bit-identical parameters,
    moments and target copies (soft update fused)."""
    from d3rlpy_amd import ops
    from d3rlpy_amd.nets import AdamGroup, GradSpace, OptimState, ParamStore
    g = torch.Generator().manual_seed(5)
    n_seg = 150
    sizes = [int(x) for x in torch.randint(1, 700, (n_seg,), generator=g)]
    parts_of = [(1, 11, 40, 70)[k % 4] for k in range(n_seg)]
    runs = []
    for use_table in (True, False):
        store = ParamStore()
        for k, n in enumerate(sizes):
            store.add(f"p{k}", (n,))
        store.allocate(dev)
        targ = store.like()
        gs = GradSpace(dev)
        gk = torch.Generator().manual_seed(9)
        views = []
        for k, n in enumerate(sizes):
            x0 = torch.randn(n, generator=gk)
            store.view(f"p{k}").copy_(x0)
            targ.view(f"p{k}").copy_(x0 * 0.5)
            views.append(gs.add(f"p{k}", (n,), parts_of[k]))
        names = [f"p{k}" for k in range(n_seg)]
        opt = AdamGroup(OptimState(store, names, lr=1e-3), gs)
        ctr = torch.zeros(8, dtype=torch.int64, device=dev)
        for it in range(3):
            for k, n in enumerate(sizes):
                views[k].copy_(torch.randn(parts_of[k], n, generator=gk).view(views[k].shape))
            ops.adam_step(opt.seg_table, n_seg, opt.n_blocks, opt.step, opt.lr, opt.beta1,
                          opt.beta2, opt.eps, 1.0, targ_delta=(targ.data.data_ptr()
                                                               - store.data.data_ptr()) // 4,
                          tau=0.005, counters=ctr, inc_mask=1,
                          blocks=opt.block_table if use_table else None)
            ops.step_end(opt.step, 1)
        torch.cuda.synchronize()
        runs.append((store.data.clone(), targ.data.clone(), opt.exp_avg.data.clone(),
                     opt.exp_avg_sq.data.clone(), ctr.clone()))
    for a, b in zip(*runs):
        assert torch.equal(a, b)


def test_adam_vector_segments(dev):
    """Segments of >= 2^18 elements (a multiple of 4) with < 64 partials run
    four elements a thread (elementwise.hip seg_vec): 2 Adam steps vs
    torch.optim.Adam on the fp64 partial sums, the partial reduction, and a
    soft target copy 4 bytes off 16-byte alignment (the four-scalar fallback)
    bitwise equal to an aligned one."""
    from d3rlpy_amd import ops
    from d3rlpy_amd.nets import AdamGroup, GradSpace, OptimState, ParamStore
    shapes = {"w": ((520, 512), 5), "b": ((7,), 3), "e": (((1 << 18) + 4,), 1),
              "u": ((300, 877), 1)}
    runs = []
    for shift in (0, 1):
        g = torch.Generator().manual_seed(4)
        store = ParamStore()
        for n, (shp, _) in shapes.items():
            store.add(n, shp)
        store.allocate(dev)
        gs = GradSpace(dev)
        views, tp = {}, {}
        for n, (shp, P) in shapes.items():
            x0 = torch.randn(*shp, generator=g)
            store.view(n).copy_(x0)
            views[n] = gs.add(n, shp, P)
            tp[n] = torch.nn.Parameter(x0.clone())
        opt = AdamGroup(OptimState(store, list(shapes), lr=1e-3), gs)
        topt = torch.optim.Adam(list(tp.values()), lr=1e-3)
        tbuf = torch.zeros(store.size + 4, device=dev)
        targ = tbuf[shift: shift + store.size]
        targ.copy_(store.data * 0.5)
        for it in range(2):
            for n, (shp, P) in shapes.items():
                parts = torch.randn(P, *shp, generator=g)
                views[n].copy_(parts.view(views[n].shape))
                tp[n].grad = parts.double().sum(0).float()
            ops.adam_step(opt.seg_table, len(shapes), opt.n_blocks, opt.step, opt.lr, opt.beta1,
                          opt.beta2, opt.eps, 1.0,
                          targ_delta=(targ.data_ptr() - store.data.data_ptr()) // 4,
                          tau=0.005, blocks=opt.block_table)
            ops.step_end(opt.step, 1)
            topt.step()
        torch.cuda.synchronize()
        for n in shapes:
            torch.testing.assert_close(store.view(n).cpu(), tp[n].detach(), rtol=1e-6, atol=1e-7,
                                       msg=n)
        opt.grad_store.data.zero_()
        opt.reduce()
        torch.cuda.synchronize()
        for n in shapes:
            torch.testing.assert_close(opt.grad(n).cpu(), tp[n].grad, rtol=2e-7, atol=1e-9, msg=n)
        runs.append((store.data.clone(), targ.clone(), opt.exp_avg.data.clone(),
                     opt.exp_avg_sq.data.clone()))
    for a, b in zip(*runs):
        assert torch.equal(a, b)


def test_philox_statistics(dev):
    from d3rlpy_amd import ops
    out = torch.zeros(1 << 20, device=dev)
    ctr = torch.zeros(1, dtype=torch.int64, device=dev)
    tk = torch.zeros(1, dtype=torch.int32, device=dev)
    nn_ = 1 << 19
    ops.philox_fill(out, nn_, nn_, -1.0, 1.0, 1234, ctr, tk)
    first = out.clone()
    ops.philox_fill(out, nn_, nn_, -1.0, 1.0, 1234, ctr, tk)
    torch.cuda.synchronize()
    assert int(ctr.item()) == 2 and int(tk.item()) == 0
    n = first[:nn_].double()
    u = first[nn_:].double()
    assert abs(float(n.mean())) < 0.01 and abs(float(n.std()) - 1) < 0.01
    assert float(u.min()) >= -1.0 and float(u.max()) < 1.0 and abs(float(u.mean())) < 0.01
    assert not torch.equal(first, out)  # the counter advanced -> fresh draws


@pytest.mark.parametrize("C,R,r0,n,K0,H,L,J,x_shared", [
    (2, 15616, 0, 15616, 14, 256, 2, 1, True),   # K2 critic pass (padded input rows)
    (2, 15616, 7680, 7936, 14, 256, 2, 1, True),  # critic rows only (r0 > 0)
    (1, 512, 0, 512, 11, 256, 2, 6, True),        # policy on [obs; next_obs]
    (2, 100, 0, 100, 4, 64, 3, 1, True),          # odd rows, 3 hidden layers, H = 64
    (3, 77, 0, 77, 37, 96, 1, 5, False),          # per-member inputs, one hidden layer
    (2, 3000, 0, 3000, 23, 256, 2, 200, True),    # QR critic (200-quantile MFMA head)
])
@pytest.mark.parametrize("bm", [0, 32, 64, 128])
def test_fused_mlp_forward(dev, C, R, r0, n, K0, H, L, J, x_shared, bm, monkeypatch):
    """d3a_mlp_fwd (every layer + head in one launch) against an fp64 torch
    MLP; hidden activations (kept for the backward) checked too, and rows
    below h_from must be left untouched.  Every workgroup shape (bm = rows
    per workgroup; 0 = the library's choice).
    Tolerance 2e-6 relative (exact-f32 MFMA chains, K <= 256)."""
    from d3rlpy_amd import mlp
    from d3rlpy_amd.nets import EnsembleMLP, ParamStore
    monkeypatch.setattr(mlp, "FUSED_MIN_ROWS", 0)  # fused kernel at every size
    monkeypatch.setattr(mlp, "_FUSED_BM", bm)
    g = torch.Generator().manual_seed(R + K0)
    st = ParamStore()
    net = EnsembleMLP(st, "m", C, [K0] + [H] * L + [J])
    st.allocate(dev)
    with torch.no_grad():
        st.data.copy_(torch.randn(st.data.numel(), generator=g) * 0.1)
    ldx = (K0 + 3) // 4 * 4 + 4
    x = torch.randn((1 if x_shared else C), R, ldx, generator=g).to(dev)
    acts = mlp.Acts.alloc(net, R, dev)
    for h in acts.h:
        h.fill_(float("nan"))
    h_from = r0 + n // 3
    assert mlp.fused_ok(net)
    mlp.forward(net, st, x.data_ptr(), x_shared, ldx, acts, r0, r0 + n, h_from=h_from)
    torch.cuda.synchronize()
    k = h_from - r0
    for c in range(C):
        a = x[0 if x_shared else c, r0:r0 + n, :K0].double()
        for l in range(L + 1):
            W, b = net.export_linear(l, c, st)
            a = a @ W.double().T + b.double()
            if l < L:
                a = a.clamp_min(0)
                assert _rel_err(acts.h[l][c, h_from:r0 + n], a[k:]) < 2e-6, (c, l)
                assert torch.isnan(acts.h[l][c, r0:h_from]).all(), (c, l)
        out = acts.out[c, r0:r0 + n] if J == 1 else acts.out[c, r0:r0 + n]
        assert _rel_err(out.reshape(n, J), a) < 2e-6, c


@pytest.mark.parametrize("C,R,r0,n,K0,L,J,x_shared", [
    (1, 512, 0, 512, 11, 2, 6, True),      # CQL policy on [obs; next_obs] (mu | logstd)
    (2, 256, 0, 256, 14, 2, 1, True),      # actor-phase critic pass
    (1, 100, 0, 100, 3, 2, 1, True),       # K1 TD3+BC policy, odd rows
    (3, 77, 5, 60, 37, 1, 5, False),       # per-member inputs, one hidden layer, r0 > 0
    (2, 300, 0, 300, 256, 3, 64, True),    # widest first layer and head, 3 hidden layers
    (2, 256, 0, 256, 23, 2, 200, True),    # K3 QR critics over the batch rows: the MFMA head
    (1, 90, 7, 70, 29, 2, 256, False),     # widest MFMA head, r0 > 0, odd rows
])
def test_small_mlp_forward(dev, C, R, r0, n, K0, L, J, x_shared, monkeypatch):
    """d3a_mlp_fwd block_rows 16 (csrc/mlp_small.hip: 16-row workgroups on
    v_mfma_f32_16x16x4_f32, the small-pass instantiation) against an fp64
    torch MLP, activations kept for rows >= h_from only (2e-6 relative)."""
    from d3rlpy_amd import mlp
    from d3rlpy_amd.nets import EnsembleMLP, ParamStore
    g = torch.Generator().manual_seed(R + K0 + J)
    st = ParamStore()
    net = EnsembleMLP(st, "m", C, [K0] + [256] * L + [J])
    st.allocate(dev)
    with torch.no_grad():
        st.data.copy_(torch.randn(st.data.numel(), generator=g) * 0.1)
    assert mlp.small_ok(net, n)
    ldx = (K0 + 3) // 4 * 4 + 4
    x = torch.randn((1 if x_shared else C), R, ldx, generator=g).to(dev)
    acts = mlp.Acts.alloc(net, R, dev)
    for h in acts.h:
        h.fill_(float("nan"))
    acts.out.fill_(float("nan"))
    h_from = r0 + n // 3
    mlp.forward(net, st, x.data_ptr(), x_shared, ldx, acts, r0, r0 + n, h_from=h_from)
    torch.cuda.synchronize()
    k = h_from - r0
    for c in range(C):
        a = x[0 if x_shared else c, r0:r0 + n, :K0].double()
        for l in range(L + 1):
            W, b = net.export_linear(l, c, st)
            a = a @ W.double().T + b.double()
            if l < L:
                a = a.clamp_min(0)
                assert _rel_err(acts.h[l][c, h_from:r0 + n], a[k:]) < 2e-6, (c, l)
                assert torch.isnan(acts.h[l][c, r0:h_from]).all(), (c, l)
        assert _rel_err(acts.out[c, r0:r0 + n].reshape(n, J), a) < 2e-6, c
        assert torch.isnan(acts.out[c, :r0]).all() and torch.isnan(acts.out[c, r0 + n:]).all()


@pytest.mark.parametrize("bm", [0, 32, 128])
@pytest.mark.parametrize("R,n_aux", [(15616, 256), (4096, 100), (300, 1000)])
def test_fused_mlp_forward_aux_pass(dev, R, n_aux, bm, monkeypatch):
    """d3a_mlp_fwd with an aux pass (a second parameter buffer of the same
    layout over other rows, e.g. the target critics over next-state rows) in
    the same launch: both passes against fp64 torch, the main pass's kept
    activations unchanged by the aux workgroups (2e-6 relative)."""
    from d3rlpy_amd import mlp
    from d3rlpy_amd.nets import EnsembleMLP, ParamStore
    monkeypatch.setattr(mlp, "FUSED_MIN_ROWS", 0)
    monkeypatch.setattr(mlp, "_FUSED_BM", bm)
    g = torch.Generator().manual_seed(R + n_aux)
    C, K0, H, L = 2, 14, 256, 2
    st = ParamStore()
    net = EnsembleMLP(st, "m", C, [K0] + [H] * L + [1])
    st.allocate(dev)
    targ = st.like()
    with torch.no_grad():
        st.data.copy_(torch.randn(st.data.numel(), generator=g) * 0.1)
        targ.data.copy_(torch.randn(st.data.numel(), generator=g) * 0.1)
    ldx = 16
    x = torch.randn(1, R, ldx, generator=g).to(dev)
    x2 = torch.randn(1, n_aux, ldx, generator=g).to(dev)
    acts = mlp.Acts.alloc(net, R, dev)
    acts2 = mlp.Acts.alloc(net, n_aux, dev)
    acts2.out.fill_(float("nan"))
    mlp.forward(net, st, x.data_ptr(), True, ldx, acts, aux=(targ, x2.data_ptr(), ldx, acts2))
    torch.cuda.synchronize()
    for store, xx, a_, rows in ((st, x, acts, R), (targ, x2, acts2, n_aux)):
        for c in range(C):
            a = xx[0, :, :K0].double()
            for l in range(L + 1):
                W, b = net.export_linear(l, c, store)
                a = a @ W.double().T + b.double()
                if l < L:
                    a = a.clamp_min(0)
                    if a_ is acts:
                        assert _rel_err(acts.h[l][c], a) < 2e-6, (c, l)
            assert _rel_err(a_.out[c].reshape(rows, 1), a) < 2e-6, (rows, c)


@pytest.mark.parametrize("R,J,C", [(256, 1, 2), (100, 1, 2), (256, 6, 1), (64, 200, 2)])
def test_per_layer_mlp_forward_aux_pair(dev, R, J, C, monkeypatch):
    """Per-layer forward with an aux pass of the same shape: every layer's GEMM
    (and the row-dot head) carries it as a second batch dimension
    (d3a_gemm_desc.batch2, d3a_rowdot2_f32).  Both passes against fp64 torch
    (2e-6 relative), and bit-identical to the two passes run separately."""
    from d3rlpy_amd import mlp
    from d3rlpy_amd.nets import EnsembleMLP, ParamStore
    monkeypatch.setattr(mlp, "_FUSED", False)
    g = torch.Generator().manual_seed(R + J)
    K0, H, L = 14, 256, 2
    st = ParamStore()
    net = EnsembleMLP(st, "m", C, [K0] + [H] * L + [J])
    st.allocate(dev)
    targ = st.like()
    with torch.no_grad():
        st.data.copy_(torch.randn(st.data.numel(), generator=g) * 0.1)
        targ.data.copy_(torch.randn(st.data.numel(), generator=g) * 0.1)
    ldx = 16
    x = torch.randn(1, R, ldx, generator=g).to(dev)
    x2 = torch.randn(1, R, ldx, generator=g).to(dev)
    acts, acts2 = mlp.Acts.alloc(net, R, dev), mlp.Acts.alloc(net, R, dev)
    mlp.forward(net, st, x.data_ptr(), True, ldx, acts, aux=(targ, x2.data_ptr(), ldx, acts2))
    s1, s2 = mlp.Acts.alloc(net, R, dev), mlp.Acts.alloc(net, R, dev)
    mlp.forward(net, st, x.data_ptr(), True, ldx, s1)
    mlp.forward(net, targ, x2.data_ptr(), True, ldx, s2)
    torch.cuda.synchronize()
    for store, xx, a_, ref in ((st, x, acts, s1), (targ, x2, acts2, s2)):
        for c in range(C):
            a = xx[0, :, :K0].double()
            for l in range(L + 1):
                W, b = net.export_linear(l, c, store)
                a = a @ W.double().T + b.double()
                if l < L:
                    a = a.clamp_min(0)
            assert _rel_err(a_.out[c].reshape(R, J), a) < 2e-6, c
        assert torch.equal(a_.out, ref.out)


@pytest.mark.parametrize("C,R,r0,n,K0,H,L,J,mode", [
    (2, 15616, 7680, 7936, 14, 256, 2, 1, "gscale"),  # K2 critic backward (IS rows scaled)
    (2, 256, 0, 256, 14, 256, 2, 1, "qmin"),          # actor: argmin critic, dQ/dx only
    (1, 512, 0, 256, 11, 256, 2, 6, "vector"),        # policy head backward (first half rows)
    (2, 100, 0, 100, 4, 64, 3, 1, "plain"),           # odd rows, 3 hidden layers
    (1, 77, 0, 77, 37, 96, 1, 5, "vector"),           # one hidden layer
])
def test_fused_mlp_backward(dev, C, R, r0, n, K0, H, L, J, mode, monkeypatch):
    """d3a_mlp_bwd (dz chain + dx in one launch) + split-K weight-gradient
    GEMMs against torch autograd in fp64 on the same forward activations.
    Tolerance 5e-6 relative (max-normalised) per tensor."""
    from d3rlpy_amd import mlp
    from d3rlpy_amd.nets import EnsembleMLP, GradSpace, ParamStore
    monkeypatch.setattr(mlp, "FUSED_MIN_ROWS", 0)
    monkeypatch.setattr(mlp, "_FUSED_BWD", True)
    g = torch.Generator().manual_seed(n + H)
    st = ParamStore()
    net = EnsembleMLP(st, "m", C, [K0] + [H] * L + [J])
    st.allocate(dev)
    with torch.no_grad():
        st.data.copy_(torch.randn(st.data.numel(), generator=g) * 0.1)
    ldx = (K0 + 3) // 4 * 4
    x = torch.randn(R, ldx, generator=g).to(dev)
    acts = mlp.Acts.alloc(net, R, dev)
    mlp.forward(net, st, x.data_ptr(), True, ldx, acts)
    grads = GradSpace(dev) if mode != "qmin" else None
    bs = mlp.BackwardSpace(net, n, grads, dev)
    assert bs.fused
    dout = torch.randn(C, n, J, generator=g).to(dev).squeeze(-1).contiguous()
    gscale = torch.tensor([0.37], device=dev)
    dx = torch.zeros(C, n, K0, device=dev)
    kw = {}
    if mode == "gscale":
        kw = dict(g_scale=gscale.data_ptr(), n_scaled=n // 3)
    if mode == "qmin":
        kw = dict(q_min=acts.out.data_ptr() + 4 * r0, sq_b=R, q_scale=-1.0 / n)
    mlp.backward(bs, st, x.data_ptr(), True, ldx, acts, dout.data_ptr(), J, n * J, r0, n,
                 weight_grads=mode != "qmin", dx=dx, **kw)
    torch.cuda.synchronize()
    # fp64 autograd reference
    xs = x[r0:r0 + n, :K0].double().cpu()
    for c in range(C):
        params = []
        a = xs.clone().requires_grad_(True)
        h = a
        for l in range(L + 1):
            W, b = (t.double().cpu().clone().requires_grad_(True)
                    for t in net.export_linear(l, c, st))
            params.append((W, b))
            h = h @ W.T + b
            if l < L:
                h = h.clamp_min(0)
        if mode == "qmin":
            qall = acts.out[:, r0:r0 + n].double().cpu()
            arg = qall.argmin(0)
            go = torch.where(arg == c, torch.tensor(-1.0 / n, dtype=torch.float64),
                             torch.tensor(0.0, dtype=torch.float64)).view(n, 1)
        else:
            go = dout[c].double().cpu().view(n, J)
            if mode == "gscale":
                go = go.clone()
                go[: n // 3] *= 0.37
        h.backward(go)
        assert _rel_err(dx[c], a.grad) < 5e-6, (c, "dx")
        if mode == "qmin":
            continue
        for l, (W, b) in enumerate(params):
            gW = grads.get(net.wname(l)).sum(0)[c]
            gb = grads.get(net.bname(l)).sum(0)[c]
            assert _rel_err(gW, W.grad) < 5e-6, (c, l, "W")
            assert _rel_err(gb, b.grad) < 5e-6, (c, l, "b")


@pytest.mark.parametrize("C,R,K0,H,J,members", [(2, 256, 23, 256, 200, 1), (2, 256, 23, 256, 200, 2),
                                                (2, 256, 14, 256, 1, 1), (2, 32, 7, 64, 16, 1)])
def test_mlp_input_gradient_member_subset(dev, C, R, K0, H, J, members):
    """Per-layer path: forward + input-gradient backward through the first
    ``members`` ensemble members (the actor's dQ_0/da) against fp64 autograd."""
    from d3rlpy_amd import mlp
    from d3rlpy_amd.nets import EnsembleMLP, ParamStore
    g = torch.Generator().manual_seed(R + J)
    st = ParamStore()
    net = EnsembleMLP(st, "m", C, [K0, H, H, J])
    st.allocate(dev)
    with torch.no_grad():
        st.data.copy_(torch.randn(st.data.numel(), generator=g) * 0.1)
    ldx = (K0 + 3) // 4 * 4
    x = torch.randn(R, ldx, generator=g).to(dev)
    acts = mlp.Acts.alloc(net, R, dev)
    mlp.forward(net, st, x.data_ptr(), True, ldx, acts, members=members)
    bs = mlp.BackwardSpace(net, R, None, dev)
    dout = torch.randn(C, R, J, generator=g).to(dev).squeeze(-1).contiguous()
    dx = torch.zeros(members, R, K0, device=dev)
    if J == 1:
        mlp.backward(bs, st, x.data_ptr(), True, ldx, acts, dout.data_ptr(), 1, R, 0, R,
                     weight_grads=False, dx=dx, members=members)
    else:
        mlp.backward(bs, st, x.data_ptr(), True, ldx, acts, dout.data_ptr(), J, R * J, 0, R,
                     weight_grads=False, dx=dx, members=members)
    torch.cuda.synchronize()
    for c in range(members):
        a = x[:, :K0].double().cpu().requires_grad_(True)
        h = a
        for l in range(3):
            W, b = (t.double().cpu() for t in net.export_linear(l, c, st))
            h = h @ W.T + b
            if l < 2:
                h = h.clamp_min(0)
        h.backward(dout[c].double().cpu().view(R, J))
        assert _rel_err(dx[c], a.grad) < 5e-6, (c, _rel_err(dx[c], a.grad))


@pytest.mark.parametrize("C_,R,n_in,n_out,S", [(1, 256, 256, 256, 8), (2, 256, 256, 256, 8),
                                               (1, 100, 256, 256, 4), (2, 512, 64, 48, 8)])
def test_gemm_pair_bit_identical(dev, C_, R, n_in, n_out, S):
    """d3a_gemm_f32_pair (one backward layer's weight- and input-gradient GEMMs
    submitted together: one launch on the register-direct kernel, or two
    launches where the pair does not fit it) writes exactly what the two
    separate d3a_gemm_f32 launches write."""
    from d3rlpy_amd import ops
    g = torch.Generator().manual_seed(C_ * 1000 + R + n_in)
    dz = torch.randn(C_, R, n_out, generator=g).to(dev)
    h = torch.randn(C_, R, n_in, generator=g).relu().to(dev)
    W = torch.randn(C_, n_out, n_in, generator=g).to(dev)
    outs = []
    for paired in (False, True):
        dW = torch.full((S, C_, n_out, n_in), 12345.0, device=dev)
        db = torch.full((S, C_, n_out), 12345.0, device=dev)
        dx = torch.full((C_, R, n_in), 12345.0, device=dev)

        def w():
            ops.linear_bwd_w(dz.data_ptr(), n_out, R * n_out, h.data_ptr(), n_in, R * n_in,
                             dW.data_ptr(), C_, R, n_in, n_out, S, db=db.data_ptr())

        def x():
            ops.linear_bwd_x(dz.data_ptr(), n_out, R * n_out, W.data_ptr(), dx.data_ptr(), n_in,
                             R * n_in, C_, R, n_in, n_out, mask=h.data_ptr(), ldm=n_in,
                             smb=R * n_in)
        if paired:
            ops.gemm_pair(w, x)
        else:
            w()
            x()
        torch.cuda.synchronize()
        outs.append((dW.cpu(), db.cpu(), dx.cpu()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    # and the pair is right: fp64 reference of dX
    ref = ((dz.double() @ W.double()) * (h > 0)).cpu()
    torch.testing.assert_close(outs[1][2].double(), ref, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("C,R,r0,n,K0,J,x_shared", [
    (1, 512, 0, 512, 11, 6, True),       # CQL policy on [obs; next_obs] (mu | logstd)
    (1, 512, 0, 512, 29, 16, True),      # K4 policy (antmaze 29 -> 2 x 8)
    (2, 300, 7, 200, 64, 5, False),      # widest input, per-member inputs, r0 > 0, ragged
    (1, 256, 0, 256, 23, 24, True),      # K3 VAE encoder (mu | logstd of 12 latents): head in LDS
    (2, 100, 3, 90, 17, 32, False),      # widest parts head, per-member inputs, ragged
])
def test_mlp_forward_parts(dev, C, R, r0, n, K0, J, x_shared):
    """d3a_mlp_fwd parts (the second hidden layer's units split into
    D3A_MLP_PARTS parts, one workgroup per 16 rows, member and part): the head
    parts summed in order against an fp64 torch MLP, kept activations for rows
    >= h_from only (2e-6 relative); rows outside [r0, r0 + n) untouched."""
    from d3rlpy_amd import _native as N
    from d3rlpy_amd import mlp
    from d3rlpy_amd.nets import EnsembleMLP, ParamStore
    g = torch.Generator().manual_seed(R + K0 + J + 1)
    st = ParamStore()
    net = EnsembleMLP(st, "m", C, [K0, 256, 256, J])
    st.allocate(dev)
    with torch.no_grad():
        st.data.copy_(torch.randn(st.data.numel(), generator=g) * 0.1)
    assert mlp.parts_ok(net)
    ldx = (K0 + 3) // 4 * 4 + 4
    x = torch.randn((1 if x_shared else C), R, ldx, generator=g).to(dev)
    acts = mlp.Acts.alloc(net, R, dev)
    for h in acts.h:
        h.fill_(float("nan"))
    parts = torch.full((N.MLP_PARTS, C, R, J), float("nan"), device=dev)
    h_from = r0 + n // 3
    mlp.forward(net, st, x.data_ptr(), x_shared, ldx, acts, r0, r0 + n, h_from=h_from,
                out_parts=parts)
    torch.cuda.synchronize()
    out = parts[0]
    for p in range(1, N.MLP_PARTS):
        out = out + parts[p]
    k = h_from - r0
    for c in range(C):
        a = x[0 if x_shared else c, r0:r0 + n, :K0].double()
        for l in range(3):
            W, b = net.export_linear(l, c, st)
            a = a @ W.double().T + b.double()
            if l < 2:
                a = a.clamp_min(0)
                assert _rel_err(acts.h[l][c, h_from:r0 + n], a[k:]) < 2e-6, (c, l)
                assert torch.isnan(acts.h[l][c, r0:h_from]).all(), (c, l)
        assert _rel_err(out[c, r0:r0 + n], a) < 2e-6, c
        assert torch.isnan(parts[:, c, :r0]).all() and torch.isnan(parts[:, c, r0 + n:]).all()
