"""d3a_iqn_embed_head (the IQN head forward in one launch: cosine prior, embed
Linear + ReLU on split-bf16 MFMA, h * phi product and the head Linear) against
the three-launch path it replaces (d3a_iqn_prior + the embed GEMM +
d3a_iqn_head_fwd, fp32 MFMA) and against fp64.

Reference: compute_iqn_feature (iqn_q_function.py:33-47) and
DiscreteIQNQFunction._compute_quantiles (iqn_q_function.py:82-88).  Bars: the
prior is bitwise the standalone kernel's (same fp32 ops); phi within 2e-6 of
fp64 relative to its rounding scale sum_e |prior We| + |be| (fp32-accurate
split products); q within 1e-5 (max-normalised) of fp64."""
import numpy as np
import pytest
import torch

from d3rlpy_amd import _native as N
from d3rlpy_amd import ops

pytestmark = pytest.mark.gpu


def _case(B, K, G, F, A, seed, dev):
    gen = torch.Generator().manual_seed(seed)
    E = 64
    rows = G * B * K
    taus = torch.rand(rows, generator=gen).to(dev)
    We = (torch.randn(F, E, generator=gen) / np.sqrt(E)).to(dev)
    be = (torch.randn(F, generator=gen) * 0.1).to(dev)
    Wf = (torch.randn(A, F, generator=gen) / np.sqrt(F)).to(dev)
    bf = (torch.randn(A, generator=gen) * 0.1).to(dev)
    hs = [torch.relu(torch.randn(B, F, generator=gen)).to(dev) for _ in range(G)]
    return rows, E, taus, We, be, Wf, bf, hs


@pytest.mark.parametrize("B,K,G,F,A,keep_groups", [(512, 64, 4, 512, 4, 3), (512, 64, 1, 512, 4, 0),
                                                   (37, 32, 2, 256, 7, 1), (16, 96, 3, 128, 1, 2)])
def test_iqn_embed_head_matches_three_launches(B, K, G, F, A, keep_groups):
    dev = torch.device("cuda")
    rows, E, taus, We, be, Wf, bf, hs = _case(B, K, G, F, A, B * K + F + A, dev)
    n_keep = keep_groups * B * K
    # the three-launch path
    prior = torch.zeros(rows, E, device=dev)
    p = N.IqnPriorDesc()
    p.taus, p.prior, p.rows, p.E = taus.data_ptr(), prior.data_ptr(), rows, E
    ops.call_desc("d3a_iqn_prior", p)
    phi = torch.zeros(rows, F, device=dev)
    ops.linear_fwd(prior.data_ptr(), True, E, We.data_ptr(), be.data_ptr(), phi.data_ptr(), 1,
                   rows, E, F, relu=True)
    q3 = torch.zeros(rows, A, device=dev)
    hd = N.IqnHeadDesc()
    for g in range(G):
        hd.h[g] = hs[g].data_ptr()
    hd.phi, hd.Wf, hd.bf, hd.q = phi.data_ptr(), Wf.data_ptr(), bf.data_ptr(), q3.data_ptr()
    hd.rows, hd.group_rows, hd.K, hd.F, hd.A = rows, B * K, K, F, A
    ops.call_desc("d3a_iqn_head_fwd", hd)
    # the fused launch
    q1 = torch.full((rows, A), float("nan"), device=dev)
    pr1 = torch.full((max(n_keep, 1), E), float("nan"), device=dev)
    ph1 = torch.full((max(n_keep, 1), F), float("nan"), device=dev)
    d = N.IqnEmbedHeadDesc()
    d.taus, d.We, d.be = taus.data_ptr(), We.data_ptr(), be.data_ptr()
    for g in range(G):
        d.h[g] = hs[g].data_ptr()
    d.Wf, d.bf, d.q = Wf.data_ptr(), bf.data_ptr(), q1.data_ptr()
    d.prior_out = pr1.data_ptr() if n_keep else None
    d.phi_out = ph1.data_ptr() if n_keep else None
    d.rows, d.group_rows, d.n_keep = rows, B * K, n_keep
    d.K, d.E, d.F, d.A = K, E, F, A
    ops.call_desc("d3a_iqn_embed_head", d)
    torch.cuda.synchronize()
    assert not torch.isnan(q1).any()
    if n_keep:
        assert torch.equal(pr1, prior[:n_keep])
        z64 = prior[:n_keep].double() @ We.double().t() + be.double()
        sc = prior[:n_keep].double().abs() @ We.double().abs().t() + be.double().abs()
        e_phi = float(((ph1.double() - z64.clamp_min(0)).abs() / sc).max())
        assert e_phi < 2e-6, e_phi
    # fp64 of the whole head
    z = (prior.double() @ We.double().t() + be.double()).clamp_min(0)
    hrow = torch.cat([hs[g].double().repeat_interleave(K, 0) for g in range(G)])
    q64 = (hrow * z) @ Wf.double().t() + bf.double()
    e1 = float((q1.double() - q64).abs().max() / q64.abs().max())
    e3 = float((q3.double() - q64).abs().max() / q64.abs().max())
    print(f"iqn head vs fp64: fused {e1:.1e}, three launches {e3:.1e}")
    assert e1 < 1e-5 and e3 < 1e-5, (e1, e3)
    # run to run bit-identical
    qa = q1.clone()
    ops.call_desc("d3a_iqn_embed_head", d)
    torch.cuda.synchronize()
    assert torch.equal(qa, q1)


def test_iqn_embed_head_rejects_bad_shapes():
    d = N.IqnEmbedHeadDesc()
    with pytest.raises(RuntimeError, match="null"):
        ops.call_desc("d3a_iqn_embed_head", d)


@pytest.mark.parametrize("B,K,NB", [(512, 64, 2), (37, 32, 3), (16, 96, 1)])
def test_iqn_head_bwd_fused_matches_two_launches(B, K, NB):
    """d3a_iqn_head_bwd_fused against d3a_iqn_head_bwd + the embed weight-
    gradient GEMM (dWe = dphi^T prior) it replaces, and against fp64: dh
    bitwise (the same per-b fma chain), dWf / dbf / dbe summed partials within
    fp32 summation-order noise, dWe within 1e-5 of fp64 (split-bf16 product)."""
    dev = torch.device("cuda")
    G, F, E, A = 3, 512, 64, 4
    gen = torch.Generator().manual_seed(B * 7 + K)
    rows = G * B * K
    h = torch.relu(torch.randn(B, F, generator=gen)).to(dev)
    phi = torch.relu(torch.randn(rows, F, generator=gen)).to(dev)
    prior = torch.cos(torch.rand(rows, E, generator=gen) * 9).to(dev)
    dq = (torch.randn(rows, A, generator=gen) * 1e-3).to(dev)
    Wf = (torch.randn(A, F, generator=gen) / np.sqrt(F)).to(dev)
    # reference: the two launches
    dphi = torch.zeros(rows, F, device=dev)
    dh2 = torch.zeros(B, F, device=dev)
    dWf2, dbf2 = torch.zeros(B, A, F, device=dev), torch.zeros(B, A, device=dev)
    hb = N.IqnHeadBwdDesc()
    hb.h, hb.phi, hb.dq, hb.Wf = h.data_ptr(), phi.data_ptr(), dq.data_ptr(), Wf.data_ptr()
    hb.dphi, hb.dh, hb.dWf_part, hb.dbf_part = dphi.data_ptr(), dh2.data_ptr(), dWf2.data_ptr(), dbf2.data_ptr()
    hb.B, hb.K, hb.F, hb.A, hb.G = B, K, F, A, G
    ops.call_desc("d3a_iqn_head_bwd", hb)
    # fused
    P = (B + NB - 1) // NB
    dh1 = torch.full((B, F), float("nan"), device=dev)
    dWf1, dbf1 = torch.full((P, A, F), float("nan"), device=dev), torch.full((P, A), float("nan"), device=dev)
    dWe1, dbe1 = torch.full((P, F, E), float("nan"), device=dev), torch.full((P, F), float("nan"), device=dev)
    fb = N.IqnHeadBwdFusedDesc()
    fb.h, fb.phi, fb.prior, fb.dq, fb.Wf = (h.data_ptr(), phi.data_ptr(), prior.data_ptr(),
                                            dq.data_ptr(), Wf.data_ptr())
    fb.dh, fb.dWf_part, fb.dbf_part = dh1.data_ptr(), dWf1.data_ptr(), dbf1.data_ptr()
    fb.dWe_part, fb.dbe_part = dWe1.data_ptr(), dbe1.data_ptr()
    fb.B, fb.K, fb.F, fb.E, fb.A, fb.G, fb.NB = B, K, F, E, A, G, NB
    ops.call_desc("d3a_iqn_head_bwd_fused", fb)
    torch.cuda.synchronize()
    assert torch.equal(dh1, dh2)
    rel = lambda a, b: float((a.double() - b.double()).abs().max() / b.double().abs().max())  # noqa: E731
    assert rel(dWf1.sum(0), dWf2.sum(0)) < 1e-6
    assert rel(dbf1.sum(0), dbf2.sum(0)) < 1e-6
    # fp64 of the embed gradients from the reference dphi (exact ops of the kernel)
    dWe64 = dphi.double().t() @ prior.double()
    dbe64 = dphi.double().sum(0)
    e_w = rel(dWe1.double().sum(0), dWe64)
    e_b = rel(dbe1.double().sum(0), dbe64)
    print(f"fused IQN head backward: dWe {e_w:.1e} dbe {e_b:.1e} vs fp64")
    assert e_w < 1e-5 and e_b < 1e-6, (e_w, e_b)


@pytest.mark.parametrize("B,K,F,A,NB", [(512, 64, 512, 4, 4), (37, 32, 512, 7, 3),
                                        (16, 96, 256, 1, 1), (9, 64, 256, 5, 4)])
def test_iqn_head_bwd_recompute_matches_kept_rows(B, K, F, A, NB):
    """d3a_iqn_head_bwd_fused in recompute mode (taus / We / be: prior and phi
    rebuilt from tau in the backward, the forward keeping nothing) against the
    same backward fed the rows d3a_iqn_embed_head kept, and against fp64.
    Bars: dh / dWf / dbf / dbe within 1e-6 (max-normalised; the per-unit sums
    meet across two lane halves instead of one chain), dWe within 1e-5 of fp64
    (split-bf16 product of dphi and the prior)."""
    dev = torch.device("cuda")
    G, E = 3, 64
    rows, _, taus, We, be, Wf, bf, hs = _case(B, K, G, F, A, 3 * B + K + F + A, dev)
    h = hs[0]
    gen = torch.Generator().manual_seed(B + K)
    dq = (torch.randn(rows, A, generator=gen) * 1e-3).to(dev)
    # forward keeping every row (prior / phi for the kept-rows backward)
    q = torch.zeros(rows, A, device=dev)
    prior = torch.zeros(rows, E, device=dev)
    phi = torch.zeros(rows, F, device=dev)
    d = N.IqnEmbedHeadDesc()
    d.taus, d.We, d.be = taus.data_ptr(), We.data_ptr(), be.data_ptr()
    for g in range(G):
        d.h[g] = h.data_ptr()
    d.Wf, d.bf, d.q = Wf.data_ptr(), bf.data_ptr(), q.data_ptr()
    d.prior_out, d.phi_out = prior.data_ptr(), phi.data_ptr()
    d.rows, d.group_rows, d.n_keep = rows, B * K, rows
    d.K, d.E, d.F, d.A = K, E, F, A
    ops.call_desc("d3a_iqn_embed_head", d)
    P = (B + NB - 1) // NB

    phi_rc = torch.full((rows, F), float("nan"), device=dev)

    def run(recompute, dbg=False):
        out = dict(dh=torch.full((B, F), float("nan"), device=dev),
                   dWf=torch.full((P, A, F), float("nan"), device=dev),
                   dbf=torch.full((P, A), float("nan"), device=dev),
                   dWe=torch.full((P, F, E), float("nan"), device=dev),
                   dbe=torch.full((P, F), float("nan"), device=dev))
        fb = N.IqnHeadBwdFusedDesc()
        fb.h, fb.dq, fb.Wf = h.data_ptr(), dq.data_ptr(), Wf.data_ptr()
        if recompute:
            fb.taus, fb.We, fb.be = taus.data_ptr(), We.data_ptr(), be.data_ptr()
            if dbg:
                fb.phi_dbg = phi_rc.data_ptr()
        else:
            fb.phi, fb.prior = phi.data_ptr(), prior.data_ptr()
        fb.dh, fb.dWf_part, fb.dbf_part = out["dh"].data_ptr(), out["dWf"].data_ptr(), out["dbf"].data_ptr()
        fb.dWe_part, fb.dbe_part = out["dWe"].data_ptr(), out["dbe"].data_ptr()
        fb.B, fb.K, fb.F, fb.E, fb.A, fb.G, fb.NB = B, K, F, E, A, G, NB
        ops.call_desc("d3a_iqn_head_bwd_fused", fb)
        torch.cuda.synchronize()
        return out

    rc = run(True)
    for k, v in rc.items():
        assert not torch.isnan(v).any(), k
    rel = lambda a, b: float((a.double() - b.double()).abs().max() / b.double().abs().max())  # noqa: E731
    # fp64 from the kept rows (the forward's phi / prior)
    hrow = torch.cat([h.double().repeat_interleave(K, 0)] * G)
    dprod = dq.double() @ Wf.double()
    dphi = dprod * hrow * (phi.double() > 0)
    dh64 = (dprod * phi.double()).view(G, B, K, F).sum((0, 2)) * (h.double() > 0)
    dWf64 = dq.double().t() @ (hrow * phi.double())
    errs = dict(dh=rel(rc["dh"], dh64), dWf=rel(rc["dWf"].sum(0), dWf64),
                dbf=rel(rc["dbf"].sum(0), dq.double().sum(0)),
                dWe=rel(rc["dWe"].sum(0), dphi.t() @ prior.double()),
                dbe=rel(rc["dbe"].sum(0), dphi.sum(0)))
    print("recompute backward vs fp64:", {k: f"{v:.1e}" for k, v in errs.items()})
    assert errs["dh"] < 1e-6 and errs["dWf"] < 1e-6 and errs["dbf"] < 1e-6, errs
    assert errs["dWe"] < 1e-5 and errs["dbe"] < 1e-6, errs
    if F == 512:
        kept = run(False)
        for k in rc:
            e = rel(rc[k].sum(0) if k != "dh" else rc[k], kept[k].sum(0) if k != "dh" else kept[k])
            assert e < 2e-6, (k, e)
    # run to run bit-identical
    rc2 = run(True)
    for k in rc:
        assert torch.equal(rc[k], rc2[k]), k
    # the recomputed phi -- whose sign is the backward's ReLU mask -- is bitwise
    # the forward's (the reference's autograd uses the saved phi): the same
    # prior, the same six part products in the same order
    rc3 = run(True, dbg=True)
    assert torch.equal(phi_rc, phi), float((phi_rc - phi).abs().max())
    for k in rc:
        assert torch.equal(rc[k], rc3[k]), k


def test_iqn_prior_cos_faithful_on_gpu():
    """d3a_iqn_prior's cosine (iqn_cos, shared by the fused head kernels) on
    the device: within 1 ulp of cos in fp64 over the prior's arguments (the
    host check of the same header: tests/test_iqn_cos.py)."""
    dev = torch.device("cuda")
    E, rows = 64, 1 << 15
    taus = torch.rand(rows, generator=torch.Generator().manual_seed(5)).to(dev)
    taus[:4] = torch.tensor([0.0, 0.5, 0.999999, 0.25])
    prior = torch.zeros(rows, E, device=dev)
    p = N.IqnPriorDesc()
    p.taus, p.prior, p.rows, p.E = taus.data_ptr(), prior.data_ptr(), rows, E
    ops.call_desc("d3a_iqn_prior", p)
    torch.cuda.synchronize()
    ps = (torch.tensor(np.pi, dtype=torch.float32) * torch.arange(1, E + 1, dtype=torch.float32)).to(dev)
    x = ps.view(1, E) * taus.view(rows, 1)          # fp32 products, as the kernel
    ref = torch.cos(x.double())
    rf = ref.float()
    ulp = (torch.nextafter(rf.abs(), torch.full_like(rf, float("inf"))) - rf.abs()).double()
    err = float(((prior.double() - ref).abs() / ulp).max())
    print(f"iqn prior cos: max {err:.3f} ulp")
    assert err < 1.0, err
