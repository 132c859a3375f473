"""Pre-split critic weight images (d3a_x6_split, d3a_mlp_fwd_desc.wp): the
split-bf16 x6 Q forward streaming W0 / W1 as bf16 parts formed by an earlier
launch is bitwise the forward that splits the fp32 weights itself, and the CQL
step forms the images inside its sampler launch (d3a_cql_sample_desc.presplit)
from the weights the step's critic forward reads."""
import numpy as np
import pytest
import torch

from d3rlpy_amd import _native as N
from d3rlpy_amd import mlp, ops

pytestmark = pytest.mark.gpu


def split_ref(W: torch.Tensor, kpad: int) -> torch.Tensor:
    """The image of W [rows][k] (fp32) as int16 [rows][kpad / 8][3][8]: p0 =
    bf16(x), p1 = bf16(x - p0), p2 = bf16(x - p0 - p1), fp32 subtractions."""
    rows, k = W.shape
    x = torch.zeros(rows, kpad, dtype=torch.float32, device=W.device)
    x[:, :k] = W
    p0 = x.to(torch.bfloat16)
    r1 = x - p0.float()
    p1 = r1.to(torch.bfloat16)
    p2 = (r1 - p1.float()).to(torch.bfloat16)
    img = torch.stack([p.view(rows, kpad // 8, 8) for p in (p0, p1, p2)], dim=2)
    return img.contiguous().view(torch.int16)


def run_split(jobs):
    d = N.X6SplitDesc()
    for i, (src, dst, rows, k, kpad) in enumerate(jobs):
        j = d.job[i]
        j.src, j.dst, j.rows, j.k, j.kpad = src.data_ptr(), dst.data_ptr(), rows, k, kpad
    d.n_jobs = len(jobs)
    ops.call_desc("d3a_x6_split", d)


@pytest.mark.parametrize("rows,k", [(512, 14), (512, 256), (33, 23), (7, 8), (256, 37)])
def test_x6_split_is_the_exact_split(rows, k):
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(rows * 1000 + k)
    W = (torch.randn(rows, k, generator=g) * torch.logspace(-6, 3, k)).to(dev)
    kpad = (k + 15) // 16 * 16
    img = torch.full((rows * kpad * 3,), -1, dtype=torch.int16, device=dev)
    run_split([(W, img, rows, k, kpad)])
    torch.cuda.synchronize()
    ref = split_ref(W, kpad)
    assert torch.equal(img.view(ref.shape), ref)
    # and the parts sum to the weight exactly (fp64)
    parts = img.view(rows, kpad // 8, 3, 8).view(torch.bfloat16).double()
    tot = parts.sum(dim=2).reshape(rows, kpad)
    assert torch.equal(tot[:, :k], W.double()) and not tot[:, k:].any()


def test_x6_split_several_jobs_in_one_launch():
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(3)
    Ws = [torch.randn(r, k, generator=g).to(dev) for r, k in ((512, 14), (512, 256), (512, 14),
                                                                (512, 256))]
    imgs = [torch.zeros(W.shape[0] * ((W.shape[1] + 15) // 16 * 16) * 3, dtype=torch.int16,
                        device=dev) for W in Ws]
    run_split([(W, im, W.shape[0], W.shape[1], (W.shape[1] + 15) // 16 * 16)
               for W, im in zip(Ws, imgs)])
    torch.cuda.synchronize()
    for W, im in zip(Ws, imgs):
        ref = split_ref(W, (W.shape[1] + 15) // 16 * 16)
        assert torch.equal(im.view(ref.shape), ref)


def _desc_case(rows, h_from, aux, n_in, C=2, seed=0):
    """A q2 forward descriptor over random weights with the mask images on,
    plus the (main, aux) weight images formed by d3a_x6_split."""
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(seed)
    sizes = [n_in, 256, 256, 1]
    ldx = (n_in + 3) // 4 * 4
    stores = []
    for _ in range(2):
        Ws = [torch.randn(C, sizes[l + 1], sizes[l], generator=g) / np.sqrt(sizes[l])
              for l in range(3)]
        bs = [torch.randn(C, sizes[l + 1], generator=g) * 0.1 for l in range(3)]
        stores.append((Ws, bs))
    # one buffer per store, W0 W1 W2 b0 b1 b2, each segment 16-byte aligned
    def pack(Ws, bs):
        segs, offs, o = [], [], 0
        for t in list(Ws) + list(bs):
            f = t.reshape(-1)
            pad = (-f.numel()) % 4
            offs.append(o)
            segs += [f, torch.zeros(pad)]
            o += f.numel() + pad
        return torch.cat(segs), offs
    buf0, offs = pack(*stores[0])
    buf1, _ = pack(*stores[1])
    buf = torch.cat([buf0, buf1]).to(dev)
    x = torch.randn(rows, ldx, generator=g).to(dev)
    xa = torch.randn(max(aux, 1), ldx, generator=g).to(dev)
    xl = (n_in + 15) // 16 * 16
    imgs = []
    for s in range(2):
        base = buf.data_ptr() + 4 * s * buf0.numel()
        w0 = torch.zeros(C * 256 * xl * 3, dtype=torch.int16, device=dev)
        w1 = torch.zeros(C * 256 * 256 * 3, dtype=torch.int16, device=dev)
        d = N.X6SplitDesc()
        for i, (l, im, k, kp) in enumerate(((0, w0, n_in, xl), (1, w1, 256, 256))):
            d.job[i].src, d.job[i].dst = base + 4 * offs[l], im.data_ptr()
            d.job[i].rows, d.job[i].k, d.job[i].kpad = C * 256, k, kp
        d.n_jobs = 2
        ops.call_desc("d3a_x6_split", d)
        imgs.append((w0, w1))

    def run(pre: bool):
        h = [torch.full((C, rows, 256), float("nan"), device=dev) for _ in range(2)]
        out = torch.full((C, rows), float("nan"), device=dev)
        aout = torch.full((C, max(aux, 1)), float("nan"), device=dev)
        hm = torch.zeros(C, rows, 8, dtype=torch.int32, device=dev)
        hmt = torch.zeros(C, (rows + 31) // 32, 256, dtype=torch.int32, device=dev)
        d = N.MlpFwdDesc()
        d.x, d.ldx, d.sxb = x.data_ptr(), ldx, 0
        d.n_in, d.n_hidden, d.H, d.n_out = n_in, 2, 256, 1
        for l in range(3):
            d.W[l] = buf.data_ptr() + 4 * offs[l]
            d.b[l] = buf.data_ptr() + 4 * offs[3 + l]
            d.sW[l], d.sb[l] = sizes[l + 1] * sizes[l], sizes[l + 1]
        for l in range(2):
            d.h[l] = h[l].data_ptr()
        d.sh = rows * 256
        d.out, d.sout, d.ldout = out.data_ptr(), rows, 1
        d.r0, d.rows, d.C, d.h_from = 0, rows, C, h_from
        d.hmask, d.s_hmask = hm.data_ptr(), rows * 8
        d.hmaskT, d.s_hmaskT = hmt.data_ptr(), hmt[0].numel()
        if aux:
            d.aux_x, d.aux_ldx, d.aux_sxb, d.aux_wdelta = xa.data_ptr(), ldx, 0, buf0.numel()
            d.aux_out, d.aux_sout, d.aux_rows = aout.data_ptr(), aux, aux
        if pre:
            d.wp[0], d.wp[1] = imgs[0][0].data_ptr(), imgs[0][1].data_ptr()
            d.aux_wp[0], d.aux_wp[1] = imgs[1][0].data_ptr(), imgs[1][1].data_ptr()
        ops.call_desc("d3a_q2_fwd_x6", d)
        torch.cuda.synchronize()
        return out, aout, h, hm, hmt
    return run


@pytest.mark.parametrize("rows,h_from,aux,n_in", [(15616, 7680, 256, 14), (300, 96, 77, 23),
                                                   (1000, 0, 0, 32), (129, 32, 5, 3)])
def test_presplit_forward_is_bitwise_the_splitting_forward(rows, h_from, aux, n_in):
    run = _desc_case(rows, h_from, aux, n_in, seed=rows + n_in)
    a, b = run(False), run(True)
    for u, v in zip(a[:2] if aux else a[:1], b[:2] if aux else b[:1]):
        assert torch.equal(u, v)
    for u, v in zip(a[2], b[2]):  # kept rows (NaN elsewhere in both)
        assert torch.equal(u[:, h_from:], v[:, h_from:])
        assert torch.isnan(v[:, :h_from]).all()
    assert torch.equal(a[3], b[3]) and torch.equal(a[4], b[4])


def test_cql_step_forms_the_images_of_the_step_weights():
    """The policy forward's presplit workgroups: after update_step, the workspace's
    images are d3a_x6_split of the critic / target weights as they were when
    the step started (the weights its critic forward read)."""
    import sys
    import os
    sys.path.insert(0, os.path.dirname(__file__))
    from cql_helpers import HostBatch, make_batch, make_impl
    D, A, N_, B = 11, 3, 10, 256
    impl = make_impl(D, A, [256, 256], N_)
    rs = np.random.RandomState(0)
    batch = HostBatch(*make_batch(rs, B, D, A))
    impl.update_step(batch)  # builds the workspace, eager first step
    torch.cuda.synchronize()
    ws = next(iter(impl._ws.values()))
    assert ws.wimg is not None
    net = impl.critic
    W = {(si, l): st.view(net.wname(l)).reshape(-1, net.sizes[l]).clone()
         for si, st in enumerate((impl.store, impl.targ)) for l in range(2)}
    impl.update_step(batch)  # the step reads (and splits) W
    torch.cuda.synchronize()
    xl = ws.wimg.xl
    for si in range(2):
        _, w0, w1 = ws.wimg.imgs[si]
        assert torch.equal(w0.view(torch.int16).view(-1), split_ref(W[si, 0], xl).view(-1))
        assert torch.equal(w1.view(torch.int16).view(-1), split_ref(W[si, 1], 256).view(-1))


@pytest.mark.parametrize("hidden", [[256, 256], [256, 256, 256]])
def test_cql_update_presplit_is_bitwise_the_splitting_update(monkeypatch, hidden):
    """Two CQL impls from one state, one with the pre-split forward and one
    without (D3A_X6_PRESPLIT=0's path): three updates leave every parameter
    bitwise equal.  [256, 256, 256]: the CQL reproduction critic, whose
    three-layer d3a_mlp_fwd_x6 streams W1 / W2 from images the sampler forms."""
    import sys
    import os
    sys.path.insert(0, os.path.dirname(__file__))
    from cql_helpers import HostBatch, make_batch, make_impl
    D, A, N_, B = 11, 3, 10, 256
    impls = []
    # (the three-layer critic's stream images are opt-in: D3A_X6_WIDE_PRESPLIT)
    monkeypatch.setattr(mlp, "_WIDE_PRESPLIT", True)
    for pre in (True, False):
        monkeypatch.setattr(mlp, "_PRESPLIT", pre)
        torch.manual_seed(0)
        impl = make_impl(D, A, hidden, N_)
        if impls:
            impl.set_state_dict(impls[0].get_state_dict())
        impls.append(impl)
    rs = np.random.RandomState(1)
    batches = [HostBatch(*make_batch(rs, B, D, A)) for _ in range(3)]
    from oracle.cql import CQLNoise
    gen = torch.Generator().manual_seed(5)
    noises = [CQLNoise.draw(gen, B, A, N_).tensors() for _ in range(3)]
    for impl, pre in zip(impls, (True, False)):
        monkeypatch.setattr(mlp, "_PRESPLIT", pre)
        for b, nz in zip(batches, noises):
            impl.update_step(b, noise=nz)
        torch.cuda.synchronize()
    assert next(iter(impls[0]._ws.values())).wimg is not None
    assert next(iter(impls[1]._ws.values())).wimg is None
    s0, s1 = impls[0].get_state_dict(), impls[1].get_state_dict()
    for k in s0:
        for n in s0[k]:
            a, b = s0[k][n], s1[k][n]
            if torch.is_tensor(a):
                assert torch.equal(a, b), (k, n)
