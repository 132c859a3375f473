"""The C-ABI registered as PyTorch custom ops (SURVEY §8(b) "registered
through TORCH_LIBRARY"): libd3rlpy_amd_torch.so / torch.ops.d3rlpy_amd.

CPU (no GPU needed): the library loads, every op has its schema, and the
Meta implementations give torch.export / FakeTensor the output shapes.
GPU: each op against the ctypes path or plain torch (fp32 tolerance for the
GEMMs, bit-exact for gather / soft update / Adam), TorchScript scripting and a
save -> load round trip of a module calling the op, torch.export of it, and
save_policy(hip_ops=True) reproducing predict()."""
import numpy as np
import pytest
import torch

from d3rlpy_amd import torch_ops

SCHEMAS = {
    "linear": "d3rlpy_amd::linear(Tensor x, Tensor W, Tensor b, bool relu) -> Tensor",
    "mlp_forward": "d3rlpy_amd::mlp_forward(Tensor x, Tensor[] Ws, Tensor[] bs) -> Tensor",
    "standardize": "d3rlpy_amd::standardize(Tensor x, Tensor mean, Tensor std, float eps) -> "
                   "Tensor",
    "soft_update_": "d3rlpy_amd::soft_update_(Tensor(a!) targ, Tensor src, float tau) -> ()",
}


# the §8(b) loss / sampling / backward ops (reference call sites in
# csrc/torch_ops.cpp): every one has a HIP and a Meta kernel
OPS_8B = ("linear_backward", "mlp_backward", "logsumexp", "logsumexp_backward", "td_mse_loss",
          "td_mse_loss_backward", "quantile_huber_loss", "quantile_huber_loss_backward",
          "iqn_cos_embed", "iqn_cos_embed_backward", "squashed_gaussian_sample",
          "squashed_gaussian_sample_backward")


def test_ops_registered_with_schemas():
    ops = torch_ops.load()
    for name, schema in SCHEMAS.items():
        assert str(getattr(ops, name).default._schema) == schema
    for name in ("adam_step_", "gather_batch") + OPS_8B:
        assert hasattr(ops, name), name
        assert torch._C._dispatch_has_kernel_for_dispatch_key(f"d3rlpy_amd::{name}", "CUDA")
        assert torch._C._dispatch_has_kernel_for_dispatch_key(f"d3rlpy_amd::{name}", "Meta")


def test_update_step_ops_registered():
    """The shipped Impls replay their captured update pipelines through
    torch.ops.d3rlpy_amd.cql_update_step / update_step (ops.replay_update)."""
    ops = torch_ops.load()
    for name in ("cql_update_step", "update_step"):
        assert str(getattr(ops, name).default._schema) == (
            f"d3rlpy_amd::{name}(int graph_exec, Tensor(a!)[] state) -> ()")
        assert torch._C._dispatch_has_kernel_for_dispatch_key(f"d3rlpy_amd::{name}", "CUDA")


def test_meta_shapes_of_loss_and_backward_ops():
    ops = torch_ops.load()
    m = lambda *s: torch.empty(*s, device="meta")  # noqa: E731
    dx, dW, db = ops.linear_backward(m(2, 9, 256), m(9, 14), m(2, 256, 14), m(2, 9, 256))
    assert (dx.shape, dW.shape, db.shape) == ((2, 9, 14), (2, 256, 14), (2, 256))
    out = ops.mlp_backward(m(9, 1), m(9, 14), [m(256, 14), m(256, 256), m(1, 256)],
                           [m(9, 256), m(9, 256)])
    assert [tuple(t.shape) for t in out] == [(9, 14), (256, 14), (256, 256), (1, 256), (256,),
                                             (256,), (1,)]
    assert ops.logsumexp(m(2, 32, 30)).shape == (2, 32)
    assert ops.logsumexp_backward(m(2, 32), m(2, 32, 30), m(2, 32)).shape == (2, 32, 30)
    loss, diff = ops.td_mse_loss(m(2, 32), m(32), m(2, 32), m(32), m(32))
    assert loss.shape == (2,) and diff.shape == (2, 32)
    assert ops.td_mse_loss_backward(m(2), m(2, 32)).shape == (2, 32)
    assert ops.quantile_huber_loss(m(8, 200), m(8, 200), m(8, 200)).shape == (8,)
    assert ops.quantile_huber_loss_backward(m(8), m(8, 200), m(8, 200), m(8, 200)).shape == \
        (8, 200)
    assert ops.iqn_cos_embed(m(8, 64), m(3136, 64), m(3136)).shape == (512, 3136)
    dW, db = ops.iqn_cos_embed_backward(m(512, 3136), m(8, 64), m(512, 3136), m(3136, 64))
    assert dW.shape == (3136, 64) and db.shape == (3136,)
    a, lp = ops.squashed_gaussian_sample(m(16, 3), m(16, 3), m(16, 3), -20.0, 2.0)
    assert a.shape == (16, 3) and lp.shape == (16, 1)
    dmu, dls = ops.squashed_gaussian_sample_backward(m(16, 3), m(16, 1), m(16, 3), m(16, 3),
                                                     m(16, 3), -20.0, 2.0)
    assert dmu.shape == dls.shape == (16, 3)


def test_meta_shapes():
    ops = torch_ops.load()
    m = lambda *s: torch.empty(*s, device="meta")  # noqa: E731
    assert ops.linear(m(9, 14), m(2, 256, 14), m(2, 256), True).shape == (2, 9, 256)
    assert ops.linear(m(9, 14), m(256, 14), m(256), False).shape == (9, 256)
    y = ops.mlp_forward(m(9, 11), [m(256, 11), m(256, 256), m(6, 256)], [m(256), m(256), m(6)])
    assert y.shape == (9, 6)
    out = ops.gather_batch(m(100, 11), m(100, 3), m(100), torch.empty(90, dtype=torch.long,
                                                                        device="meta"),
                           torch.empty(90, dtype=torch.long, device="meta"),
                           torch.empty(90, dtype=torch.long, device="meta"),
                           torch.empty(90, dtype=torch.uint8, device="meta"),
                           torch.empty(32, dtype=torch.long, device="meta"), 1, 0.99)
    assert [tuple(t.shape) for t in out] == [(32, 11), (32, 3), (32,), (32, 11), (32,), (32,)]


def test_export_sees_the_op():
    ops = torch_ops.load()

    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.W = torch.nn.Parameter(torch.randn(4, 3))
            self.b = torch.nn.Parameter(torch.randn(4))

        def forward(self, x):
            return ops.linear(x, self.W, self.b, True)

    with torch.device("meta"):
        mod = M()
        ep = torch.export.export(mod, (torch.empty(5, 3),))
    assert "d3rlpy_amd.linear" in str(ep.graph)


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_linear_and_mlp_match_torch():
    ops = torch_ops.load()
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(300, 14, device="cuda", generator=g)
    W = torch.randn(2, 256, 14, device="cuda", generator=g) * 0.2
    b = torch.randn(2, 256, device="cuda", generator=g)
    y = ops.linear(x, W, b, True)
    ref = torch.relu(torch.einsum("ri,coi->cro", x.double(), W.double()) + b.double()[:, None])
    assert torch.allclose(y.double(), ref, rtol=1e-5, atol=1e-5)
    Ws = [W[0], torch.randn(256, 256, device="cuda", generator=g) * 0.06,
          torch.randn(1, 256, device="cuda", generator=g) * 0.06]
    bs = [b[0], torch.randn(256, device="cuda", generator=g), torch.randn(1, device="cuda",
                                                                          generator=g)]
    q = ops.mlp_forward(x, Ws, bs)
    h = x.double()
    for l, (Wl, bl) in enumerate(zip(Ws, bs)):
        h = h @ Wl.double().T + bl.double()
        if l < 2:
            h = torch.relu(h)
    assert torch.allclose(q.double(), h, rtol=1e-5, atol=1e-5)
    with pytest.raises(RuntimeError):
        ops.linear(x, W[:, :, :5].contiguous(), b, True)  # TORCH_CHECK on the shapes


@pytest.mark.gpu
def test_soft_update_standardize_adam_bit_exact():
    from d3rlpy_amd import ops as nat
    ops = torch_ops.load()
    g = torch.Generator(device="cuda").manual_seed(1)
    targ = torch.randn(5000, device="cuda", generator=g)
    src = torch.randn(5000, device="cuda", generator=g)
    t2 = targ.clone()
    ops.soft_update_(targ, src, 0.005)
    nat.soft_update(t2, src, 0.005)
    assert torch.equal(targ, t2)
    x = torch.randn(64, 11, device="cuda", generator=g)
    mean, std = torch.randn(11, device="cuda", generator=g), torch.rand(11, device="cuda") + 0.5
    y = ops.standardize(x, mean, std, 1e-3)
    y2 = torch.empty_like(x)
    nat.standardize(x, y2, mean, std, 1e-3)
    assert torch.equal(y, y2)
    # one torch.optim.Adam step
    p = torch.randn(3000, device="cuda", generator=g)
    grad = torch.randn(3000, device="cuda", generator=g)
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    step = torch.zeros(1, dtype=torch.long, device="cuda")
    pt = torch.nn.Parameter(p.cpu().clone())
    opt = torch.optim.Adam([pt], lr=3e-4, foreach=False)
    for _ in range(2):
        ops.adam_step_(p, m, v, grad, step, 3e-4, 0.9, 0.999, 1e-8)
        pt.grad = grad.cpu().clone()
        opt.step()
    torch.cuda.synchronize()
    assert int(step.item()) == 2
    assert float((p.cpu() - pt.detach()).abs().max()) <= 1e-7


@pytest.mark.gpu
def test_gather_batch_matches_device_dataset():
    from d3rlpy_amd.dataset import DeviceDataset
    from d3rlpy_amd.datasets import get_synthetic_d4rl
    ops = torch_ops.load()
    dd = DeviceDataset(get_synthetic_d4rl("hopper-medium-v0", n=4000, episode_len=300, seed=1))
    idx = torch.randint(0, len(dd), (128,), device="cuda")
    for ns, gamma in ((1, 0.99), (3, 0.95)):
        out = dd.alloc_batch(128)
        dd.gather(out, idx, n_steps=ns, gamma=gamma)
        got = ops.gather_batch(dd.obs, dd.act, dd.rew, dd.t_row, dd.t_ep_start, dd.t_ep_last,
                               dd.t_terminal, idx, ns, gamma)
        for a, b in zip(got, (out.obs, out.act, out.rew, out.next_obs, out.term, out.n_steps)):
            assert torch.equal(a.view(-1), b.reshape(-1))


@pytest.mark.gpu
def test_torchscript_roundtrip_and_save_policy(tmp_path):
    from d3rlpy_amd.algos.cql import CQL
    from d3rlpy_amd.datasets import get_synthetic_d4rl
    from d3rlpy_amd.export import HipMLP
    torch_ops.load()
    g = torch.Generator(device="cuda").manual_seed(2)
    mlp = HipMLP([torch.randn(32, 5, device="cuda", generator=g),
                  torch.randn(2, 32, device="cuda", generator=g)],
                  [torch.randn(32, device="cuda", generator=g),
                   torch.randn(2, device="cuda", generator=g)])
    s = torch.jit.script(mlp)
    f = str(tmp_path / "m.pt")
    s.save(f)
    x = torch.randn(7, 5, device="cuda", generator=g)
    assert torch.equal(torch.jit.load(f, map_location="cuda")(x), mlp(x))
    ds = get_synthetic_d4rl("hopper-medium-v0", n=3000, seed=0)
    algo = CQL(batch_size=64)
    list(algo.fitter(ds, n_steps=10, n_steps_per_epoch=10, save_metrics=False, verbose=False))
    fp = str(tmp_path / "policy.pt")
    algo.save_policy(fp, hip_ops=True)
    prog = torch.jit.load(fp, map_location="cuda")
    assert "d3rlpy_amd::mlp_forward" in str(prog.inlined_graph)
    xo = ds.observations[:33]
    got = prog(torch.as_tensor(xo, device="cuda")).cpu().numpy()
    np.testing.assert_allclose(got, algo.predict(xo), rtol=2e-6, atol=2e-6)


@pytest.mark.gpu
def test_cql_impl_replays_through_the_update_step_op(monkeypatch):
    """CQLImpl.update_step's graph replays go through the custom op, and three
    replayed steps are bitwise the CUDAGraph.replay path's (D3A_OP_REPLAY=0)."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    from cql_helpers import HostBatch, make_batch, make_impl
    from d3rlpy_amd import ops as dops
    D, A, N_, B = 11, 3, 10, 256
    calls = []
    real = dops.replay_update

    def spy(g, state, cql=False):
        calls.append((dops._OP_REPLAY, cql, len(state)))
        real(g, state, cql)
    monkeypatch.setattr(dops, "replay_update", spy)
    impls = []
    for via_op in (True, False):
        torch.manual_seed(0)
        impl = make_impl(D, A, [256, 256], N_)
        if impls:
            impl.set_state_dict(impls[0][0].get_state_dict())
        impls.append((impl, via_op))
    for impl, via_op in impls:
        monkeypatch.setattr(dops, "_OP_REPLAY", via_op)
        rs = np.random.RandomState(2)
        ws = impl._workspace(B)
        ws.seed = 1234  # both impls draw the same device noise
        ws._build_descs()
        for _ in range(4):  # eager, capture + replay, replay, replay
            impl.update_step(HostBatch(*make_batch(rs, B, D, A)))
        torch.cuda.synchronize()
    assert any(c[0] and c[1] and c[2] > 8 for c in calls)
    s0, s1 = impls[0][0].get_state_dict(), impls[1][0].get_state_dict()
    for k in s0:
        for n in s0[k]:
            if torch.is_tensor(s0[k][n]):
                assert torch.equal(s0[k][n], s1[k][n]), (k, n)
