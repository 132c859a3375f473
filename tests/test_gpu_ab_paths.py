"""The round-5 alternative pipelines against the default ones, same state and
draws: K5 with and without its concurrent graph branches, with the early
head / encoder-fc Adam, and K3 with its (opt-in) graph branches -- the same
kernels in the same per-buffer order, so parameters and metrics bitwise equal;
K3's parts-path small-net forwards against the one-workgroup kernel (head
partial sums added in order: within fp32 rounding)."""
import numpy as np
import pytest
import torch

from cql_helpers import HostBatch
from test_gpu_bcq_parity import BCQNoise, _batch as bcq_batch, make_bcq_impl
from test_gpu_discrete_cql import _HB, _batch as dcql_batch, make_impl as make_dcql

pytestmark = pytest.mark.gpu


def _dcql_run(monkeypatch, branches, early, sd=None):
    from d3rlpy_amd.algos import discrete_cql_impl as m
    monkeypatch.setattr(m, "_K5_BRANCHES", branches)
    monkeypatch.setattr(m, "_K5_EARLY_ADAM", early)
    impl = make_dcql(4)
    if sd is not None:
        impl.set_state_dict(sd)
    impl._workspace(512).seed = 9
    data = dcql_batch(np.random.RandomState(3), 512, 4)
    ms = [impl.update_step(_HB(*data), update_target=it == 1, use_graph=it > 0) for it in range(3)]
    torch.cuda.synchronize()
    return impl, ms


def test_k5_branches_and_early_adam_are_bitwise_the_single_stream(monkeypatch):
    a = make_dcql(4)
    sd = a.get_state_dict()
    base, m0 = _dcql_run(monkeypatch, False, False, sd)
    for branches, early in ((True, False), (True, True)):
        other, m1 = _dcql_run(monkeypatch, branches, early, sd)
        assert m0 == m1, (branches, early, m0, m1)
        assert torch.equal(base.store.data, other.store.data), (branches, early)
        assert torch.equal(base.targ.data, other.targ.data), (branches, early)


def _bcq_run(monkeypatch, branches, parts, sd):
    from d3rlpy_amd.algos import bcq_impl as m
    monkeypatch.setattr(m, "_BRANCHES", branches)
    monkeypatch.setattr(m, "_PARTS", parts)
    D, A, H, N, K, B = 17, 6, [256, 256], 100, 200, 256
    impl = make_bcq_impl(D, A, H, N, K)
    impl.set_state_dict(sd)
    rs = np.random.RandomState(4)
    ms = []
    for step in range(3):
        arrs = bcq_batch(rs, B, D, A)
        nz = BCQNoise.draw(torch.Generator().manual_seed(step), B, A, N)
        noise = {k: getattr(nz, k).numpy() for k in ("eps_vae", "z_target", "z_actor")}
        ms.append(impl.update_step(HostBatch(*arrs), noise=noise))
    torch.cuda.synchronize()
    return impl, ms


def test_k3_branches_bitwise_and_parts_within_rounding(monkeypatch):
    D, A, H, N, K = 17, 6, [256, 256], 100, 200
    sd = make_bcq_impl(D, A, H, N, K).get_state_dict()
    base, m0 = _bcq_run(monkeypatch, False, True, sd)
    br, m1 = _bcq_run(monkeypatch, True, True, sd)
    assert m0 == m1
    assert torch.equal(base.store.data, br.store.data)
    small, m2 = _bcq_run(monkeypatch, False, False, sd)
    for a, b in zip(m0, m2):
        for k in a:
            assert abs(a[k] - b[k]) <= 1e-5 * max(1.0, abs(b[k])), (k, a[k], b[k])
    d = (base.store.data - small.store.data).abs().max().item()
    print(f"parts vs one-workgroup small-net forwards: max param diff {d:.2e} after 3 steps")
    assert d <= 1e-5
