"""The CQL loss stage inside the slice critic backward (d3a_q2_bwd_x6_cql,
cql_impl._LOSS_IN_BWD): every workgroup takes the alpha Adam step itself from
the logsumexp stage's outputs, workgroup 0 the temperature's and the metrics,
and the critic Adam commits the staged scalar state.  At K2 shapes (C B <=
512) its sums run in the loss kernel's order, so whole updates are bitwise the
two-launch path's (d3a_cql_loss's logsumexp + one-workgroup loss stage)."""
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.dirname(__file__))
from cql_helpers import HostBatch, make_batch, make_impl  # noqa: E402

pytestmark = pytest.mark.gpu


def _pair(monkeypatch, **kw):
    from d3rlpy_amd.algos import cql_impl
    impls = []
    for fused in (True, False):
        monkeypatch.setattr(cql_impl, "_LOSS_IN_BWD", fused)
        torch.manual_seed(0)
        impl = make_impl(11, 3, [256, 256], 10, **kw)
        if impls:
            impl.set_state_dict(impls[0].get_state_dict())
        impls.append(impl)
    return impls


def _equal_states(a, b):
    s0, s1 = a.get_state_dict(), b.get_state_dict()
    for k in s0:
        for n in s0[k]:
            if torch.is_tensor(s0[k][n]):
                assert torch.equal(s0[k][n], s1[k][n]), (k, n)
            elif isinstance(s0[k][n], dict):
                for m in s0[k][n]:
                    v0, v1 = s0[k][n][m], s1[k][n][m]
                    if torch.is_tensor(v0):
                        assert torch.equal(v0, v1), (k, n, m)


@pytest.mark.parametrize("kw", [{}, {"alpha_learning_rate": 0.0, "conservative_weight": 10.0},
                                {"temp_learning_rate": 0.0}])
def test_loss_in_backward_is_bitwise_the_loss_launch(monkeypatch, kw):
    """Three injected-noise updates (eager) through each path: metrics and
    every parameter / optimiser state bitwise equal."""
    from d3rlpy_amd.algos import cql_impl
    from oracle.cql import CQLNoise
    impls = _pair(monkeypatch, **kw)
    B, D, A, N_ = 256, 11, 3, 10
    rs = np.random.RandomState(3)
    batches = [HostBatch(*make_batch(rs, B, D, A)) for _ in range(3)]
    gen = torch.Generator().manual_seed(9)
    noises = [CQLNoise.draw(gen, B, A, N_).tensors() for _ in range(3)]
    mets = []
    for impl, fused in zip(impls, (True, False)):
        monkeypatch.setattr(cql_impl, "_LOSS_IN_BWD", fused)
        m = [impl.update_step(b, noise=nz) for b, nz in zip(batches, noises)]
        torch.cuda.synchronize()
        mets.append(m)
    for ma, mb in zip(*mets):
        assert ma == mb, (ma, mb)
    _equal_states(*impls)


def test_loss_in_backward_graph_replays_match(monkeypatch):
    """Graph-replayed steps (device noise, the same seed) through each path:
    bitwise equal parameters, optimiser state and metric ring."""
    from d3rlpy_amd.algos import cql_impl
    impls = _pair(monkeypatch)
    B, D, A = 256, 11, 3
    for impl, fused in zip(impls, (True, False)):
        monkeypatch.setattr(cql_impl, "_LOSS_IN_BWD", fused)
        rs = np.random.RandomState(4)
        ws = impl._workspace(B)
        ws.seed = 777
        ws._build_descs()
        for _ in range(5):
            impl.update_step(HostBatch(*make_batch(rs, B, D, A)))
        torch.cuda.synchronize()
    _equal_states(*impls)
    r0 = next(iter(impls[0]._ws.values())).ring[:5]
    r1 = next(iter(impls[1]._ws.values())).ring[:5]
    assert torch.equal(r0, r1)
