"""save_policy export (algos/torch/base.py:87-127) of the plain-torch greedy
modules (CPU): a traced .pt round trip equals the module, the scaler is
applied in front, bad extensions raise ValueError as in the reference."""
import os

import numpy as np
import pytest
import torch

from d3rlpy_amd.export import (IQNGreedy, TanhMeanPolicy, DeterministicPolicy, conv_from,
                               linear_from, mlp_module, save_traced)
from d3rlpy_amd.nets import EnsembleMLP, ParamStore
from d3rlpy_amd.preprocessing import PixelScaler, StandardScaler

CPU = torch.device("cpu")


def _mlp(sizes, C=1, seed=0):
    st = ParamStore()
    net = EnsembleMLP(st, "m", C, sizes)
    st.allocate(CPU)
    with torch.no_grad():
        st.data.copy_(torch.randn(st.data.numel(), generator=torch.Generator().manual_seed(seed))
                      * 0.2)
    return net, st


def _ref_mlp(net, st, x, member=0):
    h = x
    for l in range(net.n_layers):
        W, b = net.export_linear(l, member, st)
        h = h @ W.T + b
        if l < net.n_layers - 1:
            h = h.clamp_min(0)
    return h


def test_tanh_mean_policy_roundtrip_with_scaler(tmp_path):
    net, st = _mlp([5, 32, 32, 4])
    sc = StandardScaler(mean=np.arange(5, dtype=np.float32), std=np.full(5, 2.0, np.float32))
    f = str(tmp_path / "policy.pt")
    save_traced(TanhMeanPolicy(mlp_module(net, st), 2), (5,), CPU, f, sc)
    m = torch.jit.load(f)
    x = torch.randn(9, 5)
    xs = (x - torch.arange(5.0)) / (2.0 + 1e-3)
    torch.testing.assert_close(m(x), torch.tanh(_ref_mlp(net, st, xs)[:, :2]), rtol=1e-6,
                               atol=1e-6)


def test_deterministic_policy_and_bad_extension(tmp_path):
    net, st = _mlp([3, 16, 1], seed=1)
    f = str(tmp_path / "policy.pt")
    save_traced(DeterministicPolicy(mlp_module(net, st)), (3,), CPU, f)
    x = torch.randn(4, 3)
    torch.testing.assert_close(torch.jit.load(f)(x), torch.tanh(_ref_mlp(net, st, x)))
    with pytest.raises(ValueError):
        save_traced(DeterministicPolicy(mlp_module(net, st)), (3,), CPU,
                    str(tmp_path / "policy.bin"))


def test_iqn_greedy_matches_explicit_computation(tmp_path):
    g = torch.Generator().manual_seed(3)
    geo = [(4, 8, 4), (8, 4, 2), (8, 3, 1)]  # (c_out, k, stride) on a 4x36x36 input
    convs, c = [], 4
    for co, k, s in geo:
        convs.append(conv_from(torch.randn(co, c, k, k, generator=g) * 0.1,
                               torch.randn(co, generator=g) * 0.1, s))
        c = co
    flat = 8 * 1 * 1
    F, E, A, K = 16, 8, 3, 5
    fc = linear_from(torch.randn(F, flat, generator=g) * 0.3, torch.randn(F, generator=g) * 0.1)
    emb = linear_from(torch.randn(F, E, generator=g) * 0.3, torch.randn(F, generator=g) * 0.1)
    head = linear_from(torch.randn(A, F, generator=g) * 0.3, torch.randn(A, generator=g) * 0.1)
    mod = IQNGreedy(torch.nn.ModuleList(convs), fc, emb, head, K, E)
    f = str(tmp_path / "q.pt")
    save_traced(mod, (4, 36, 36), CPU, f, PixelScaler())
    x = torch.randint(0, 256, (6, 4, 36, 36)).float()
    got = torch.jit.load(f)(x)
    # explicit DiscreteIQNQFunction eval forward (iqn_q_function.py:16-47)
    h = x / 255.0
    for conv in convs:
        h = torch.relu(conv(h))
    h = torch.relu(fc(h.reshape(6, -1)))
    taus = torch.linspace(0, 1, K)
    prior = torch.cos(np.pi * torch.arange(1, E + 1).float().view(1, 1, -1) * taus.view(1, -1, 1))
    q = head(h.view(6, 1, -1) * torch.relu(emb(prior))).transpose(1, 2).mean(dim=2)
    assert torch.equal(got, q.argmax(dim=1))
