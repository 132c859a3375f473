"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py).

CPU: the oracle reproduces its committed vectors bit-for-bit (guards the
oracle against drift).  GPU (marked): the HIP gather is bit-exact against the
gather fixture, and one HIP CQL update matches the CQL fixture.
"""
import copy
import os

import numpy as np
import pytest
import torch

from oracle import gather as og
from oracle.cql import Batch, CQLNoise, CQLOracle

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    return np.load(os.path.join(HERE, name), allow_pickle=False)


def _state_from(g, prefix):
    keys = ("_q_func", "_targ_q_func", "_policy", "_targ_policy", "_log_temp", "_log_alpha")
    sd = {k: {} for k in keys}
    for f in g.files:
        if f.startswith(prefix):
            k, n = f[len(prefix):].split("/", 1)
            sd[k][n] = torch.from_numpy(g[f])
    return sd


def _oracle_from_fixture(g):
    D, A, H, L, N, B = (int(v) for v in g["cfg"])
    orc = CQLOracle(D, A, n_critics=2, n_action_samples=N, hidden_units=[H] * L, seed=0)
    for k, v in _state_from(g, "init/").items():
        getattr(orc, k).load_state_dict(copy.deepcopy(v))
    return orc, (D, A, H, L, N, B)


def test_oracle_reproduces_cql_fixture():
    g = _load("cql_small.npz")
    orc, (D, A, H, L, N, B) = _oracle_from_fixture(g)
    batch = Batch.from_numpy(g["obs"], g["act"], g["rew"], g["next_obs"], g["term"], g["n_steps"])
    nz = CQLNoise(**{k: torch.from_numpy(g[f"noise/{k}"]) for k in CQLNoise.__dataclass_fields__
                     if f"noise/{k}" in g})
    m = orc.update(batch, nz)
    got = np.array([m["temp_loss"], m["temp"], m["alpha_loss"], m["alpha"], m["critic_loss"],
                    m["actor_loss"]], dtype=np.float32)
    assert np.array_equal(got, g["metrics"])
    final = _state_from(g, "final/")
    for k, sd in final.items():
        for n, t in sd.items():
            assert torch.equal(getattr(orc, k).state_dict()[n], t), (k, n)


def test_oracle_reproduces_gather_fixture():
    g = _load("gather_small.npz")
    trans_v, trans_i = [], []
    eps = og.to_episodes(g["obs"], g["act"], g["rew"], g["term"], g["ep_term"])
    epi = og.to_episodes(g["frames"], g["act"], g["rew"], g["term"], g["ep_term"])
    for (o, a, r, t), (f, _, _, _) in zip(eps, epi):
        trans_v += og.to_transitions(o, a, r, t)
        trans_i += og.to_transitions(f, a, r, t)
    idx = g["idx"]
    for ns in (1, 3):
        b = og.gather([trans_v[i] for i in idx], 1, ns, 0.99)
        for k, v in b.items():
            assert np.array_equal(v, g[f"vec_n{ns}/{k}"]), (ns, k)
    b = og.gather([trans_i[i] for i in idx], 4, 2, 0.99)
    for k, v in b.items():
        assert np.array_equal(v, g[f"img_f4_n2/{k}"]), k


def test_transition_table_matches_oracle_links():
    """d3rlpy_amd's device transition table encodes the reference's links."""
    from d3rlpy_amd.dataset import MDPDataset, transition_table
    g = _load("gather_small.npz")
    ds = MDPDataset(g["obs"], g["act"], g["rew"], g["term"], episode_terminals=g["ep_term"])
    t_row, t_s, t_l, t_t = transition_table(ds.episode_bounds())
    trans = []
    for o, a, r, t in og.to_episodes(g["obs"], g["act"], g["rew"], g["term"], g["ep_term"]):
        trans += og.to_transitions(o, a, r, t)
    assert len(trans) == len(t_row) == 11
    for i, tr in enumerate(trans):
        assert np.array_equal(g["obs"][t_row[i]], tr.observation)
        assert (tr.next is None) == (t_l[i] == i)
        assert bool(t_t[i]) == bool(tr.terminal)
        if not t_t[i]:
            assert np.array_equal(g["obs"][t_row[i] + 1], tr.next_observation)


@pytest.mark.gpu
def test_hip_gather_bit_exact_vs_fixture():
    from d3rlpy_amd.dataset import DeviceDataset, MDPDataset
    g = _load("gather_small.npz")
    idx = torch.from_numpy(g["idx"]).cuda()
    ds = MDPDataset(g["obs"], g["act"], g["rew"], g["term"], episode_terminals=g["ep_term"])
    dd = DeviceDataset(ds)
    for ns in (1, 3):
        out = dd.alloc_batch(len(g["idx"]))
        dd.gather(out, idx, n_steps=ns, gamma=0.99)
        torch.cuda.synchronize()
        pre = f"vec_n{ns}/"
        assert np.array_equal(out.obs.cpu().numpy(), g[pre + "observations"])
        assert np.array_equal(out.next_obs.cpu().numpy(), g[pre + "next_observations"])
        assert np.array_equal(out.act.cpu().numpy(), g[pre + "actions"])
        assert np.array_equal(out.rew.cpu().numpy(), g[pre + "rewards"].ravel())
        assert np.array_equal(out.term.cpu().numpy(), g[pre + "terminals"].ravel())
        assert np.array_equal(out.n_steps.cpu().numpy(), g[pre + "n_steps"].ravel())
    dsi = MDPDataset(g["frames"], g["act"], g["rew"], g["term"], episode_terminals=g["ep_term"])
    ddi = DeviceDataset(dsi)
    out = ddi.alloc_batch(len(g["idx"]), n_frames=4)
    ddi.gather(out, idx, n_steps=2, gamma=0.99, n_frames=4)
    torch.cuda.synchronize()
    assert np.array_equal(out.obs.cpu().numpy(), g["img_f4_n2/observations"])
    assert np.array_equal(out.next_obs.cpu().numpy(), g["img_f4_n2/next_observations"])
    assert np.array_equal(out.rew.cpu().numpy(), g["img_f4_n2/rewards"].ravel())
    assert np.array_equal(out.n_steps.cpu().numpy(), g["img_f4_n2/n_steps"].ravel())


@pytest.mark.gpu
def test_hip_cql_update_vs_fixture():
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from cql_helpers import HostBatch, make_impl, oracle_state
    g = _load("cql_small.npz")
    orc, (D, A, H, L, N, B) = _oracle_from_fixture(g)
    impl = make_impl(D, A, [H] * L, N)
    impl.set_state_dict(oracle_state(orc))
    noise = {k: g[f"noise/{k}"] for k in CQLNoise.__dataclass_fields__ if f"noise/{k}" in g}
    m = impl.update_step(HostBatch(g["obs"], g["act"], g["rew"], g["next_obs"], g["term"],
                                   g["n_steps"]), noise=noise)
    got = np.array([m["temp_loss"], m["temp"], m["alpha_loss"], m["alpha"], m["critic_loss"],
                    m["actor_loss"]])
    assert np.allclose(got, g["metrics"], rtol=1e-5, atol=1e-5)
    sd = impl.get_state_dict()
    for k, d in _state_from(g, "final/").items():
        for n, t in d.items():
            assert float((sd[k][n].view(-1) - t.view(-1)).abs().max()) <= 1e-5, (k, n)


def _td3_from_fixture(g, prefix):
    keys = ("_q_func", "_targ_q_func", "_policy", "_targ_policy")
    sd = {k: {} for k in keys}
    for f in g.files:
        if f.startswith(prefix):
            k, n = f[len(prefix):].split("/", 1)
            sd[k][n] = torch.from_numpy(g[f])
    return sd


def _td3_oracle(g):
    from oracle.td3bc import StandardScalerT, TD3PlusBCOracle
    D, A, H, L, B = (int(v) for v in g["cfg"])
    orc = TD3PlusBCOracle(D, A, n_critics=2, hidden_units=[H] * L,
                          scaler=StandardScalerT(g["scaler_mean"], g["scaler_std"]), seed=0)
    for k, v in _td3_from_fixture(g, "init/").items():
        getattr(orc, k).load_state_dict(copy.deepcopy(v))
    # fresh Adam state, as in the fixture (built right before its first update)
    orc._critic_optim = torch.optim.Adam(orc._q_func.parameters(), lr=3e-4)
    orc._actor_optim = torch.optim.Adam(orc._policy.parameters(), lr=3e-4)
    return orc, (D, A, H, L, B)


def _td3_step_batch(g, step):
    return [g[f"step{step}/{k}"] for k in ("obs", "act", "rew", "next_obs", "term", "n_steps")]


def test_oracle_reproduces_td3bc_fixture():
    g = _load("td3bc_small.npz")
    orc, _ = _td3_oracle(g)
    got = []
    for step in range(2):
        m = orc.update(Batch.from_numpy(*_td3_step_batch(g, step)),
                       torch.from_numpy(g[f"step{step}/noise"]), grad_step=step)
        got.append([m["critic_loss"], m.get("actor_loss", np.nan)])
    assert np.array_equal(np.array(got, dtype=np.float32), g["metrics"], equal_nan=True)
    for k, sd in _td3_from_fixture(g, "final/").items():
        for n, t in sd.items():
            assert torch.equal(getattr(orc, k).state_dict()[n], t), (k, n)


@pytest.mark.gpu
def test_hip_td3bc_updates_vs_fixture():
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from cql_helpers import HostBatch
    from td3_helpers import make_td3_impl
    g = _load("td3bc_small.npz")
    D, A, H, L, B = (int(v) for v in g["cfg"])
    impl = make_td3_impl(D, A, [H] * L, scaler_stats=(g["scaler_mean"], g["scaler_std"]))
    cr, pr = impl._critic_refs(), impl._policy_refs()
    from d3rlpy_amd import checkpoint as ckpt
    init = _td3_from_fixture(g, "init/")
    ckpt.load_module_state(impl.store, cr, init["_q_func"])
    ckpt.load_module_state(impl.targ, cr, init["_targ_q_func"])
    ckpt.load_module_state(impl.store, pr, init["_policy"])
    ckpt.load_module_state(impl.targ, pr, init["_targ_policy"])
    for step in range(2):
        m = impl.update_step(HostBatch(*_td3_step_batch(g, step)), update_actor=step == 0,
                             noise=g[f"step{step}/noise"])
        exp = g["metrics"][step]
        assert abs(m["critic_loss"] - exp[0]) <= 1e-5 * max(1.0, abs(exp[0]))
        if step == 0:
            assert abs(m["actor_loss"] - exp[1]) <= 1e-5 * max(1.0, abs(exp[1]))
    sd = impl.get_state_dict()
    for k, d in _td3_from_fixture(g, "final/").items():
        for n, t in d.items():
            assert float((sd[k][n].view(-1) - t.view(-1)).abs().max()) <= 1e-5, (k, n)


@pytest.mark.gpu
def test_round_iterator_epoch_semantics():
    """RoundIterator (iterators/round_iterator.py:39-53): len = n // batch,
    one epoch visits np.random.shuffle's permutation of the transitions in
    order (global numpy RNG, as the reference), gathered bit-exactly."""
    from d3rlpy_amd.dataset import DeviceDataset, MDPDataset
    from d3rlpy_amd.iterators import RoundIterator
    from oracle.gather import gather, to_episodes, to_transitions
    g = _load("gather_small.npz")
    ds = MDPDataset(g["obs"], g["act"], g["rew"], g["term"], episode_terminals=g["ep_term"])
    dd = DeviceDataset(ds)
    B = 8
    it = RoundIterator(dd, batch_size=B, shuffle=True)
    np.random.seed(5)
    batches = [(b.obs.cpu().numpy().copy(), b.rew.cpu().numpy().copy()) for b in it]
    n = len(dd)
    assert len(it) == n // B and len(batches) == n // B
    np.random.seed(5)
    perm = np.arange(n)
    np.random.shuffle(perm)
    trans = []
    for o, a, r, t in to_episodes(g["obs"], g["act"], g["rew"], g["term"], g["ep_term"]):
        trans += to_transitions(o, a, r, t)
    for k, (obs, rew) in enumerate(batches):
        ref = gather([trans[i] for i in perm[k * B:(k + 1) * B]])
        assert np.array_equal(obs, ref["observations"])
        assert np.array_equal(rew, ref["rewards"].ravel())
