"""MDPDataset host utilities (dataset.pyx:330-600): append/extend, stats,
episode returns, dump/load round trip.  CPU only."""
import numpy as np
import pytest

from d3rlpy_amd.dataset import MDPDataset


def _make(n=50, discrete=False, seed=0):
    rng = np.random.default_rng(seed)
    obs = rng.standard_normal((n, 4)).astype(np.float32)
    act = rng.integers(0, 3, n) if discrete else rng.standard_normal((n, 2)).astype(np.float32)
    rew = rng.standard_normal(n).astype(np.float32)
    term = np.zeros(n, np.float32)
    term[9::10] = 1.0
    return MDPDataset(obs, act, rew, term)


def test_episode_returns_and_getitem():
    ds = _make()
    assert len(ds) == 5
    for i, ep in enumerate(ds):
        assert ds[i] is ep
        assert ep.compute_return() == pytest.approx(float(ds.rewards[10 * i:10 * i + 10].sum()),
                                                    rel=1e-6)


def test_append_extend():
    a, b = _make(seed=0), _make(seed=1)
    a.extend(b)
    assert len(a) == 10 and a.observations.shape == (100, 4) and a.actions.shape == (100, 2)
    np.testing.assert_array_equal(a.rewards[50:], b.rewards)
    np.testing.assert_array_equal(a[7].observations, b[2].observations)
    with pytest.raises(AssertionError):
        a.append(np.zeros((3, 5), np.float32), np.zeros((3, 2)), np.zeros(3), np.zeros(3))


def test_append_discrete_warns_on_new_action():
    ds = _make(discrete=True)
    with pytest.warns(UserWarning):
        ds.append(np.zeros((2, 4), np.float32), np.array([5, 5]), np.zeros(2), np.array([0, 1]))
    assert ds.actions.dtype == np.int32 and ds.get_action_size() == 6


@pytest.mark.parametrize("discrete", [False, True])
def test_compute_stats(discrete):
    ds = _make(discrete=discrete)
    st = ds.compute_stats()
    rets = [ep.compute_return() for ep in ds]
    assert st["return"]["mean"] == pytest.approx(np.mean(rets))
    assert st["reward"]["max"] == ds.rewards.max()
    assert st["return"]["histogram"][0].sum() == 5
    np.testing.assert_allclose(st["observation"]["std"], ds.observations.std(axis=0))
    if discrete:
        counts, labels = st["action"]["histogram"]
        assert sum(counts) == 50 and list(labels) == [0, 1, 2]
    else:
        assert len(st["action"]["histogram"]) == 2
        np.testing.assert_allclose(st["action"]["mean"], ds.actions.mean(axis=0))


@pytest.mark.parametrize("discrete", [False, True])
def test_dump_load_roundtrip(tmp_path, discrete):
    ds = _make(discrete=discrete)
    ds._episode_terminals = ds.terminals.copy()
    ds._episode_terminals[24] = 1.0          # a timeout, not a terminal
    f = tmp_path / "ds.npz"
    ds.dump(str(f))
    back = MDPDataset.load(str(f))
    for k in ("observations", "actions", "rewards", "terminals", "episode_terminals"):
        np.testing.assert_array_equal(getattr(back, k), getattr(ds, k))
    assert back.is_action_discrete() == discrete and len(back) == len(ds) == 6
