"""The minibatch sampler on the GPU: RandomIterator's two index streams and
the gather (iterators/random_iterator.py:38-41, tests/iterators/
test_random_iterator.py:16-88, dataset.pyx:1139-1342).

* index_source="numpy": exactly the reference's stream — one
  ``np.random.randint(len(transitions))`` per sample from numpy's global RNG —
  and a data-parallel shard takes its slice of one global draw; the gathered
  batch is bit-identical to the oracle's TransitionMiniBatch of those indices.
* index_source="device" (Philox, the default): indices in range, uniform over
  transitions (chi-square), rank k's rows (row_offset = k*B) are slice k of
  the world-1 draw of the same step, each step's draw is fresh, and the batch
  gathered from the drawn indices is bit-identical to the oracle's.
* n-step returns with a discount whose powf differs from the rounded fp64
  power (gamma 0.95, n 60; tests/test_nstep_pin.py) stay bit-exact.
"""
import numpy as np
import pytest
import torch

from oracle import gather as og

pytestmark = pytest.mark.gpu


def _data(n=3000, D=5, A=2, ep=250, seed=0):
    from d3rlpy_amd.datasets import synthetic_arrays
    from d3rlpy_amd.dataset import MDPDataset
    obs, act, rew, term = synthetic_arrays(n, D, A, ep, seed)
    ds = MDPDataset(obs, act, rew, term)
    trans = []
    for o, a, r, t in og.to_episodes(obs, act, rew, term):
        trans += og.to_transitions(o, a, r, t)
    return ds, trans


def _check_batch(out, trans, idx, n_steps=1, gamma=0.99):
    ref = og.gather([trans[i] for i in idx], 1, n_steps, gamma)
    assert np.array_equal(out.obs.cpu().numpy(), ref["observations"])
    assert np.array_equal(out.act.cpu().numpy(), ref["actions"])
    assert np.array_equal(out.rew.cpu().numpy(), ref["rewards"].ravel())
    assert np.array_equal(out.next_obs.cpu().numpy(), ref["next_observations"])
    assert np.array_equal(out.term.cpu().numpy(), ref["terminals"].ravel())
    assert np.array_equal(out.n_steps.cpu().numpy(), ref["n_steps"].ravel())


def test_numpy_stream_is_the_reference_stream():
    from d3rlpy_amd.dataset import DeviceDataset
    from d3rlpy_amd.iterators import RandomIterator
    ds, trans = _data()
    dd = DeviceDataset(ds)
    assert len(dd) == len(trans)
    B = 64
    it = RandomIterator(dd, 5, batch_size=B, index_source="numpy")
    np.random.seed(123)
    got = []
    for batch in it:
        idx = it.indices.cpu().numpy()
        got.append(idx)
        _check_batch(batch, trans, idx)
    np.random.seed(123)
    want = [np.array([np.random.randint(len(trans)) for _ in range(B)]) for _ in range(5)]
    assert all(np.array_equal(a, b) for a, b in zip(got, want))
    assert len(it) == 5


def test_numpy_stream_shards_one_global_draw():
    from d3rlpy_amd.dataset import DeviceDataset
    from d3rlpy_amd.iterators import RandomIterator
    ds, trans = _data()
    dd = DeviceDataset(ds)
    B, W = 32, 4
    np.random.seed(5)
    glob = [np.array([np.random.randint(len(trans)) for _ in range(B * W)]) for _ in range(3)]
    for k in range(W):
        np.random.seed(5)
        it = RandomIterator(dd, 3, batch_size=B, index_source="numpy", seed=0, shard=(k, W))
        for s, batch in enumerate(it):
            idx = it.indices.cpu().numpy()
            assert np.array_equal(idx, glob[s][k * B:(k + 1) * B])
            _check_batch(batch, trans, idx)


def test_device_stream_range_uniformity_and_batches():
    from scipy.stats import chisquare
    from d3rlpy_amd.dataset import DeviceDataset
    from d3rlpy_amd.iterators import RandomIterator
    ds, trans = _data(n=1000, ep=100)
    dd = DeviceDataset(ds)
    n, B, S = len(trans), 512, 200
    it = RandomIterator(dd, S, batch_size=B, seed=77)
    counts = np.zeros(n, np.int64)
    prev = None
    for s, batch in enumerate(it):
        idx = it.indices.cpu().numpy()
        assert idx.min() >= 0 and idx.max() < n
        counts += np.bincount(idx, minlength=n)
        if prev is not None:
            assert not np.array_equal(idx, prev)  # a fresh draw every step
        prev = idx
        if s < 3:
            _check_batch(batch, trans, idx)
    p = chisquare(counts).pvalue
    print(f"device stream: {S * B} draws over {n} transitions, chi-square p = {p:.3f}")
    assert p > 1e-4


def test_device_stream_shards_equal_slices_of_the_world1_draw():
    from d3rlpy_amd.dataset import DeviceDataset
    ds, _ = _data()
    W, B = 4, 64
    dd_all = DeviceDataset(ds)
    out = dd_all.alloc_batch(B * W)
    idx_all = torch.zeros(B * W, dtype=torch.int64, device="cuda")
    steps_all = []
    for _ in range(3):
        dd_all.gather(out, None, seed=99, idx_out=idx_all)
        steps_all.append(idx_all.cpu().numpy().copy())
    for k in range(W):
        dd = DeviceDataset(ds)  # fresh sampler counter, as every rank starts
        o = dd.alloc_batch(B)
        idx = torch.zeros(B, dtype=torch.int64, device="cuda")
        for s in range(3):
            dd.gather(o, None, seed=99, idx_out=idx, row_offset=k * B)
            assert np.array_equal(idx.cpu().numpy(), steps_all[s][k * B:(k + 1) * B]), (k, s)


def test_gather_nstep_with_powf_discount():
    """gamma 0.95 with n_steps 60 reaches powf(0.95, 58), which differs from
    the correctly rounded power: the kernel must use the host's powf table."""
    from d3rlpy_amd.dataset import DeviceDataset
    ds, trans = _data(n=600, ep=200, seed=3)
    dd = DeviceDataset(ds)
    idx_np = np.arange(0, len(trans), 7)
    out = dd.alloc_batch(len(idx_np))
    dd.gather(out, torch.from_numpy(idx_np).cuda(), n_steps=60, gamma=0.95)
    torch.cuda.synchronize()
    _check_batch(out, trans, idx_np, n_steps=60, gamma=0.95)
