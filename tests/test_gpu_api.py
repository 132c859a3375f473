"""Algo-level API on the GPU: params.json + save_model -> from_json +
load_model reproduces predict (base.py:186-232); set_grad_step drives
TD3+BC's delayed actor on resume (base.py:1033-1044, td3_plus_bc.py:177-192);
fit after an in-place MDPDataset.extend trains on the new transitions
(the reference rebuilds its transitions from dataset.episodes per fit,
base.py:513-530); fit(scorers, eval_episodes) evaluates each epoch
(base.py:672-673, :806-821)."""
import glob
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_from_json_load_model_reproduces_predict(tmp_path):
    from d3rlpy_amd.algos.cql import CQL
    from d3rlpy_amd.datasets import get_synthetic_d4rl
    ds = get_synthetic_d4rl("hopper-medium-v0", n=3000, seed=0)
    algo = CQL(batch_size=64, scaler="standard")
    list(algo.fitter(ds, n_steps=20, n_steps_per_epoch=20, logdir=str(tmp_path),
                     experiment_name="e", with_timestamp=False, verbose=False))
    logdir = os.path.join(str(tmp_path), "e")
    model = sorted(glob.glob(os.path.join(logdir, "model_*.pt")))[-1]
    algo2 = CQL.from_json(os.path.join(logdir, "params.json"), use_gpu=True)
    algo2.load_model(model)
    x = ds.observations[:17]
    np.testing.assert_array_equal(algo2.predict(x), algo.predict(x))
    np.testing.assert_array_equal(algo2.scaler._mean, algo.scaler._mean)


def test_set_grad_step_drives_the_delayed_actor():
    from d3rlpy_amd.algos.td3_plus_bc import TD3PlusBC
    from d3rlpy_amd.datasets import get_synthetic_d4rl
    from d3rlpy_amd.dataset import DeviceDataset
    from d3rlpy_amd.iterators import RandomIterator
    ds = get_synthetic_d4rl("pendulum-random", n=2000, seed=0)
    algo = TD3PlusBC(batch_size=100, scaler="standard")
    algo.scaler.fit_dataset(ds)
    algo.build_with_dataset(ds)
    it = RandomIterator(DeviceDataset(ds), 10, batch_size=100, seed=3)
    batch = next(iter(it))
    algo.set_grad_step(1)  # odd step: critic only
    m = algo.update(batch)
    assert "actor_loss" not in m or np.isnan(m["actor_loss"])
    assert algo.grad_step == 2
    m = algo.update(batch)  # even step: actor + targets
    assert np.isfinite(m["actor_loss"])


def test_fit_after_extend_uses_the_new_transitions():
    from d3rlpy_amd.algos.cql import CQL
    from d3rlpy_amd.datasets import get_synthetic_d4rl
    ds = get_synthetic_d4rl("hopper-medium-v0", n=2000, episode_len=500, seed=0)
    extra = get_synthetic_d4rl("hopper-medium-v0", n=1000, episode_len=500, seed=1)
    algo = CQL(batch_size=32)
    list(algo.fitter(ds, n_steps=4, n_steps_per_epoch=4, save_metrics=False, verbose=False))
    first = algo._device_dataset_cache[2]
    assert len(first) == 2000
    ds.extend(extra)
    list(algo.fitter(ds, n_steps=4, n_steps_per_epoch=4, save_metrics=False, verbose=False))
    second = algo._device_dataset_cache[2]
    assert second is not first and len(second) == 3000
    # unchanged dataset: the HBM copy is reused
    list(algo.fitter(ds, n_steps=4, n_steps_per_epoch=4, save_metrics=False, verbose=False))
    assert algo._device_dataset_cache[2] is second


def test_fit_evaluates_scorers_each_epoch():
    from d3rlpy_amd.algos.cql import CQL
    from d3rlpy_amd.datasets import get_synthetic_d4rl
    ds = get_synthetic_d4rl("hopper-medium-v0", n=2000, episode_len=500, seed=0)
    calls = []

    def value_scorer(algo, episodes):
        calls.append(len(episodes))
        x = np.concatenate([e.observations for e in episodes])
        return float(np.mean(algo.predict_value(x, algo.predict(x))))

    algo = CQL(batch_size=32)
    res = algo.fit(ds, n_steps=6, n_steps_per_epoch=3, save_metrics=False, verbose=False,
                   scorers={"value": value_scorer}, eval_episodes=ds.episodes[:2])
    assert calls == [2, 2]
    assert [np.isfinite(m["value"]) for _, m in res] == [True, True]
    assert len(algo._eval_results["value"]) == 2
    with pytest.raises(NotImplementedError):
        algo.fit(ds, n_steps=3, n_steps_per_epoch=3, save_metrics=False,
                 tensorboard_dir="tb")
