"""params.json compatibility (base.py:78-128 _serialize_params /
_deseriealize_params, :186-232 from_json, :823-850 save_params) and
grad-step resume (base.py:1033-1044 set_grad_step).

REFERENCE_CQL_PARAMS is written out by hand from the reference's own code:
the keys save_params collects through get_params (base.py:266-318: every
``_attr`` of the algo minus the excluded ones, ``impl`` skipped), plus
``algorithm`` / ``observation_shape`` / ``action_size``; factories as
{"type", "params"} with the get_params of models/encoders.py:238-250,
:319-324 and models/q_functions.py:117-120; optimiser factories as
models/optimizers.py:55-69; StandardScaler as preprocessing/scalers.py
get_params (mean/std lists through default_json_encoder); use_gpu as the
Device id (argument_utility.check_use_gpu -> Device.get_id)."""
import json
from types import SimpleNamespace

import numpy as np
import pytest

from d3rlpy_amd.algos.cql import CQL
from d3rlpy_amd.algos.td3_plus_bc import TD3PlusBC

REFERENCE_CQL_PARAMS = {
    "action_scaler": None,
    "actor_encoder_factory": {"type": "vector", "params": {
        "hidden_units": [256, 256, 256], "activation": "relu", "use_batch_norm": False,
        "dropout_rate": None, "use_dense": False}},
    "actor_learning_rate": 0.0001,
    "actor_optim_factory": {"optim_cls": "Adam", "betas": [0.9, 0.999], "eps": 1e-08,
                            "weight_decay": 0, "amsgrad": False},
    "alpha_learning_rate": 0.0,
    "alpha_optim_factory": {"optim_cls": "Adam", "betas": [0.9, 0.999], "eps": 1e-08,
                            "weight_decay": 0, "amsgrad": False},
    "alpha_threshold": 10.0,
    "batch_size": 256,
    "conservative_weight": 10.0,
    "critic_encoder_factory": {"type": "default", "params": {
        "activation": "relu", "use_batch_norm": False, "dropout_rate": None}},
    "critic_learning_rate": 0.0003,
    "critic_optim_factory": {"optim_cls": "Adam", "betas": [0.9, 0.999], "eps": 1e-08,
                             "weight_decay": 0, "amsgrad": False},
    "gamma": 0.99,
    "generated_maxlen": 100000,
    "initial_alpha": 1.0,
    "initial_temperature": 1.0,
    "n_action_samples": 10,
    "n_critics": 2,
    "n_frames": 1,
    "n_steps": 1,
    "q_func_factory": {"type": "mean", "params": {"share_encoder": False}},
    "real_ratio": 1.0,
    "reward_scaler": None,
    "scaler": {"type": "standard", "params": {"mean": [[0.5, -1.0, 2.0]],
                                              "std": [[1.0, 2.0, 0.25]], "eps": 0.001}},
    "soft_q_backup": False,
    "tau": 0.005,
    "temp_learning_rate": 0.0001,
    "temp_optim_factory": {"optim_cls": "Adam", "betas": [0.9, 0.999], "eps": 1e-08,
                           "weight_decay": 0, "amsgrad": False},
    "use_gpu": 0,
    "algorithm": "CQL",
    "observation_shape": [3],
    "action_size": 2,
}


def _write(tmp_path, d, name="params.json"):
    p = tmp_path / name
    p.write_text(json.dumps(d, indent=2))
    return str(p)


def test_reference_params_json_configures_the_algo(tmp_path):
    shape, asize, kw = CQL.params_from_json(_write(tmp_path, REFERENCE_CQL_PARAMS))
    assert shape == (3,) and asize == 2
    algo = CQL(**kw)
    assert algo._actor_encoder_factory.hidden_units == [256, 256, 256]
    assert algo._critic_encoder_factory.get_type() == "default"
    assert algo._q_func_factory.get_type() == "mean"
    assert algo._alpha_learning_rate == 0.0 and algo._conservative_weight == 10.0
    assert algo._critic_optim_factory.betas == (0.9, 0.999)
    assert algo._critic_optim_factory.eps == 1e-8
    np.testing.assert_array_equal(np.asarray(algo.scaler._mean).reshape(-1), [0.5, -1.0, 2.0])
    np.testing.assert_array_equal(np.asarray(algo.scaler._std).reshape(-1), [1.0, 2.0, 0.25])


def test_params_json_of_a_related_class_loads(tmp_path):
    """The reference's from_json passes the remaining keys through **kwargs
    without checking ``algorithm`` (base.py:216-232): a params.json written
    for one class configures a subclass too."""
    class MyCQL(CQL):
        pass

    shape, asize, kw = MyCQL.params_from_json(_write(tmp_path, REFERENCE_CQL_PARAMS))
    assert "algorithm" not in kw and shape == (3,)
    algo = MyCQL(**kw)
    assert algo._conservative_weight == 10.0


def test_save_params_writes_the_reference_schema(tmp_path):
    shape, asize, kw = CQL.params_from_json(_write(tmp_path, REFERENCE_CQL_PARAMS))
    algo = CQL(**dict(kw, use_gpu=0))
    # save_params needs only the Impl's shapes
    object.__setattr__(algo, "_impl", SimpleNamespace(observation_shape=shape, action_size=asize))
    out = tmp_path / "out"
    out.mkdir()
    algo.save_params(str(out))
    got = json.loads((out / "params.json").read_text())
    assert set(got) == set(REFERENCE_CQL_PARAMS)
    for k, v in REFERENCE_CQL_PARAMS.items():
        assert got[k] == v, k
    # and it reads back to the same configuration
    shape2, asize2, kw2 = CQL.params_from_json(str(out / "params.json"))
    assert (shape2, asize2) == (shape, asize)
    algo2 = CQL(**kw2)
    for k in ("_tau", "_n_critics", "_batch_size", "_gamma", "_temp_learning_rate"):
        assert getattr(algo2, k) == getattr(algo, k)


def test_set_grad_step():
    algo = TD3PlusBC()
    assert algo.grad_step == 0
    algo.set_grad_step(1233)
    assert algo.grad_step == 1233
