"""save_policy on the HIP Impls (GPU): the exported TorchScript greedy policy
reproduces Algo.predict (algos/torch/base.py:87-127) — continuous policies to
2e-6 (plain torch vs the HIP MLP kernels: fp32 summation order only), the
IQN argmax on all but near-tied rows, BCQ (stochastic) in shape and range."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["cql", "sac", "td3", "ddpg", "td3_plus_bc"])
def test_continuous_save_policy_matches_predict(name, tmp_path):
    from d3rlpy_amd.algos import get_algo
    from d3rlpy_amd.datasets import get_synthetic_d4rl
    ds = get_synthetic_d4rl("hopper-medium-v0", n=3000, seed=0)
    kw = {"scaler": "standard"} if name == "td3_plus_bc" else {}
    algo = get_algo(name, discrete=False)(batch_size=64, **kw)
    list(algo.fitter(ds, n_steps=20, n_steps_per_epoch=20, save_metrics=False))
    f = str(tmp_path / "policy.pt")
    algo.save_policy(f)
    m = torch.jit.load(f, map_location="cuda")
    x = ds.observations[:33]
    got = m(torch.as_tensor(x, device="cuda")).cpu().numpy()
    np.testing.assert_allclose(got, algo.predict(x), rtol=2e-6, atol=2e-6)


def test_bcq_save_policy(tmp_path):
    from d3rlpy_amd.algos import BCQ
    from d3rlpy_amd.datasets import get_synthetic_d4rl
    from d3rlpy_amd.factories import QRQFunctionFactory
    ds = get_synthetic_d4rl("halfcheetah-medium-v0", n=3000, seed=0)
    algo = BCQ(batch_size=64, q_func_factory=QRQFunctionFactory(n_quantiles=200))
    algo.build_with_dataset(ds)
    f = str(tmp_path / "bcq.pt")
    algo.save_policy(f)
    a = torch.jit.load(f, map_location="cuda")(torch.as_tensor(ds.observations[:9],
                                                             device="cuda")).cpu().numpy()
    assert a.shape == (9, 6) and np.all(np.abs(a) <= 1.0)


def test_discrete_cql_save_policy(tmp_path):
    from test_gpu_discrete_cql import OBS, make_impl
    impl = make_impl(4)
    f = str(tmp_path / "dcql.pt")
    impl.save_policy(f)
    x = np.random.RandomState(0).randint(0, 256, size=(32,) + OBS).astype(np.uint8)
    got = torch.jit.load(f, map_location="cuda")(
        torch.as_tensor(x, device="cuda").float()).cpu().numpy()
    ref = impl.predict_best_action(x)
    assert got.shape == ref.shape
    assert (got == ref).mean() >= 0.9, (got, ref)
