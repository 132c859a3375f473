"""DiscreteCQL with an IQN Q-function on pixels (K5): HIP DiscreteCQLImpl vs
the CPU oracle restatement (GPU only).

Same initial state (reference checkpoint layout), same uint8 frames, same
injected taus for the five IQN evaluations of an update.  Compared: the loss,
every reduced gradient (max-normalised 2e-5), parameters after Adam (1e-5).
"""
import numpy as np
import pytest
import torch

from cql_helpers import max_rel
from oracle.discrete_cql import DiscreteCQLIQNOracle, IQNTaus, PixelBatch

pytestmark = pytest.mark.gpu

OBS = (4, 84, 84)
TAU_KEYS = ("loss", "cons_lse", "cons_data", "next_online", "next_target")
TAU_FIELDS = {"loss": "loss", "cons_lse": "cons_lse", "cons_data": "cons_data",
              "next_online": "next_online", "next_target": "next_target"}


def make_impl(A=4, lr=6.25e-5):
    from d3rlpy_amd.algos.discrete_cql_impl import DiscreteCQLImpl
    from d3rlpy_amd.factories import AdamFactory, IQNQFunctionFactory, PixelEncoderFactory
    from d3rlpy_amd.preprocessing import PixelScaler
    impl = DiscreteCQLImpl(OBS, A, learning_rate=lr, optim_factory=AdamFactory(),
                           encoder_factory=PixelEncoderFactory(),
                           q_func_factory=IQNQFunctionFactory(), gamma=0.99, n_critics=1,
                           alpha=1.0, use_gpu=0, scaler=PixelScaler(), reward_scaler=None)
    impl.build()
    return impl


def oracle_state(orc):
    p = "_q_funcs.0."
    return {"_q_func": {p + k: v for k, v in orc._q_func.state_dict().items()},
            "_targ_q_func": {p + k: v for k, v in orc._targ_q_func.state_dict().items()},
            "_optim": orc._optim.state_dict()}


class _HB:
    def __init__(self, obs, act, rew, nobs, term, nst):
        self.observations, self.actions = obs, act
        self.rewards, self.next_observations = rew.reshape(-1, 1), nobs
        self.terminals, self.n_steps = term.reshape(-1, 1), nst.reshape(-1, 1)


def _batch(rs, B, A):
    obs = rs.randint(0, 256, size=(B,) + OBS).astype(np.uint8)
    nobs = rs.randint(0, 256, size=(B,) + OBS).astype(np.uint8)
    act = rs.randint(0, A, size=B).astype(np.int32)
    rew = rs.choice([-1.0, 0.0, 1.0], size=B).astype(np.float32)
    term = (rs.rand(B) < 0.1).astype(np.float32)
    return obs, act, rew, nobs, term, np.ones(B, np.float32)


@pytest.mark.parametrize("B", [16, 64])
def test_discrete_cql_iqn_update_parity(B):
    A, K = 4, 64
    torch.set_num_threads(8)
    orc = DiscreteCQLIQNOracle(OBS, A, seed=5)
    impl = make_impl(A)
    rs = np.random.RandomState(1)
    gen = torch.Generator().manual_seed(2)
    for step in range(2):
        impl.set_state_dict(oracle_state(orc))
        obs, act, rew, nobs, term, nst = _batch(rs, B, A)
        taus = IQNTaus.draw(gen, B, K)
        pb = PixelBatch(torch.from_numpy(obs), torch.from_numpy(act).long(),
                        torch.from_numpy(rew).view(-1, 1), torch.from_numpy(nobs),
                        torch.from_numpy(term).view(-1, 1), torch.from_numpy(nst).view(-1, 1))
        lo = orc.update(pb, taus)
        grads = [p.grad.clone() for p in orc._q_func.parameters()]
        m = impl.update_step(_HB(obs, act, rew, nobs, term, nst),
                             taus={k: getattr(taus, k).numpy() for k in TAU_KEYS})
        torch.cuda.synchronize()
        assert abs(m["loss"] - lo) <= 1e-5 * max(1.0, abs(lo)), (step, m, lo)
        worst = 0.0
        for (key, seg, member, sl), g in zip(impl._refs(), grads):
            e = max_rel(impl.grad(seg)[member], g)
            if e > 2e-5:
                print(f"  {key}: rel {e:.2e}")
            worst = max(worst, e)
        sd = impl.get_state_dict()
        ref = oracle_state(orc)
        perr = max(float((sd["_q_func"][k] - t).abs().max()) for k, t in ref["_q_func"].items())
        print(f"[B={B}] step {step}: loss {m['loss']:.6f} vs {lo:.6f}, grad rel {worst:.2e}, "
              f"param abs {perr:.2e}")
        assert worst <= 2e-5
        assert perr <= 1e-5


def test_discrete_cql_graph_replay_and_target_sync():
    """K5 shape (B=512): graph replay == eager bit for bit, and the folded
    hard target sync copies the parameters exactly."""
    A, B = 4, 512
    a = make_impl(A)
    b = make_impl(A)
    b.set_state_dict(a.get_state_dict())
    for impl in (a, b):
        impl._workspace(B).seed = 9
    data = _batch(np.random.RandomState(3), B, A)
    for it in range(3):
        ma = a.update_step(_HB(*data), update_target=it == 1, use_graph=False)
        mb = b.update_step(_HB(*data), update_target=it == 1, use_graph=True)
        assert ma == mb, (it, ma, mb)
        if it == 1:
            torch.cuda.synchronize()
            assert torch.equal(a.targ.data, a.store.data)
    torch.cuda.synchronize()
    assert torch.equal(a.store.data, b.store.data)
    assert np.isfinite(ma["loss"])


def test_discrete_cql_predict_and_checkpoint(tmp_path):
    A = 4
    impl = make_impl(A)
    x = np.random.RandomState(0).randint(0, 256, size=(5,) + OBS).astype(np.uint8)
    act = impl.predict_best_action(x)
    assert act.shape == (5,) and act.min() >= 0 and act.max() < A
    v = impl.predict_value(x, act)
    assert v.shape == (5,) and np.all(np.isfinite(v))
    f = tmp_path / "dcql.pt"
    impl.save_model(str(f))
    orc = DiscreteCQLIQNOracle(OBS, A)
    sd = torch.load(str(f), weights_only=True)
    orc._q_func.load_state_dict({k[len("_q_funcs.0."):]: t for k, t in sd["_q_func"].items()})
    impl2 = make_impl(A)
    impl2.load_model(str(f))
    assert torch.equal(impl2.store.data, impl.store.data)


def test_discrete_cql_taus_in_pack_launch_are_bitwise_the_fill_launch(monkeypatch):
    """K5's taus drawn on the weight-copy launch's appended workgroups
    (d3a_conv_pack_weights_philox, round 6) against their own d3a_philox_fill
    launch: three graph-replayed updates from one state and seed leave the
    parameters, the taus and the draw counter bitwise equal."""
    from d3rlpy_amd.algos import discrete_cql_impl as dci
    A, B = 4, 64
    a = make_impl(A)
    b = make_impl(A)
    b.set_state_dict(a.get_state_dict())
    for impl, fused in ((a, True), (b, False)):
        monkeypatch.setattr(dci, "_PHILOX_IN_PACK", fused)
        impl._workspace(B).seed = 9
        rs = np.random.RandomState(3)
        for it in range(3):
            impl.update_step(_HB(*_batch(rs, B, A)), update_target=False, use_graph=True)
        torch.cuda.synchronize()
    wa, wb = a._workspace(B), b._workspace(B)
    assert torch.equal(wa.taus, wb.taus) and torch.equal(wa.rng_ctr, wb.rng_ctr)
    assert int(wa.rng_ctr.item()) == 3
    assert torch.equal(a.store.data, b.store.data)
