"""CPU checks of the ReLU-decision-aware arbiter itself (tests/relu_arbiter.py):
forcing an evaluation's own decisions reproduces it bit for bit, a forced
flip is reported with its |z| / scale, and merging two data-parallel shards'
decisions reproduces the global batch's."""
import numpy as np
import torch

from arbiter_helpers import module_grads
from cql_helpers import make_batch, make_oracle, oracle_state
from oracle.cql import Batch, CQLNoise
from relu_arbiter import (CriticReluForcer, critic_stage, merge_rank_masks, oracle_from_state,
                          to64)

D, A, H, N, B = 11, 3, [32, 32], 4, 16


def _setup(B=B):
    sd0 = oracle_state(make_oracle(D, A, H, N, seed=3))
    tb = Batch.from_numpy(*make_batch(np.random.RandomState(1), B, D, A))
    nz = CQLNoise.draw(torch.Generator().manual_seed(2), B, A, N)
    return sd0, tb, nz


def _mk():
    return make_oracle(D, A, H, N, seed=0)


def test_forcing_own_decisions_is_bit_identical():
    sd0, tb, nz = _setup()
    o = oracle_from_state(_mk, sd0, torch.float32)
    rec = CriticReluForcer(o._q_func, B, N)
    g = critic_stage(o, tb, nz, rec)
    plain = oracle_from_state(_mk, sd0, torch.float32)
    plain.update_temp(tb, nz.eps_temp)
    plain.update_alpha(tb, nz)
    plain.update_critic(tb, nz)
    g_plain = module_grads(plain._q_func)
    o2 = oracle_from_state(_mk, sd0, torch.float32)
    forced = CriticReluForcer(o2._q_func, B, N, masks=rec.recorded_masks())
    g2 = critic_stage(o2, tb, nz, forced)
    for k in g:
        assert torch.equal(g[k], g_plain[k]), k
        assert torch.equal(g[k], g2[k]), k
    assert forced.tie_report()[0] == 0
    # every block and layer was seen
    for r in rec.recorded:
        assert r["data"] is not None and all(b is not None and len(b) == len(H) for b in r["blocks"])


def test_forced_flip_is_reported_and_moves_the_gradient():
    sd0, tb, nz = _setup()
    o = oracle_from_state(_mk, sd0, torch.float32)
    rec = CriticReluForcer(o._q_func, B, N)
    g = critic_stage(o, tb, nz, rec)
    masks = rec.recorded_masks()
    m = masks[1]["blocks"][2][1].clone()
    m[5, 7] = ~m[5, 7]
    masks[1]["blocks"][2][1] = m
    o2 = oracle_from_state(_mk, sd0, torch.float64)
    f = CriticReluForcer(o2._q_func, B, N, masks=masks)
    g2 = critic_stage(o2, to64(tb), to64(nz), f)
    flips, worst = f.tie_report()
    assert flips == 1 and worst > 0
    k = "_q_funcs.1._encoder._fcs.1.weight"
    assert float((g2[k][7] - g[k][7].double()).abs().max()) > 1e-6
    # critic 0 is untouched by critic 1's flip (fp32 vs fp64 rounding only)
    k0 = "_q_funcs.0._encoder._fcs.1.weight"
    assert float((g2[k0] - g[k0].double()).abs().max()) <= 1e-5 * float(g2[k0].abs().max())


def test_merged_shard_decisions_equal_the_global_batch():
    sd0, tb, nz = _setup(B=2 * B)
    o = oracle_from_state(_mk, sd0, torch.float32)
    full = CriticReluForcer(o._q_func, 2 * B, N)
    critic_stage(o, tb, nz, full)
    shards = []
    for r in range(2):
        sl = slice(r * B, (r + 1) * B)
        tbr = Batch(*(getattr(tb, k)[sl] for k in tb.__dataclass_fields__))
        fields = {}
        for k in nz.__dataclass_fields__:
            v = getattr(nz, k)
            if v is None:
                fields[k] = None
            elif k in ("eps_temp", "eps_actor", "eps_targ"):
                fields[k] = v[sl]
            elif k.endswith("_rand"):
                fields[k] = v.reshape(2 * B, N, A)[sl].reshape(-1, A)
            else:
                fields[k] = v[:, sl]
        orr = oracle_from_state(_mk, sd0, torch.float32)
        fr = CriticReluForcer(orr._q_func, B, N)
        critic_stage(orr, tbr, type(nz)(**fields), fr)
        shards.append(fr.recorded_masks())
    merged = merge_rank_masks(shards)
    ref = full.recorded_masks()
    for c in range(2):
        for l in range(len(H)):
            # layer 0 decisions depend on the inputs only: equal
            if l == 0:
                assert torch.equal(merged[c]["data"][l], ref[c]["data"][l])
                for kb in range(3):
                    assert torch.equal(merged[c]["blocks"][kb][l], ref[c]["blocks"][kb][l])
            assert merged[c]["blocks"][0][l].shape == ref[c]["blocks"][0][l].shape
