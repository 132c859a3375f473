"""The conservative term's softmax weights, pinned against fp64.

d3a_cql_loss forms the importance-sampled rows' dL/dQ weights as
exp(v_j - max) / sum_j exp(v_j - max) (csrc/cql.hip cql_lse_wave), where
torch.logsumexp's backward -- the reference's arithmetic (cql_impl.py:101-138
via torch.logsumexp) -- computes exp(v_j - lse): the same value without lse's
absolute rounding, a deliberate accuracy departure.  This
pins HIP's per-row dL/dQ of the critic-set IS rows (the weights times the
conservative scale, ws.dq x scalars[2]) and of the data rows against fp64
autograd's dL/dQ of the same rows, with the fp64 forward evaluated on HIP's
ReLU decisions (relu_arbiter).  Bar: 2e-6 max-normalised per block (measured
3e-7 .. 9e-7 on the hopper shape, round 5), so a regression to a less
accurate formula or a wrong weight shows."""
import copy

import numpy as np
import pytest
import torch

from cql_helpers import HostBatch, make_batch, make_impl, make_oracle, noise_dict, oracle_state
from oracle.cql import Batch, CQLNoise
from relu_arbiter import CriticReluForcer, critic_stage, hip_critic_masks, oracle_from_state, to64

pytestmark = pytest.mark.gpu


def _hook_q_outputs(o64, B, N, forcer):
    """dL/dQ of every critic call in the critic stage: per member the data
    rows' (summed over calls) and IS blocks 0..2 ([B N] each)."""
    rec = [{"data": None, "blocks": [None, None, None]} for _ in o64._q_func.q_funcs]
    calls = [0] * len(rec)
    for c, qf in enumerate(o64._q_func.q_funcs):
        orig = qf.forward

        def fwd(x, action, c=c, orig=orig):
            out = orig(x, action)
            if forcer._on and out.requires_grad and torch.is_grad_enabled():
                if out.shape[0] == B:
                    def h(g, c=c):
                        g = g.detach().reshape(-1).clone()
                        rec[c]["data"] = g if rec[c]["data"] is None else rec[c]["data"] + g
                    out.register_hook(h)
                elif out.shape[0] == B * N:
                    k = calls[c] % 3
                    calls[c] += 1

                    def h(g, c=c, k=k):
                        rec[c]["blocks"][k] = g.detach().reshape(-1).clone()
                    out.register_hook(h)
            return out
        qf.forward = fwd
    return rec


def test_cql_softmax_weights_vs_fp64():
    from test_gpu_cql_parity import _oracle_step
    D, A, H, N, B, C = 11, 3, [256, 256], 10, 256, 2
    orc = make_oracle(D, A, H, N, C=C, seed=11)
    impl = make_impl(D, A, H, N, C=C)
    rs = np.random.RandomState(0)
    gen = torch.Generator().manual_seed(1)
    sd0 = copy.deepcopy(oracle_state(orc))
    impl.set_state_dict(copy.deepcopy(sd0))
    arrs = make_batch(rs, B, D, A)
    nz = CQLNoise.draw(gen, B, A, N)
    tb = Batch.from_numpy(*arrs)
    _oracle_step(orc, tb, nz, A)
    impl.update_step(HostBatch(*arrs), noise=noise_dict(nz))
    torch.cuda.synchronize()
    ws = impl._last_ws()
    mk = lambda: make_oracle(D, A, H, N, C=C, seed=0)  # noqa: E731
    o64 = oracle_from_state(mk, sd0, torch.float64)
    fh = CriticReluForcer(o64._q_func, B, N, masks=hip_critic_masks(ws))
    rec = _hook_q_outputs(o64, B, N, fh)
    critic_stage(o64, to64(tb), to64(nz), fh)
    NB = N * B
    dq = ws.dq.double().cpu()
    sc = float(ws.scalars[2].item())
    worst = 0.0
    for c in range(C):
        for k in range(3):
            hip = dq[c, 3 * NB + k * NB: 3 * NB + (k + 1) * NB] * sc
            ref = rec[c]["blocks"][k]
            e = float((hip - ref).abs().max() / ref.abs().max())
            print(f"c{c} IS block {k}: {e:.2e}")
            worst = max(worst, e)
        hip_d, ref_d = dq[c, 6 * NB: 6 * NB + B], rec[c]["data"]
        if ws._loss_in_bwd:
            # the loss stage inside the slice backward leaves the data rows'
            # TD part in ws.dq; the backward subtracts the conservative
            # constant (scalars[2]) as it reads them (q2_x6_bwd2.hip)
            hip_d = (dq[c, 6 * NB: 6 * NB + B].float() - ws.scalars[2].cpu()).double()
        e = float((hip_d - ref_d).abs().max() / ref_d.abs().max())
        print(f"c{c} data rows: {e:.2e}")
        worst = max(worst, e)
    assert worst < 2e-6, worst
