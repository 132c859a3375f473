"""d3a_sac_actor_q (the actor phase's critic pass: every member's Q at (s, a)
and its unscaled gradient dQ_c/da, one launch) and d3a_sac_actor_head's
dq_min mode (the backward of min over the ensemble) against fp64 autograd of
the reference's critic (GPU only).

Reference: d3rlpy/algos/torch/sac_impl.py:114-121 (q_t = self._q_func(obs,
action, "min"); (entropy - q_t).mean()), ensemble_q_function.py:12-13
(y.min(dim=0).values), encoders.py:265-275 + mean_q_function.py:255-256 (the
[n_in, 256, 256, 1] critic).  Bars: q within 1e-5 (max-normalised over the
batch), dQ/da within 1e-5 of fp64 (max-normalised per member) — the bar of the
parity suite's gradients.
"""
import pytest
import torch

from d3rlpy_amd import _native as N
from d3rlpy_amd import ops

pytestmark = pytest.mark.gpu


def _critic(C, n_in, g):
    ws = []
    for fan_in, fan_out in ((n_in, 256), (256, 256), (256, 1)):
        bound = fan_in ** -0.5
        ws.append(((torch.rand(C, fan_out, fan_in, device="cuda", generator=g) * 2 - 1) * bound,
                   (torch.rand(C, fan_out, device="cuda", generator=g) * 2 - 1) * bound))
    return ws


def _fp64(ws, x, da_off, A):
    """Every member's Q and dQ_c/da by fp64 autograd (dL/dQ_c = 1)."""
    x64 = x.double().clone().requires_grad_(True)
    (W0, b0), (W1, b1), (Wh, bh) = [(w.double(), b.double()) for w, b in ws]
    h = torch.relu(torch.einsum("ri,coi->cro", x64, W0) + b0[:, None])
    h = torch.relu(torch.einsum("cri,coi->cro", h, W1) + b1[:, None])
    q = (torch.einsum("cri,coi->cro", h, Wh) + bh[:, None])[..., 0]
    jac = []
    for c in range(q.shape[0]):
        (gx,) = torch.autograd.grad(q[c].sum(), x64, retain_graph=True)
        jac.append(gx[:, da_off:da_off + A])
    return q.detach(), torch.stack(jac)


@pytest.mark.parametrize("B,D,A,C", [(256, 11, 3, 2),    # K2 hopper
                                     (256, 29, 8, 2),    # K4 antmaze
                                     (100, 3, 1, 2),     # K1 pendulum shapes, ragged B
                                     (37, 17, 6, 3),     # ragged, three members
                                     (64, 58, 6, 10),    # n_in = 64, ten members
                                     (50, 20, 13, 2),    # A = 13: 208 (row, action) pairs
                                     (40, 17, 16, 2)])   # A = 16: all 256 threads write
def test_sac_actor_q_vs_fp64(B, D, A, C):
    g = torch.Generator(device="cuda").manual_seed(B + 7 * D + C)
    n_in = D + A
    ldx = (n_in + 3) // 4 * 4
    ws = _critic(C, n_in, g)
    x = torch.zeros(B, ldx, device="cuda")
    x[:, :D] = torch.randn(B, D, device="cuda", generator=g)
    x[:, D:n_in] = torch.tanh(torch.randn(B, A, device="cuda", generator=g))
    P = N.ACTOR_Q_PARTS
    qp = torch.full((P, C, B), float("nan"), device="cuda")
    jp = torch.full((P, C, B, A), float("nan"), device="cuda")
    d = N.SacActorQDesc()
    d.x, d.ldx = x.data_ptr(), ldx
    (W0, b0), (W1, b1), (Wh, bh) = ws
    d.W0, d.b0, d.W1, d.b1 = W0.data_ptr(), b0.data_ptr(), W1.data_ptr(), b1.data_ptr()
    d.wh, d.bh = Wh.data_ptr(), bh.data_ptr()
    d.q, d.dq_da = qp.data_ptr(), jp.data_ptr()
    d.B, d.C, d.n_in, d.A, d.da_off = B, C, n_in, A, D
    ops.call_desc("d3a_sac_actor_q", d)
    torch.cuda.synchronize()
    assert not torch.isnan(qp).any() and not torch.isnan(jp).any()
    # the parts summed in order, as d3a_sac_actor_head does
    q, dq = qp[0].clone(), jp[0].clone()
    for p in range(1, P):
        q, dq = q + qp[p], dq + jp[p]
    q64, j64 = _fp64(ws, x[:, :n_in], D, A)
    eq = float((q.double() - q64).abs().max()) / float(q64.abs().max())
    assert eq <= 1e-5, eq
    for c in range(C):
        ej = float((dq[c].double() - j64[c]).abs().max()) / float(j64[c].abs().max())
        assert ej <= 1e-5, (c, ej)


def test_sac_actor_q_rejects_bad_shapes():
    d = N.SacActorQDesc()
    with pytest.raises(RuntimeError, match="null operand"):
        ops.call_desc("d3a_sac_actor_q", d)
    t = torch.zeros(16, device="cuda")
    p = t.data_ptr()
    d.x = d.W0 = d.b0 = d.W1 = d.b1 = d.wh = d.bh = d.q = d.dq_da = p
    d.B, d.C, d.n_in, d.A, d.da_off, d.ldx = 4, 2, 65, 1, 0, 65
    with pytest.raises(RuntimeError, match="n_in <= 64"):
        ops.call_desc("d3a_sac_actor_q", d)
    d.n_in, d.A, d.da_off = 8, 3, 6
    with pytest.raises(RuntimeError, match="da_off"):
        ops.call_desc("d3a_sac_actor_q", d)


@pytest.mark.parametrize("C,P", [(2, 1), (3, 1), (2, 4)])
def test_actor_head_dq_min_matches_summed_path(C, P):
    """dq_min mode (dQ/da = -1/B * the argmin member's unscaled dQ_c/da, q and
    dQ/da given as P parts summed in order) is bit-identical to the summed
    path fed with the parts' sums and the min's backward already applied
    (zeros on the other members), ties included (first member wins, as
    y.min(dim=0) of the reference)."""
    g = torch.Generator(device="cuda").manual_seed(5 + C + P)
    B, A, D = 200, 3, 11
    H = 256
    qparts = torch.randn(P, C, B, device="cuda", generator=g)
    qparts[:, 1, :40] = qparts[:, 0, :40]  # ties
    jparts = torch.randn(P, C, B, D + A, device="cuda", generator=g)
    q, jac = qparts[0].clone(), jparts[0].clone()
    for p in range(1, P):
        q, jac = q + qparts[p], jac + jparts[p]
    # the first member of least q (strict <, as y.min(dim=0) on ties)
    arg = torch.zeros(B, dtype=torch.long, device="cuda")
    mn = q[0].clone()
    for c in range(1, C):
        upd = q[c] < mn
        arg[upd] = c
        mn = torch.where(upd, q[c], mn)
    scaled = torch.zeros_like(jac)
    for c in range(C):
        sel = arg == c
        scaled[c, sel] = jac[c, sel] * (-1.0 / B)
    head = torch.randn(B, 2 * A, device="cuda", generator=g)
    eps = torch.randn(B, A, device="cuda", generator=g)
    u = torch.randn(B, A, device="cuda", generator=g)
    logp = torch.randn(B, device="cuda", generator=g)
    scalars = torch.tensor([0.3, 0, 0, 0], device="cuda")
    hp = torch.relu(torch.randn(B, H, device="cuda", generator=g))
    wh = torch.randn(2 * A, H, device="cuda", generator=g) * 0.05

    def run(dq_buf, q_buf, dq_min):
        out = {k: torch.zeros(*s, device="cuda") for k, s in
               (("dhead", (B, 2 * A)), ("metrics", (16,)), ("dz", (B, H)),
                ("dW", (B, 2 * A, H)), ("db", (B, 2 * A)))}
        h = N.SacActorHeadDesc()
        h.head, h.eps, h.u, h.logp = head.data_ptr(), eps.data_ptr(), u.data_ptr(), logp.data_ptr()
        h.dq_da, h.ld_da, h.da_off, h.sda_c = dq_buf.data_ptr(), D + A, D, B * (D + A)
        h.q, h.sqc, h.scalars = q_buf.data_ptr(), B, scalars.data_ptr()
        h.dhead, h.metrics = out["dhead"].data_ptr(), out["metrics"].data_ptr()
        h.B, h.A, h.C = B, A, C
        h.min_logstd, h.max_logstd = -20.0, 2.0
        h.w_head, h.h, h.ldh, h.H = wh.data_ptr(), hp.data_ptr(), H, H
        h.dz, h.lddz = out["dz"].data_ptr(), H
        h.dW_part, h.db_part = out["dW"].data_ptr(), out["db"].data_ptr()
        h.dq_min, h.dq_scale = dq_min, -1.0 / B
        h.n_part, h.sq_part, h.sda_part = P, C * B, C * B * (D + A)
        ops.call_desc("d3a_sac_actor_head", h)
        torch.cuda.synchronize()
        return out

    a = run(jparts, qparts, 1)
    b = run(scaled, q, 0)
    for k in a:
        assert torch.equal(a[k], b[k]), k
