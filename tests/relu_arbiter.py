"""ReLU-decision-aware fp64 arbiter for the CQL critic gradient.

The critic stage of one CQL update makes C x (3NB + B) x (sum of hidden
widths) ReLU decisions (K2: 2 x 7,936 x 512 = 8.1 M; the K4 data-parallel
global batch: 16.3 M).  A handful of pre-activations lie within fp32 rounding
of zero, and an fp32 evaluation -- HIP or the oracle -- may put one on the
other side of the exact sign.  A flipped decision is not a rounding-sized
error: the whole term dz * h of that (row, unit) enters or leaves the weight
gradient, while the conservative loss's sampled and data rows cancel over the
pass, so one flip can show at 1e-4 .. 1e-3 of a tensor's max-normalised
gradient (test_gpu_dp / test_gpu_production_path measured 1.1e-3 and 1.0e-3).

So the critic gradient is arbitrated as the K5 encoder's is
(test_gpu_arbiters.test_dcql_k5_b512_parity):

1. the fp32 oracle (torch CPU, the reference's arithmetic) runs the stage and
   its own ReLU decisions are recorded;
2. fp64 with the ORACLE's decisions forced -> e32, the fp32 oracle's pure
   rounding error on each gradient tensor;
3. fp64 with HIP's decisions forced (read from the kept critic activations)
   -> HIP must be within max(1e-5, 2 x e32) of it per tensor (max-normalised),
   and every decision where HIP differs from the exact fp64 sign must be a
   tie: |z| <= 2e-5 of its rounding scale sum_k |w_k h_k| + |b| (a 256-term
   fp32 dot product is within 256 x 2^-24 = 1.5e-5 of that scale).

Reference: d3rlpy/models/torch/encoders.py:265-275 (relu after every fc),
algos/torch/cql_impl.py:110-117, 143-223 (the critic stage's Q evaluations:
TD on (s, a), then the policy-sample blocks at s and s', the uniform block and
the data values).
"""
from __future__ import annotations

import copy

from typing import Dict, List, Optional

import torch

from arbiter_helpers import GRAD_TOL, max_rel, module_grads

TIE_TOL = 2e-5


class CriticReluForcer:
    """Patches every critic encoder of ``q_func`` (oracle.models
    VectorEncoderWithAction) so that, inside ``critic_stage()``:

    * record mode (``masks=None``): the ReLU decisions are recorded;
    * forced mode: relu(z) is replaced by z * mask with the given decisions,
      and (z, rounding scale, mask) of every layer is kept for the tie check.

    A call with B rows is the data block (TD error and data values: the same
    inputs); calls with B*N rows are the blocks 0 (pi at s), 1 (pi at s'),
    2 (uniform) in the order _compute_conservative_loss makes them.  Outside
    ``critic_stage()`` the encoders are the plain relu MLP."""

    def __init__(self, q_func, B: int, N: int, masks: Optional[List[dict]] = None):
        assert N != 1, "the block calls are told from the data call by their row count"
        self.B, self.N = B, N
        self.masks = masks
        self.q_funcs = list(q_func._q_funcs)
        self.recorded = [{"blocks": [None, None, None], "data": None} for _ in self.q_funcs]
        self.records = []
        self._on = False
        self._blk = [0] * len(self.q_funcs)
        for c, qf in enumerate(self.q_funcs):
            enc = qf._encoder
            enc.forward = (lambda cc, ee: (lambda x, action: self._forward(cc, ee, x, action)))(c, enc)

    class _Stage:
        def __init__(self, f):
            self.f = f

        def __enter__(self):
            self.f._on = True
            self.f._blk = [0] * len(self.f.q_funcs)

        def __exit__(self, *exc):
            self.f._on = False

    def critic_stage(self):
        return CriticReluForcer._Stage(self)

    def _forward(self, c: int, enc, x: torch.Tensor, action: torch.Tensor) -> torch.Tensor:
        h = torch.cat([x, action], dim=1)
        if not self._on:
            for fc in enc._fcs:
                h = torch.relu(fc(h))
            return h
        rows = h.shape[0]
        if rows == self.B:
            where = "data"
        elif rows == self.B * self.N:
            where = self._blk[c] % 3
            self._blk[c] += 1
        else:
            raise AssertionError(f"unexpected critic call with {rows} rows")
        for l, fc in enumerate(enc._fcs):
            z = fc(h)
            if self.masks is None:
                m = (z.detach() > 0)
                slot = self.recorded[c]
                if where == "data":
                    if slot["data"] is None:
                        slot["data"] = []
                    if len(slot["data"]) <= l:
                        slot["data"].append(m)
                else:
                    if slot["blocks"][where] is None:
                        slot["blocks"][where] = []
                    slot["blocks"][where].append(m)
                h = torch.relu(z)
            else:
                sel = self.masks[c]["data" if where == "data" else "blocks"]
                m = (sel[l] if where == "data" else sel[where][l]).to(z.dtype)
                with torch.no_grad():
                    scale = h.detach().abs() @ fc.weight.detach().abs().t() + fc.bias.detach().abs()
                self.records.append((c, where, l, z.detach(), scale, m))
                h = z * m
        return h

    def recorded_masks(self) -> List[dict]:
        return [{"blocks": [list(b) for b in r["blocks"]], "data": list(r["data"])}
                for r in self.recorded]

    def tie_report(self):
        """(decisions that differ from the exact fp64 sign, max |z| / scale
        over them) -- the data block is counted once."""
        flips, worst, seen = 0, 0.0, set()
        for c, where, l, z, scale, m in self.records:
            key = (c, where, l)
            if key in seen:
                continue
            seen.add(key)
            diff = (z > 0) != (m > 0)
            if bool(diff.any()):
                flips += int(diff.sum())
                worst = max(worst, float((z.abs() / scale)[diff].max()))
        return flips, worst


def hip_critic_masks(ws) -> List[dict]:
    """HIP's ReLU decisions of the critic stage, from the kept critic
    activations (rows [3NB, 6NB+B) of ws.qacts: blocks 0..2, then data)."""
    NB, R = ws.NB, ws.R
    out = []
    for c in range(ws.C):
        ls = [m.cpu() for m in ws.qacts.relu_decisions(c, 3 * NB, R)]
        out.append({"blocks": [[m[k * NB:(k + 1) * NB] for m in ls] for k in range(3)],
                    "data": [m[3 * NB:] for m in ls]})
    return out


def merge_rank_masks(per_rank: List[List[dict]]) -> List[dict]:
    """Data-parallel shards -> the global batch's decisions: rank r holds
    batch rows [r*Bl, (r+1)*Bl), i.e. rows [r*Bl*N, (r+1)*Bl*N) of each
    sample block (row b*N + n) and [r*Bl, (r+1)*Bl) of the data block."""
    C = len(per_rank[0])
    out = []
    for c in range(C):
        L = len(per_rank[0][c]["data"])
        out.append({"blocks": [[torch.cat([pr[c]["blocks"][k][l] for pr in per_rank])
                                for l in range(L)] for k in range(3)],
                    "data": [torch.cat([pr[c]["data"][l] for pr in per_rank]) for l in range(L)]})
    return out


def oracle_from_state(make_oracle, sd0: Dict[str, dict], dtype):
    o = make_oracle()
    for k, v in sd0.items():
        if hasattr(o, k):
            # a private copy: torch's Optimizer.load_state_dict keeps the given
            # state tensors (same dtype / device), and this oracle's optimiser
            # steps would otherwise advance the caller's state dict in place
            getattr(o, k).load_state_dict(copy.deepcopy(v))
    if dtype == torch.float64:
        for mod in (o._q_func, o._policy, o._targ_q_func, o._targ_policy, o._log_temp,
                    o._log_alpha):
            mod.double()
        for opt in (o._critic_optim, o._actor_optim, o._temp_optim, o._alpha_optim):
            for st in opt.state.values():
                for k_, v_ in st.items():
                    if torch.is_tensor(v_) and k_ != "step":
                        st[k_] = v_.double()
    return o


def to64(x):
    return type(x)(**{k: (None if getattr(x, k) is None else getattr(x, k).double())
                      for k in x.__dataclass_fields__})


def critic_stage(o, tb, nz, forcer: CriticReluForcer) -> Dict[str, torch.Tensor]:
    """update_temp / update_alpha (as CQL._update gates them) and
    update_critic with ``forcer`` active; the critic gradients."""
    if o._temp_learning_rate > 0:
        o.update_temp(tb, nz.eps_temp)
    if o._alpha_learning_rate > 0:
        o.update_alpha(tb, nz)
    with forcer.critic_stage():
        o.update_critic(tb, nz)
    return module_grads(o._q_func)


def cql_critic_arbiter(label: str, make_oracle, sd0, tb, nz, g_hip: Dict[str, torch.Tensor],
                       hip_masks: List[dict], B: int, N: int, tol: float = GRAD_TOL):
    """Steps 1-3 of the module doc.  Returns (the fp64 oracle with HIP's
    decisions, after its critic step; a summary dict)."""
    o32 = oracle_from_state(make_oracle, sd0, torch.float32)
    f32 = CriticReluForcer(o32._q_func, B, N)
    g32 = critic_stage(o32, tb, nz, f32)
    tb64, nz64 = to64(tb), to64(nz)
    oa = oracle_from_state(make_oracle, sd0, torch.float64)
    fa = CriticReluForcer(oa._q_func, B, N, masks=f32.recorded_masks())
    g64a = critic_stage(oa, tb64, nz64, fa)
    o64 = oracle_from_state(make_oracle, sd0, torch.float64)
    fh = CriticReluForcer(o64._q_func, B, N, masks=hip_masks)
    g64 = critic_stage(o64, tb64, nz64, fh)
    flips, worst_tie = fh.tie_report()
    oflips, oworst = fa.tie_report()
    # do HIP and the fp32 oracle take the same decisions everywhere?
    orec = f32.recorded_masks()
    same = all(torch.equal(hip_masks[c][kind][l] if kind == "data" else hip_masks[c][kind][k][l],
                           orec[c][kind][l] if kind == "data" else orec[c][kind][k][l])
               for c in range(len(orec)) for kind in ("data", "blocks")
               for k in (range(1) if kind == "data" else range(3))
               for l in range(len(orec[c]["data"])))
    assert worst_tie <= TIE_TOL, (label, flips, worst_tie)
    worst, worst_ratio = 0.0, 0.0
    for k, r64 in g64.items():
        e_hip, e32 = max_rel(g_hip[k], r64), max_rel(g32[k], g64a[k])
        bar = max(tol, 2.0 * e32)
        # every tensor's margin (committed per round: profiles/r05_arbiter_margins.log)
        print(f"  {label} {k}: hip vs fp64(HIP masks) {e_hip:.1e}, oracle32 vs "
              f"fp64(own masks) {e32:.1e}, bar {bar:.1e}")
        assert e_hip <= bar, (label, k, e_hip, e32)
        worst = max(worst, e_hip)
        worst_ratio = max(worst_ratio, e_hip / bar)
    info = dict(worst=worst, worst_ratio=worst_ratio, hip_flips=flips, hip_tie=worst_tie,
                oracle_flips=oflips, oracle_tie=oworst, same_decisions=same)
    print(f"  {label}: critic grads within {worst:.1e} of fp64 with HIP's ReLU decisions "
          f"({flips} decisions differ from the exact sign, max |z|/scale {worst_tie:.1e}; the "
          f"fp32 oracle: {oflips}, {oworst:.1e}; HIP and the oracle decide alike: {same})")
    return o64, info
