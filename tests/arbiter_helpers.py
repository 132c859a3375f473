"""fp64 arbiters: is the HIP update within 1e-5 of EXACT arithmetic?

The fp32 oracle and the HIP pipeline are two fp32 evaluations of the same
formulas with different summation orders; where they disagree by more than
1e-5 the question is which one is off.  An arbiter runs the oracle in fp64
(modules, batch and draws cast to double; every constant the reference holds
in fp32 — the scaler's mean/std, QR taus — keeps its fp32 value, as in the
reference) from the SAME state HIP starts a stage from, and compares:

  gradients   max|g_hip - g64| / max|g64| <= 1e-5 per tensor
  parameters  |p_hip - p64| <= 1e-5 per entry, EXCEPT entries where Adam's
              first step amplifies a near-zero gradient: there the update is
              lr * g / (|g| + eps), whose sensitivity to g is lr * eps / (|g|+eps)^2,
              so a gradient entry of ~1e-8 that is accurate to 1e-5 of the
              tensor's max can move the parameter by anything up to 2 * lr.
              For every such entry the arbiter proves the difference is that
              amplification and nothing else: HIP's parameter equals the Adam
              map applied (in fp64) to HIP's own gradient within 1e-7, and that
              gradient passed the 1e-5 gradient check above.
"""
from __future__ import annotations

import copy

import math
from typing import Dict

import torch

GRAD_TOL = 1e-5
PARAM_TOL = 1e-5
ADAM_SELF_TOL = 1e-7


def to_double(orc, names) -> None:
    for n in names:
        getattr(orc, n).double()


def batch64(tb):
    return type(tb)(*(getattr(tb, f).double() for f in tb.__dataclass_fields__))


def load_state(orc, sd: Dict[str, dict]) -> None:
    """Load an Impl's get_state_dict() (reference layout) into an oracle;
    modules keep their dtype (load_state_dict copies with conversion)."""
    for k, v in sd.items():
        getattr(orc, k).load_state_dict(copy.deepcopy(v))  # (optimiser state tensors are kept, not copied)


def hip_grads(refs, getter) -> Dict[str, torch.Tensor]:
    out = {}
    for key, seg, member, sl in refs:
        g = getter(seg)[member]
        out[key] = (g if sl is None else g[sl]).detach().double().cpu().clone()
    return out


def module_grads(module) -> Dict[str, torch.Tensor]:
    return {n: p.grad.detach().double().clone() for n, p in module.named_parameters()}


def max_rel(a, b) -> float:
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return float((a - b).abs().max()) / max(1e-30, float(b.abs().max()))


def check_grads(label: str, g_hip: Dict[str, torch.Tensor], g64: Dict[str, torch.Tensor],
                g32: Dict[str, torch.Tensor] = None, tol: float = GRAD_TOL) -> float:
    worst = 0.0
    for k, ref in g64.items():
        e = max_rel(g_hip[k], ref)
        e32 = max_rel(g32[k], ref) if g32 is not None else float("nan")
        if e > tol or g32 is not None:
            print(f"  {label} grad {k}: hip-vs-fp64 {e:.1e}  oracle32-vs-fp64 {e32:.1e}")
        worst = max(worst, e)
    assert worst <= tol, (label, worst)
    return worst


def adam_state_by_key(optim_sd: dict, keys) -> Dict[str, tuple]:
    """torch.optim.Adam state_dict -> {param key: (exp_avg, exp_avg_sq, step)}
    with ``keys`` in parameters() order (the reference checkpoint layout)."""
    ids = optim_sd["param_groups"][0]["params"]
    out = {}
    for k, i in zip(keys, ids):
        st = optim_sd["state"].get(i)
        if st:
            out[k] = (st["exp_avg"].double(), st["exp_avg_sq"].double(), int(st["step"]))
    return out


def adam_map(p0, g, lr, state=None, betas=(0.9, 0.999), eps=1e-8):
    """torch.optim.Adam's update (weight_decay 0) in fp64 from the state
    before the step (None: the first step)."""
    b1, b2 = betas
    g = g.double()
    m0, v0, t0 = state if state is not None else (torch.zeros_like(g), torch.zeros_like(g), 0)
    t = t0 + 1
    m = b1 * m0 + (1 - b1) * g
    v = b2 * v0 + (1 - b2) * g * g
    denom = v.sqrt() / math.sqrt(1 - b2 ** t) + eps
    return p0.double() - lr / (1 - b1 ** t) * m / denom


def check_params_adam(label: str, p0: Dict[str, torch.Tensor], p_hip: Dict[str, torch.Tensor],
                      p_ref: Dict[str, torch.Tensor], g_hip: Dict[str, torch.Tensor], lr: float,
                      states: Dict[str, tuple] = None, tol: float = PARAM_TOL):
    """Parameters after one Adam step from the state ``states`` (None: the
    first step): within ``tol`` of the reference, or — entry by entry —
    HIP's value is Adam applied to HIP's own (1e-5-checked) gradient.
    Returns (max |p_hip - p_ref|, number of such entries)."""
    worst, n_amp = 0.0, 0
    for k, ref in p_ref.items():
        ph, pr = p_hip[k].double().cpu(), ref.double().cpu()
        d = (ph - pr).abs()
        worst = max(worst, float(d.max()))
        bad = d > tol
        if bool(bad.any()):
            g = g_hip[k]
            st = None if states is None else states.get(k)
            pred = adam_map(p0[k].cpu(), g, lr, st)
            self_err = float((ph - pred).abs()[bad].max())
            print(f"  {label} param {k}: {int(bad.sum())} entries differ by up to "
                  f"{float(d.max()):.1e}; their |g| <= {float(g.abs()[bad].max()):.1e} "
                  f"(tensor max {float(g.abs().max()):.1e}); HIP vs Adam(own grad) {self_err:.1e}")
            assert self_err <= ADAM_SELF_TOL, (label, k, self_err)
            n_amp += int(bad.sum())
    return worst, n_amp


def check_params_adam1(label: str, p0: Dict[str, torch.Tensor], p_hip: Dict[str, torch.Tensor],
                       p64: Dict[str, torch.Tensor], g_hip: Dict[str, torch.Tensor], lr: float,
                       eps: float = 1e-8, tol: float = PARAM_TOL):
    """Parameters after an optimiser's FIRST Adam step (see module doc).
    Returns (max |p_hip - p64|, number of amplified entries)."""
    worst, n_amp = 0.0, 0
    for k, ref in p64.items():
        ph, pr = p_hip[k].double().cpu(), ref.double().cpu()
        d = (ph - pr).abs()
        worst = max(worst, float(d.max()))
        bad = d > tol
        if bool(bad.any()):
            g = g_hip[k]
            pred = p0[k].double().cpu() - lr * g / (g.abs() + eps)
            self_err = float((ph - pred).abs()[bad].max())
            gmax = float(g.abs().max())
            print(f"  {label} param {k}: {int(bad.sum())} entries differ by up to "
                  f"{float(d.max()):.1e}; their |g| <= {float(g.abs()[bad].max()):.1e} "
                  f"(tensor max {gmax:.1e}); HIP vs Adam(own grad) {self_err:.1e}")
            assert self_err <= ADAM_SELF_TOL, (label, k, self_err)
            # amplification needs |g| within reach of the gradient error bound
            assert float(g.abs()[bad].max()) <= 1e-3 * gmax, (label, k)
            n_amp += int(bad.sum())
    return worst, n_amp
