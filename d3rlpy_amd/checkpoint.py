"""Reference-compatible checkpoints: the ``torch.save(get_state_dict(impl))``
layout of d3rlpy/torch_utility.py:97-117 / algos/torch/base.py:137-142.

A checkpoint is a dict keyed by the Impl attribute names (``_q_func``,
``_targ_q_func``, ``_policy``, ``_targ_policy``, ``_log_temp``, ... ,
``_critic_optim``, ...), each value the ``state_dict()`` the reference's
nn.Module / torch.optim.Adam would produce: module keys such as
``_q_funcs.0._encoder._fcs.1.weight`` and Adam states
``{"state": {i: {"step", "exp_avg", "exp_avg_sq"}}, "param_groups": [...]}``
with parameters indexed in ``module.parameters()`` order.  The HIP engine's
flat buffers are read/written through views, so checkpoints interchange with
reference users in both directions.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch

from .nets import OptimState, ParamStore

# (state-dict key, store segment name, ensemble member, slice of the first dim or None)
ParamRef = Tuple[str, str, int, Optional[slice]]


def _view(store: ParamStore, ref: ParamRef) -> torch.Tensor:
    _, seg, member, sl = ref
    v = store.view(seg)[member]
    return v if sl is None else v[sl]


def module_state(store: ParamStore, refs: Sequence[ParamRef]) -> "OrderedDict[str, torch.Tensor]":
    return OrderedDict((r[0], _view(store, r).detach().clone().cpu()) for r in refs)


def load_module_state(store: ParamStore, refs: Sequence[ParamRef], sd: Dict[str, torch.Tensor]
                      ) -> None:
    keys = {r[0] for r in refs}
    missing = keys - set(sd)
    if missing:
        raise KeyError(f"missing keys in state dict: {sorted(missing)}")
    with torch.no_grad():
        for r in refs:
            v = _view(store, r)
            src = torch.as_tensor(sd[r[0]])
            if tuple(src.shape) != tuple(v.shape):
                raise ValueError(f"shape mismatch for {r[0]}: {tuple(src.shape)} vs {tuple(v.shape)}")
            v.copy_(src.to(v.device, v.dtype))


def _param_group(lr: float, betas, eps: float, n: int) -> dict:
    return {"lr": lr, "betas": tuple(betas), "eps": eps, "weight_decay": 0, "amsgrad": False,
            "maximize": False, "foreach": None, "capturable": False, "differentiable": False,
            "fused": None, "decoupled_weight_decay": False, "params": list(range(n))}


def adam_state(st: OptimState, refs: Sequence[ParamRef]) -> dict:
    step = int(st.step.item())
    state = {}
    if step > 0:
        for i, r in enumerate(refs):
            state[i] = {"step": torch.tensor(float(step)),
                        "exp_avg": _view(st.exp_avg, r).detach().clone().cpu(),
                        "exp_avg_sq": _view(st.exp_avg_sq, r).detach().clone().cpu()}
    return {"state": state, "param_groups": [_param_group(st.lr, st.betas, st.eps, len(refs))]}


def load_adam_state(st: OptimState, refs: Sequence[ParamRef], sd: dict) -> None:
    state = sd.get("state", {})
    with torch.no_grad():
        if not state:
            st.exp_avg.data.zero_()
            st.exp_avg_sq.data.zero_()
            st.step.zero_()
            return
        steps = set()
        for i, r in enumerate(refs):
            s = state[i] if i in state else state[str(i)]
            _view(st.exp_avg, r).copy_(torch.as_tensor(s["exp_avg"]))
            _view(st.exp_avg_sq, r).copy_(torch.as_tensor(s["exp_avg_sq"]))
            steps.add(int(float(s["step"])))
        if len(steps) != 1:
            raise ValueError("all parameters of one optimiser must share the step count")
        st.step.fill_(steps.pop())


def scalar_adam_state(m: torch.Tensor, v: torch.Tensor, step: torch.Tensor, lr: float, betas,
                      eps: float) -> dict:
    t = int(step.item())
    state = {}
    if t > 0:
        state[0] = {"step": torch.tensor(float(t)), "exp_avg": m.detach().view(1, 1).cpu().clone(),
                    "exp_avg_sq": v.detach().view(1, 1).cpu().clone()}
    return {"state": state, "param_groups": [_param_group(lr, betas, eps, 1)]}


def load_scalar_adam_state(m: torch.Tensor, v: torch.Tensor, step: torch.Tensor, sd: dict) -> None:
    state = sd.get("state", {})
    with torch.no_grad():
        if not state:
            m.zero_(); v.zero_(); step.zero_()
            return
        s = state[0] if 0 in state else state["0"]
        m.copy_(torch.as_tensor(s["exp_avg"]).view(-1))
        v.copy_(torch.as_tensor(s["exp_avg_sq"]).view(-1))
        step.fill_(int(float(s["step"])))
