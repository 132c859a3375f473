"""The C-ABI as PyTorch custom ops: ``torch.ops.d3rlpy_amd.*``, and autograd
functions over their forward / backward pairs.

``load()`` loads libd3rlpy_amd_torch.so (csrc/torch_ops.cpp, built by
``_build.build``), which registers the ``d3rlpy_amd`` op namespace through
TORCH_LIBRARY with HIP (CUDA-key) and Meta implementations — SURVEY §8(b).
There is no fallback: a missing library raises.

    from d3rlpy_amd import torch_ops
    ops = torch_ops.load()
    y = ops.linear(x, W, b, True)           # every ensemble member, one launch
    q = ops.mlp_forward(x, [W0, W1, W2], [b0, b1, b2])

The differentiable wrappers below (``linear``, ``logsumexp``, ``td_mse_loss``,
``quantile_huber_loss``, ``iqn_cos_embed``, ``squashed_gaussian_sample``) let a
reference-shaped torch module — the Q functions, policy and losses of
d3rlpy/models/torch and algos/torch — run its forward AND backward on the HIP
kernels under ordinary ``loss.backward()``; tests/test_torch_ops.py checks a
CQL critic / SAC actor / QR / IQN loss written this way against the oracle.
"""
from __future__ import annotations

import os

import torch

_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libd3rlpy_amd_torch.so")
_loaded = False


def load():
    """Register the ops (idempotent) and return the ``torch.ops.d3rlpy_amd`` namespace."""
    global _loaded
    if not _loaded:
        if not os.path.exists(_LIB):
            raise RuntimeError(f"{_LIB} is missing: run d3rlpy_amd._build.build() "
                               "(no CPU fallback)")
        from . import _native
        _native.lib()  # the C-ABI library the op library links against
        torch.ops.load_library(_LIB)
        _loaded = True
    return torch.ops.d3rlpy_amd


def library_path() -> str:
    return _LIB


# ------------------------------------------------------------------ autograd
class _Linear(torch.autograd.Function):
    """y = act(x W^T + b) of every ensemble member (x [R, in] shared or
    [C, R, in], W [C, out, in] or [out, in]); ReLU when ``relu``."""

    @staticmethod
    def forward(ctx, x, W, b, relu: bool):
        y = load().linear(x.contiguous(), W.contiguous(), b.contiguous(), relu)
        ctx.relu = relu
        ctx.x_dim = x.dim()
        ctx.save_for_backward(x, W, y if relu else None)
        return y

    @staticmethod
    def backward(ctx, g):
        x, W, y = ctx.saved_tensors
        dx, dW, db = load().linear_backward(g.contiguous(), x.contiguous(), W.contiguous(),
                                            y if ctx.relu else None)
        if ctx.x_dim == 2 and W.dim() == 3:
            dx = dx.sum(0)  # x shared by the members
        return dx, dW, db, None


def linear(x: torch.Tensor, W: torch.Tensor, b: torch.Tensor, relu: bool = False) -> torch.Tensor:
    return _Linear.apply(x, W, b, relu)


class _LogSumExp(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        r = load().logsumexp(x)
        ctx.save_for_backward(x, r)
        return r

    @staticmethod
    def backward(ctx, g):
        x, r = ctx.saved_tensors
        return load().logsumexp_backward(g.contiguous(), x, r)


def logsumexp(x: torch.Tensor, keepdim: bool = False) -> torch.Tensor:
    """torch.logsumexp(x, dim=-1) on HIP (cql_impl.py:208-213)."""
    r = _LogSumExp.apply(x)
    return r.unsqueeze(-1) if keepdim else r


class _TdMse(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, rew, target, term, gamma):
        loss, diff = load().td_mse_loss(q.contiguous(), rew.contiguous(), target.contiguous(),
                                        term.contiguous(), gamma.contiguous())
        ctx.save_for_backward(diff)
        return loss

    @staticmethod
    def backward(ctx, g):
        (diff,) = ctx.saved_tensors
        return load().td_mse_loss_backward(g.contiguous(), diff), None, None, None, None


def td_mse_loss(q, rew, target, term, gamma) -> torch.Tensor:
    """Per-member mean of (q - (rew + gamma * target * (1 - term)))^2
    (ContinuousMeanQFunction.compute_error, mean_q_function.py:74-87); q and
    target [C, B] or [B], the rest [B] (gamma = gamma ** n_steps per row)."""
    return _TdMse.apply(q, rew, target, term, gamma)


class _QuantileHuber(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, y, taus):
        q, y, taus = q.contiguous(), y.contiguous(), taus.contiguous()
        ctx.save_for_backward(q, y, taus)
        return load().quantile_huber_loss(q, y, taus)

    @staticmethod
    def backward(ctx, g):
        q, y, taus = ctx.saved_tensors
        return load().quantile_huber_loss_backward(g.contiguous(), q, y, taus), None, None


def quantile_huber_loss(q, y, taus) -> torch.Tensor:
    """compute_quantile_huber_loss (q_functions/utility.py:27-46) of q [B, N]
    against the (detached) targets y [B, M] at fractions taus [B, N] -> [B]."""
    return _QuantileHuber.apply(q, y, taus)


class _IqnEmbed(torch.autograd.Function):
    @staticmethod
    def forward(ctx, taus, W, b):
        taus = taus.contiguous()
        phi = load().iqn_cos_embed(taus, W.contiguous(), b.contiguous())
        ctx.save_for_backward(taus, phi, W)
        return phi

    @staticmethod
    def backward(ctx, g):
        taus, phi, W = ctx.saved_tensors
        dW, db = load().iqn_cos_embed_backward(g.contiguous(), taus, phi, W.contiguous())
        return None, dW, db


def iqn_cos_embed(taus, W, b) -> torch.Tensor:
    """relu(embed(cos(pi * (i + 1) * tau))) of compute_iqn_feature
    (iqn_q_function.py:33-47): taus (R elements) -> [R, F]."""
    return _IqnEmbed.apply(taus, W, b)


class _SquashedGaussian(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mu, logstd, eps, lo: float, hi: float):
        mu, logstd, eps = mu.contiguous(), logstd.contiguous(), eps.contiguous()
        act, logp = load().squashed_gaussian_sample(mu, logstd, eps, lo, hi)
        ctx.save_for_backward(mu, logstd, eps)
        ctx.lo, ctx.hi = lo, hi
        return act, logp

    @staticmethod
    def backward(ctx, ga, gl):
        mu, logstd, eps = ctx.saved_tensors
        ga = torch.zeros_like(mu) if ga is None else ga.contiguous()
        gl = torch.zeros(mu.shape[0], 1, device=mu.device) if gl is None else gl.contiguous()
        dmu, dls = load().squashed_gaussian_sample_backward(ga, gl, mu, logstd, eps, ctx.lo,
                                                            ctx.hi)
        return dmu, dls, None, None, None


def squashed_gaussian_sample(mu, logstd, eps, min_logstd: float = -20.0,
                             max_logstd: float = 2.0):
    """(tanh(raw), log_prob) of SquashedNormalPolicy.sample_with_log_prob with
    the noise given: raw = mu + eps * exp(clamp(logstd)) (policies.py:196-216,
    distributions.py:112-135); log_prob [B, 1]."""
    return _SquashedGaussian.apply(mu, logstd, eps, min_logstd, max_logstd)
