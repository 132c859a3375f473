"""Greedy-policy export for ``save_policy`` (d3rlpy/algos/torch/base.py:87-127).

The reference traces ``_predict_best_action`` (with the observation scaler in
front and the action scaler's reverse transform behind) into TorchScript and
saves it as ``.pt`` or exports it as ``.onnx``.  The HIP Impls run their
networks through ctypes calls, which ``torch.jit.trace`` cannot record, so
the exported program is a plain-torch restatement of each Impl's greedy
action built from a snapshot of its current parameters — the same layer
arithmetic (Linear / ReLU chains, the Nature-DQN convolutions, tanh, the IQN
cosine embedding), runnable without this library, as the reference's traced
script is.  It is a deployment artefact, not a compute path of the engine.
"""
from __future__ import annotations

import math
import torch
from torch import nn

from .nets import EnsembleMLP, ParamStore

# save_policy(..., hip_ops=True): MLP trunks export as one call of the
# registered custom op torch.ops.d3rlpy_amd.mlp_forward (the HIP GEMM kernels;
# loading the program needs d3rlpy_amd.torch_ops.load() first) instead of the
# portable plain-torch Linear / ReLU chain
_HIP_OPS = False


class HipMLP(nn.Module):
    """An ensemble member's ReLU MLP through torch.ops.d3rlpy_amd.mlp_forward
    (scriptable / traceable: the op is registered with TORCH_LIBRARY)."""

    def __init__(self, Ws, bs):
        super().__init__()
        from . import torch_ops
        torch_ops.load()
        self.Ws = nn.ParameterList([nn.Parameter(W.detach().clone(), requires_grad=False)
                                    for W in Ws])
        self.bs = nn.ParameterList([nn.Parameter(b.detach().clone(), requires_grad=False)
                                    for b in bs])

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        Ws = [w for w in self.Ws]
        bs = [b for b in self.bs]
        return torch.ops.d3rlpy_amd.mlp_forward(x.contiguous(), Ws, bs)


def mlp_module(net: EnsembleMLP, store: ParamStore, member: int = 0) -> nn.Module:
    """Member ``member`` of an ensemble as Linear / ReLU layers (encoders.py:265-275
    + the linear head), weights copied from ``store`` (or, under
    save_policy(hip_ops=True), as one HipMLP)."""
    if _HIP_OPS:
        pairs = [net.export_linear(l, member, store) for l in range(net.n_layers)]
        return HipMLP([W for W, _ in pairs], [b for _, b in pairs])
    layers = []
    for l in range(net.n_layers):
        W, b = net.export_linear(l, member, store)
        lin = nn.Linear(W.shape[1], W.shape[0], device=W.device)
        with torch.no_grad():
            lin.weight.copy_(W)
            lin.bias.copy_(b)
        layers.append(lin)
        if l < net.n_layers - 1:
            layers.append(nn.ReLU())
    return nn.Sequential(*layers)


class _Scaled(nn.Module):
    """scaler.transform -> greedy action -> action_scaler.reverse_transform
    (the ``_func`` of algos/torch/base.py:94-103)."""

    def __init__(self, body: nn.Module, scaler=None, action_scaler=None):
        super().__init__()
        self.body = body
        self.scaler = scaler
        self.action_scaler = action_scaler

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.scaler is not None:
            x = self.scaler.transform(x)
        a = self.body(x)
        if self.action_scaler is not None:
            a = self.action_scaler.reverse_transform(a)
        return a


class TanhMeanPolicy(nn.Module):
    """SquashedNormalPolicy.best_action: tanh(mu(s)) (policies.py:218-224); the
    head's first ``action_size`` outputs are mu."""

    def __init__(self, trunk: nn.Sequential, action_size: int):
        super().__init__()
        self.trunk = trunk
        self.action_size = action_size

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return torch.tanh(self.trunk(x)[:, :self.action_size])


class DeterministicPolicy(nn.Module):
    """DeterministicPolicy.forward: tanh(W h + b) (policies.py:57-59)."""

    def __init__(self, trunk: nn.Sequential):
        super().__init__()
        self.trunk = trunk

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return torch.tanh(self.trunk(x))


class BCQGreedy(nn.Module):
    """BCQImpl._predict_best_action (bcq_impl.py:204-210): N latent draws per
    state clipped to [-0.5, 0.5], VAE decode, residual perturbation, argmax of
    the first QR critic's quantile mean."""

    def __init__(self, dec: nn.Sequential, policy: nn.Sequential, critic0: nn.Sequential,
                 action_size: int, n_samples: int, flexibility: float):
        super().__init__()
        self.dec, self.policy, self.critic0 = dec, policy, critic0
        self.A, self.N, self.flex = action_size, n_samples, flexibility

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        B = x.shape[0]
        rx = x.repeat_interleave(self.N, dim=0)
        z = torch.randn(rx.shape[0], 2 * self.A, device=x.device).clamp(-0.5, 0.5)
        a_dec = torch.tanh(self.dec(torch.cat([rx, z], 1)))
        act = (a_dec + self.flex * torch.tanh(self.policy(torch.cat([rx, a_dec], 1)))).clamp(-1, 1)
        q0 = self.critic0(torch.cat([rx, act], 1)).mean(dim=1)
        idx = q0.view(B, self.N).argmax(dim=1)
        return act.view(B, self.N, self.A)[torch.arange(B, device=x.device), idx]


class IQNGreedy(nn.Module):
    """argmax_a of DiscreteIQNQFunction.forward in eval mode (iqn_q_function.py:
    16-47, 97-110): PixelEncoder (encoders.py:130-162), linspace taus, cosine
    prior, ReLU embedding, head, mean over quantiles."""

    def __init__(self, convs: nn.ModuleList, fc: nn.Linear, embed: nn.Linear, head: nn.Linear,
                 n_greedy: int, embed_size: int):
        super().__init__()
        self.convs, self.fc, self.embed, self.head = convs, fc, embed, head
        self.K, self.E = n_greedy, embed_size

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        h = x
        for conv in self.convs:
            h = torch.relu(conv(h))
        h = torch.relu(self.fc(h.reshape(h.shape[0], -1)))
        taus = torch.linspace(0, 1, self.K, device=x.device, dtype=torch.float32)
        steps = torch.arange(self.E, device=x.device).float() + 1
        prior = torch.cos(math.pi * steps.view(1, 1, -1) * taus.view(1, -1, 1))
        phi = torch.relu(self.embed(prior))                   # (1, K, F)
        q = self.head(h.view(h.shape[0], 1, -1) * phi)        # (B, K, A)
        return q.mean(dim=1).argmax(dim=1)


class MeanQGreedy(nn.Module):
    """argmax_a of DiscreteMeanQFunction.forward (mean_q_function.py:22-23):
    PixelEncoder (encoders.py:130-162) then the linear head (DQNImpl.
    _predict_best_action, dqn_impl.py:139-141)."""

    def __init__(self, convs: nn.ModuleList, fc: nn.Linear, head: nn.Linear):
        super().__init__()
        self.convs, self.fc, self.head = convs, fc, head

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        h = x
        for conv in self.convs:
            h = torch.relu(conv(h))
        h = torch.relu(self.fc(h.reshape(h.shape[0], -1)))
        return self.head(h).argmax(dim=1)


def linear_from(W: torch.Tensor, b: torch.Tensor) -> nn.Linear:
    lin = nn.Linear(W.shape[1], W.shape[0], device=W.device)
    with torch.no_grad():
        lin.weight.copy_(W)
        lin.bias.copy_(b)
    return lin


def save_traced(module: nn.Module, observation_shape, device: torch.device, fname: str,
                scaler=None, action_scaler=None) -> None:
    """Trace ``module`` (behind the scalers) and write ``.pt`` / ``.onnx``
    (algos/torch/base.py:105-124)."""
    wrapped = _Scaled(module, scaler, action_scaler).eval()
    for p in wrapped.parameters():  # freeze(), algos/torch/base.py:91
        p.requires_grad_(False)
    dummy = torch.rand(1, *observation_shape, device=device)
    with torch.no_grad():
        traced = torch.jit.trace(wrapped, dummy, check_trace=False)
    if fname.endswith(".onnx"):
        try:
            import onnx  # noqa: F401  (the exporter's serialiser)
        except ImportError as e:
            raise RuntimeError("ONNX export needs the 'onnx' package, which is not installed "
                               "in this environment; save as .pt (TorchScript)") from e
        torch.onnx.export(traced, dummy, fname, export_params=True, opset_version=11,
                          input_names=["input_0"], output_names=["output_0"], dynamo=False)
    elif fname.endswith(".pt"):
        traced.save(fname)
    else:
        raise ValueError(f"invalid format type: {fname}. .pt and .onnx extensions are currently "
                         "supported.")


def conv_from(W: torch.Tensor, b: torch.Tensor, stride: int) -> nn.Conv2d:
    co, ci, k, _ = W.shape
    conv = nn.Conv2d(ci, co, kernel_size=k, stride=stride, device=W.device)
    with torch.no_grad():
        conv.weight.copy_(W)
        conv.bias.copy_(b)
    return conv

