"""Op-for-op CPU restatement of the reference torch modules on the hot path.

TEST INFRASTRUCTURE (see oracle/__init__.py).  Every random draw of the
reference is replaced by an explicit noise tensor argument so that the HIP
path can be fed the identical numbers.

Citations are to /root/reference (d3rlpy v1.1.0).
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F
from torch import nn
from torch.distributions import Normal


# ---------------------------------------------------------------------------
# encoders (d3rlpy/models/torch/encoders.py:219-344)
# ---------------------------------------------------------------------------
class VectorEncoder(nn.Module):
    """_VectorEncoder + VectorEncoder (encoders.py:219-296): relu after every fc."""

    def __init__(self, in_size: int, hidden_units: Sequence[int] = (256, 256)):
        super().__init__()
        in_units = [in_size] + list(hidden_units[:-1])
        self._fcs = nn.ModuleList(
            [nn.Linear(i, o) for i, o in zip(in_units, hidden_units)]
        )
        self._feature_size = hidden_units[-1]

    def get_feature_size(self) -> int:
        return self._feature_size

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        h = x
        for fc in self._fcs:  # _fc_encode (encoders.py:265-275)
            h = torch.relu(fc(h))
        return h


class VectorEncoderWithAction(VectorEncoder):
    """encoders.py:299-344: concat [x, action] then the MLP trunk."""

    def __init__(self, obs_size: int, action_size: int,
                 hidden_units: Sequence[int] = (256, 256)):
        super().__init__(obs_size + action_size, hidden_units)
        self._action_size = action_size

    def forward(self, x: torch.Tensor, action: torch.Tensor) -> torch.Tensor:  # type: ignore
        return super().forward(torch.cat([x, action], dim=1))


# ---------------------------------------------------------------------------
# Q functions (q_functions/mean_q_function.py:244-284, ensemble_q_function.py)
# ---------------------------------------------------------------------------
class ContinuousMeanQFunction(nn.Module):
    def __init__(self, encoder: VectorEncoderWithAction):
        super().__init__()
        self._encoder = encoder
        self._fc = nn.Linear(encoder.get_feature_size(), 1)

    def forward(self, x, action):
        return self._fc(self._encoder(x, action))

    def compute_error(self, observations, actions, rewards, target, terminals,
                      gamma=0.99, reduction="mean"):
        value = self.forward(observations, actions)
        y = rewards + gamma * target * (1 - terminals)
        loss = F.mse_loss(value, y, reduction="none")
        return compute_reduce(loss, reduction)

    def compute_target(self, x, action):
        return self.forward(x, action)


def compute_reduce(value: torch.Tensor, reduction: str) -> torch.Tensor:
    """q_functions/utility.py compute_reduce."""
    if reduction == "mean":
        return value.mean()
    if reduction == "sum":
        return value.sum()
    if reduction == "none":
        return value.view(-1, 1)
    raise ValueError("invalid reduction type.")


def reduce_ensemble(y: torch.Tensor, reduction: str = "min", dim: int = 0,
                    lam: float = 0.75) -> torch.Tensor:
    """ensemble_q_function.py:9-24."""
    if reduction == "min":
        return y.min(dim=dim).values
    if reduction == "max":
        return y.max(dim=dim).values
    if reduction == "mean":
        return y.mean(dim=dim)
    if reduction == "none":
        return y
    if reduction == "mix":
        max_values = y.max(dim=dim).values
        min_values = y.min(dim=dim).values
        return lam * min_values + (1.0 - lam) * max_values
    raise ValueError


class EnsembleContinuousQFunction(nn.Module):
    """ensemble_q_function.py:69-184 (continuous, mean heads)."""

    def __init__(self, q_funcs: List[ContinuousMeanQFunction]):
        super().__init__()
        self._q_funcs = nn.ModuleList(q_funcs)

    def forward(self, x, action, reduction="mean"):
        values = []
        for q_func in self._q_funcs:
            values.append(q_func(x, action).view(1, x.shape[0], 1))
        return reduce_ensemble(torch.cat(values, dim=0), reduction)

    def compute_error(self, observations, actions, rewards, target, terminals, gamma=0.99):
        assert target.ndim == 2
        td_sum = torch.tensor(0.0, dtype=torch.float32, device=observations.device)
        for q_func in self._q_funcs:
            loss = q_func.compute_error(
                observations=observations, actions=actions, rewards=rewards,
                target=target, terminals=terminals, gamma=gamma, reduction="none")
            td_sum += loss.mean()
        return td_sum

    def compute_target(self, x, action, reduction="min", lam=0.75):
        values_list = []
        for q_func in self._q_funcs:
            target = q_func.compute_target(x, action)
            values_list.append(target.reshape(1, x.shape[0], -1))
        values = torch.cat(values_list, dim=0)
        assert values.shape[2] == 1
        return reduce_ensemble(values, reduction, lam=lam)

    @property
    def q_funcs(self):
        return self._q_funcs


# ---------------------------------------------------------------------------
# policies / distributions (policies.py:47-271, distributions.py:91-143)
# ---------------------------------------------------------------------------
class SquashedGaussian:
    """SquashedGaussianDistribution with rsample noise supplied by the caller."""

    def __init__(self, loc: torch.Tensor, std: torch.Tensor):
        self._mean = loc
        self._std = std
        self._dist = Normal(loc, std)

    def _log_prob_from_raw_y(self, raw_y: torch.Tensor) -> torch.Tensor:
        # distributions.py:133-135
        jacob = 2 * (math.log(2) - raw_y - F.softplus(-2 * raw_y))
        return (self._dist.log_prob(raw_y) - jacob).sum(dim=-1, keepdims=True)

    def rsample(self, eps: torch.Tensor) -> torch.Tensor:
        # torch.distributions.Normal.rsample: loc + eps * scale
        return self._mean + eps * self._std

    def sample_with_log_prob(self, eps: torch.Tensor):
        raw_y = self.rsample(eps)
        log_prob = self._log_prob_from_raw_y(raw_y)
        return torch.tanh(raw_y), log_prob

    def sample_n_with_log_prob(self, eps_n: torch.Tensor):
        # eps_n: (n, batch, action) as drawn by rsample((n,))
        raw_y = self.rsample(eps_n)
        log_prob = self._log_prob_from_raw_y(raw_y)
        return torch.tanh(raw_y), log_prob

    def mean_with_log_prob(self):
        return torch.tanh(self._mean), self._log_prob_from_raw_y(self._mean)

    def log_prob(self, y: torch.Tensor) -> torch.Tensor:
        clipped_y = y.clamp(-0.999999, 0.999999)
        raw_y = torch.atanh(clipped_y)
        return self._log_prob_from_raw_y(raw_y)


class SquashedNormalPolicy(nn.Module):
    """NormalPolicy(squash_distribution=True), use_std_parameter=False."""

    def __init__(self, encoder: VectorEncoder, action_size: int,
                 min_logstd: float = -20.0, max_logstd: float = 2.0):
        super().__init__()
        self._action_size = action_size
        self._encoder = encoder
        self._min_logstd = min_logstd
        self._max_logstd = max_logstd
        self._mu = nn.Linear(encoder.get_feature_size(), action_size)
        self._logstd = nn.Linear(encoder.get_feature_size(), action_size)

    def dist(self, x: torch.Tensor) -> SquashedGaussian:
        h = self._encoder(x)
        mu = self._mu(h)
        clipped_logstd = self._logstd(h).clamp(self._min_logstd, self._max_logstd)
        return SquashedGaussian(mu, clipped_logstd.exp())

    def sample_with_log_prob(self, x, eps):
        return self.dist(x).sample_with_log_prob(eps)

    def sample_n_with_log_prob(self, x, eps_n):
        # policies.py:202-216: (n, batch, *) -> (batch, n, *)
        action_T, log_prob_T = self.dist(x).sample_n_with_log_prob(eps_n)
        return action_T.transpose(0, 1), log_prob_T.transpose(0, 1)

    def best_action(self, x):
        return self.dist(x).mean_with_log_prob()[0]


class DeterministicPolicy(nn.Module):
    """policies.py:47-79."""

    def __init__(self, encoder: VectorEncoder, action_size: int):
        super().__init__()
        self._encoder = encoder
        self._fc = nn.Linear(encoder.get_feature_size(), action_size)

    def forward(self, x):
        return torch.tanh(self._fc(self._encoder(x)))

    def best_action(self, x):
        return self.forward(x)


class Parameter(nn.Module):
    """models/torch/parameters.py:5-21."""

    def __init__(self, data: torch.Tensor):
        super().__init__()
        self._parameter = nn.Parameter(data)

    def forward(self):
        return self._parameter


def create_parameter(shape: Sequence[int], initial_value: float) -> Parameter:
    """models/builders.py:219-221."""
    return Parameter(torch.full(shape, initial_value, dtype=torch.float32))


def create_continuous_q_function(obs_size: int, action_size: int, n_ensembles: int,
                                 hidden_units: Sequence[int] = (256, 256)):
    """models/builders.py:48-70 (share_encoder=False, mean heads)."""
    q_funcs = []
    for _ in range(n_ensembles):
        enc = VectorEncoderWithAction(obs_size, action_size, hidden_units)
        q_funcs.append(ContinuousMeanQFunction(enc))
    return EnsembleContinuousQFunction(q_funcs)


def soft_sync(targ_model: nn.Module, model: nn.Module, tau: float) -> None:
    """torch_utility.py:27-33."""
    with torch.no_grad():
        for p, p_targ in zip(model.parameters(), targ_model.parameters()):
            p_targ.data.mul_(1 - tau)
            p_targ.data.add_(tau * p.data)


def hard_sync(targ_model: nn.Module, model: nn.Module) -> None:
    """torch_utility.py:36-41."""
    with torch.no_grad():
        for p, p_targ in zip(model.parameters(), targ_model.parameters()):
            p_targ.data.copy_(p.data)


def huber_loss(y: torch.Tensor, target: torch.Tensor, beta: float = 1.0) -> torch.Tensor:
    """q_functions/utility.py:27-32 compute_huber_loss."""
    diff = target - y
    cond = diff.detach().abs() < beta
    return torch.where(cond, 0.5 * diff**2, beta * (diff.abs() - 0.5 * beta))


def quantile_huber_loss(y: torch.Tensor, target: torch.Tensor, taus: torch.Tensor) -> torch.Tensor:
    """q_functions/utility.py:35-43 compute_quantile_huber_loss."""
    assert y.dim() == 3 and target.dim() == 3 and taus.dim() == 3
    huber = huber_loss(y, target)
    delta = ((target - y).detach() < 0.0).float()
    element_wise_loss = (taus - delta).abs() * huber
    return element_wise_loss.sum(dim=2).mean(dim=1)
