"""CPU restatement of DiscreteCQLImpl (IQN) and DQN / DoubleDQN / DiscreteCQL (mean Q) on pixels — TEST INFRASTRUCTURE.

Follows, op for op and in the same order:
  d3rlpy/algos/torch/dqn_impl.py:97-171          (update, DoubleDQN target, hard sync)
  d3rlpy/algos/torch/cql_impl.py:279-302          (DiscreteCQL loss, conservative term)
  d3rlpy/algos/dqn.py:127-132                     (target update schedule)
  d3rlpy/models/torch/encoders.py:57-162          (PixelEncoder, Nature-DQN filters)
  d3rlpy/models/torch/q_functions/iqn_q_function.py:16-143 (DiscreteIQNQFunction)
  d3rlpy/models/torch/q_functions/ensemble_q_function.py (n_critics = 1 reductions)
  d3rlpy/preprocessing/scalers.py:109-110         (PixelScaler x / 255)
with every torch.rand tau draw passed in explicitly (IQNTaus).
"""
from __future__ import annotations

import copy
import math
from dataclasses import dataclass
from typing import Dict, Sequence

import torch
import torch.nn.functional as F
from torch import nn

from .bcq import compute_quantile_loss
from .models import hard_sync


class PixelEncoder(nn.Module):
    """encoders.py:57-162 with the default filters and no batch norm / dropout."""

    def __init__(self, observation_shape: Sequence[int], feature_size: int = 512,
                 filters=((32, 8, 4), (64, 4, 2), (64, 3, 1))):
        super().__init__()
        in_channels = [observation_shape[0]] + [f[0] for f in filters[:-1]]
        self._convs = nn.ModuleList([nn.Conv2d(i, f[0], kernel_size=f[1], stride=f[2])
                                     for i, f in zip(in_channels, filters)])
        with torch.no_grad():
            n = self._conv_encode(torch.zeros((1,) + tuple(observation_shape))).view(1, -1).shape[1]
        self._fc = nn.Linear(n, feature_size)
        self._feature_size = feature_size

    def _conv_encode(self, x):
        h = x
        for conv in self._convs:
            h = torch.relu(conv(h))
        return h

    def forward(self, x):
        h = self._conv_encode(x)
        return torch.relu(self._fc(h.view(h.shape[0], -1)))

    def get_feature_size(self) -> int:
        return self._feature_size


def compute_iqn_feature(h, taus, embed: nn.Linear, embed_size: int):
    """iqn_q_function.py:33-47."""
    steps = torch.arange(embed_size, device=h.device).float() + 1
    expanded_taus = taus.view(h.shape[0], -1, 1)
    prior = torch.cos(math.pi * steps.view(1, 1, -1) * expanded_taus)
    phi = torch.relu(embed(prior))
    return h.view(h.shape[0], 1, -1) * phi


def pick_quantile_value_by_action(values, action):
    """q_functions/utility.py:14-21."""
    action_size = values.shape[1]
    one_hot = F.one_hot(action.view(-1), num_classes=action_size)
    mask = one_hot.view(-1, action_size, 1).float()
    return (values * mask).sum(dim=1, keepdim=False)


class DiscreteIQNQFunction(nn.Module):
    """iqn_q_function.py:50-143 (training-mode taus supplied)."""

    def __init__(self, encoder: PixelEncoder, action_size: int, n_quantiles: int = 64,
                 embed_size: int = 64):
        super().__init__()
        self._encoder = encoder
        self._action_size = action_size
        self._fc = nn.Linear(encoder.get_feature_size(), action_size)
        self._n_quantiles = n_quantiles
        self._embed_size = embed_size
        self._embed = nn.Linear(embed_size, encoder.get_feature_size())

    def _compute_quantiles(self, h, taus):
        prod = compute_iqn_feature(h, taus, self._embed, self._embed_size)
        return self._fc(prod).transpose(1, 2)

    def forward(self, x, taus):
        h = self._encoder(x)
        return self._compute_quantiles(h, taus).mean(dim=2)

    def compute_error(self, observations, actions, rewards, target, terminals, taus, gamma=0.99):
        h = self._encoder(observations)
        all_quantiles = self._compute_quantiles(h, taus)
        quantiles = pick_quantile_value_by_action(all_quantiles, actions)
        loss = compute_quantile_loss(quantiles, rewards, target, terminals, taus, gamma)
        return loss.mean()

    def compute_target(self, x, action, taus):
        h = self._encoder(x)
        quantiles = self._compute_quantiles(h, taus)
        return pick_quantile_value_by_action(quantiles, action)


@dataclass
class IQNTaus:
    """The torch.rand(B, K) draws of one DiscreteCQL update, in call order:
    next_online   _predict_best_action(next_obs)       (online, argmax)
    next_target   targ compute_target(next_obs, action)
    loss          q_func.compute_error(obs, ...)        (also the loss's taus)
    cons_lse      _compute_conservative_loss: q_func(obs) for logsumexp
    cons_data     _compute_conservative_loss: q_func(obs) for the data values"""
    next_online: torch.Tensor
    next_target: torch.Tensor
    loss: torch.Tensor
    cons_lse: torch.Tensor
    cons_data: torch.Tensor

    @staticmethod
    def draw(gen: torch.Generator, B: int, K: int) -> "IQNTaus":
        return IQNTaus(*(torch.rand(B, K, generator=gen) for _ in range(5)))


@dataclass
class PixelBatch:
    observations: torch.Tensor   # (B, C, H, W) uint8
    actions: torch.Tensor        # (B,) int64
    rewards: torch.Tensor        # (B, 1)
    next_observations: torch.Tensor
    terminals: torch.Tensor      # (B, 1)
    n_steps: torch.Tensor        # (B, 1)


class DiscreteCQLIQNOracle:
    """DiscreteCQLImpl (n_critics 1) with an IQN Q-function and the pixel scaler."""

    def __init__(self, observation_shape: Sequence[int], action_size: int,
                 learning_rate: float = 6.25e-5, gamma: float = 0.99, alpha: float = 1.0,
                 n_quantiles: int = 64, embed_size: int = 64, feature_size: int = 512,
                 seed: int = 0):
        torch.manual_seed(seed)
        self._gamma, self._alpha = gamma, alpha
        self._action_size = action_size
        self._q_func = DiscreteIQNQFunction(PixelEncoder(observation_shape, feature_size),
                                            action_size, n_quantiles, embed_size)
        self._targ_q_func = copy.deepcopy(self._q_func)
        self._optim = torch.optim.Adam(self._q_func.parameters(), lr=learning_rate)

    @staticmethod
    def _scale(x):
        return x.float() / 255.0  # PixelScaler.transform

    def compute_target(self, batch: PixelBatch, taus: IQNTaus):
        """DoubleDQNImpl.compute_target (dqn_impl.py:162-171)."""
        with torch.no_grad():
            nobs = self._scale(batch.next_observations)
            action = self._q_func(nobs, taus.next_online).argmax(dim=1)
            return self._targ_q_func.compute_target(nobs, action, taus.next_target)

    def update(self, batch: PixelBatch, taus: IQNTaus) -> float:
        """DQNImpl.update (dqn_impl.py:97-126) with DiscreteCQLImpl.compute_loss."""
        self._optim.zero_grad()
        q_tpn = self.compute_target(batch, taus)
        obs = self._scale(batch.observations)
        act = batch.actions.long()
        loss = self._q_func.compute_error(obs, act, batch.rewards, q_tpn, batch.terminals,
                                          taus.loss, gamma=self._gamma ** batch.n_steps)
        policy_values = self._q_func(obs, taus.cons_lse)
        logsumexp = torch.logsumexp(policy_values, dim=1, keepdim=True)
        one_hot = F.one_hot(act.view(-1), num_classes=self._action_size)
        data_values = (self._q_func(obs, taus.cons_data) * one_hot).sum(dim=1, keepdim=True)
        loss = loss + self._alpha * (logsumexp - data_values).mean()
        loss.backward()
        self._optim.step()
        return float(loss.detach())

    def update_target(self):
        hard_sync(self._targ_q_func, self._q_func)


# ---------------------------------------------------------------------------
# DQN / DoubleDQN / DiscreteCQL with the mean Q-function (the reference's
# default q_func_factory="mean") on pixels
#   d3rlpy/models/torch/q_functions/mean_q_function.py:13-55  (DiscreteMeanQFunction)
#   d3rlpy/models/torch/q_functions/utility.py:9-32          (pick_value_by_action, huber)
#   d3rlpy/algos/torch/dqn_impl.py:97-171                    (DQN / DoubleDQN target, update)
#   d3rlpy/algos/torch/cql_impl.py:279-302                   (DiscreteCQL loss)
# ---------------------------------------------------------------------------
def compute_huber_loss(y, target, beta: float = 1.0):
    """q_functions/utility.py:27-32."""
    diff = target - y
    cond = diff.detach().abs() < beta
    return torch.where(cond, 0.5 * diff ** 2, beta * (diff.abs() - 0.5 * beta))


def pick_value_by_action(values, action, keepdim: bool = False):
    """q_functions/utility.py:9-15."""
    one_hot = F.one_hot(action.view(-1), num_classes=values.shape[1])
    masked_values = values * one_hot.float()
    return masked_values.sum(dim=1, keepdim=keepdim)


class DiscreteMeanQFunction(nn.Module):
    """mean_q_function.py:13-55 (reduction 'mean' of compute_error)."""

    def __init__(self, encoder: PixelEncoder, action_size: int):
        super().__init__()
        self._encoder = encoder
        self._action_size = action_size
        self._fc = nn.Linear(encoder.get_feature_size(), action_size)

    def forward(self, x):
        return self._fc(self._encoder(x))

    def compute_error(self, observations, actions, rewards, target, terminals, gamma=0.99):
        one_hot = F.one_hot(actions.view(-1), num_classes=self._action_size)
        value = (self.forward(observations) * one_hot.float()).sum(dim=1, keepdim=True)
        y = rewards + gamma * target * (1 - terminals)
        return compute_huber_loss(value, y).mean()

    def compute_target(self, x, action=None):
        if action is None:
            return self.forward(x)
        return pick_value_by_action(self.forward(x), action, keepdim=True)


class DiscreteMeanOracle:
    """DQNImpl (variant 'dqn'), DoubleDQNImpl ('double_dqn') or DiscreteCQLImpl
    ('cql') with n_critics 1, the mean Q-function and the pixel scaler."""

    def __init__(self, observation_shape: Sequence[int], action_size: int, variant: str = "dqn",
                 learning_rate: float = 6.25e-5, gamma: float = 0.99, alpha: float = 1.0,
                 feature_size: int = 512, seed: int = 0):
        assert variant in ("dqn", "double_dqn", "cql")
        torch.manual_seed(seed)
        self._variant = variant
        self._gamma, self._alpha = gamma, alpha
        self._action_size = action_size
        self._q_func = DiscreteMeanQFunction(PixelEncoder(observation_shape, feature_size),
                                             action_size)
        self._targ_q_func = copy.deepcopy(self._q_func)
        self._optim = torch.optim.Adam(self._q_func.parameters(), lr=learning_rate)

    _scale = staticmethod(DiscreteCQLIQNOracle._scale)

    def compute_target(self, batch: PixelBatch):
        """DQNImpl.compute_target (dqn_impl.py:128-137) / DoubleDQNImpl's
        (:162-171)."""
        with torch.no_grad():
            nobs = self._scale(batch.next_observations)
            if self._variant == "dqn":
                action = self._targ_q_func(nobs).argmax(dim=1)
            else:
                action = self._q_func(nobs).argmax(dim=1)
            return self._targ_q_func.compute_target(nobs, action)

    def update(self, batch: PixelBatch) -> float:
        """DQNImpl.update (dqn_impl.py:97-126) [+ DiscreteCQLImpl.compute_loss]."""
        self._optim.zero_grad()
        q_tpn = self.compute_target(batch)
        obs = self._scale(batch.observations)
        act = batch.actions.long()
        loss = self._q_func.compute_error(obs, act, batch.rewards, q_tpn, batch.terminals,
                                          gamma=self._gamma ** batch.n_steps)
        if self._variant == "cql":
            policy_values = self._q_func(obs)
            logsumexp = torch.logsumexp(policy_values, dim=1, keepdim=True)
            one_hot = F.one_hot(act.view(-1), num_classes=self._action_size)
            data_values = (self._q_func(obs) * one_hot).sum(dim=1, keepdim=True)
            loss = loss + self._alpha * (logsumexp - data_values).mean()
        loss.backward()
        self._optim.step()
        return float(loss.detach())

    def update_target(self):
        hard_sync(self._targ_q_func, self._q_func)
