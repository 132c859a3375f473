"""CPU restatement of BCQImpl updates (continuous, QR critics) — TEST INFRASTRUCTURE.

Follows, op for op and in the same order:
  d3rlpy/algos/torch/bcq_impl.py:101-226        (build, update_imitator, target, actor loss)
  d3rlpy/algos/torch/ddpg_impl.py:138-183        (update_critic / update_actor)
  d3rlpy/algos/bcq.py:261-279                    (BCQ._update schedule)
  d3rlpy/models/torch/imitators.py:13-118        (ConditionalVAE)
  d3rlpy/models/torch/policies.py:82-97          (DeterministicResidualPolicy)
  d3rlpy/models/torch/q_functions/qr_q_function.py:15-19, 97-161 (ContinuousQRQFunction)
  d3rlpy/models/torch/q_functions/utility.py:27-61 (quantile Huber loss)
  d3rlpy/models/torch/q_functions/__init__.py:8-72 (compute_max_with_n_actions)
with every torch.randn draw passed in explicitly (BCQNoise).
"""
from __future__ import annotations

import copy
from dataclasses import dataclass
from typing import Dict, List, Sequence

import torch
import torch.nn.functional as F
from torch import nn
from torch.distributions import Normal, kl_divergence

from .cql import Batch
from .models import VectorEncoderWithAction, compute_reduce, soft_sync


def make_taus(n_quantiles: int) -> torch.Tensor:
    """qr_q_function.py:15-19."""
    steps = torch.arange(n_quantiles, dtype=torch.float32)
    taus = ((steps + 1).float() / n_quantiles).view(1, -1)
    taus_dot = (steps.float() / n_quantiles).view(1, -1)
    return (taus + taus_dot) / 2.0


def compute_huber_loss(y, target, beta: float = 1.0):
    diff = target - y
    cond = diff.detach().abs() < beta
    return torch.where(cond, 0.5 * diff ** 2, beta * (diff.abs() - 0.5 * beta))


def compute_quantile_huber_loss(y, target, taus):
    huber_loss = compute_huber_loss(y, target)
    delta = ((target - y).detach() < 0.0).float()
    element_wise_loss = (taus - delta).abs() * huber_loss
    return element_wise_loss.sum(dim=2).mean(dim=1)


def compute_quantile_loss(quantiles, rewards, target, terminals, taus, gamma):
    """q_functions/utility.py:46-61."""
    batch_size, n_quantiles = quantiles.shape
    expanded_quantiles = quantiles.view(batch_size, 1, -1)
    y = rewards + gamma * target * (1 - terminals)
    expanded_y = y.view(batch_size, -1, 1)
    expanded_taus = taus.view(-1, 1, n_quantiles)
    return compute_quantile_huber_loss(expanded_quantiles, expanded_y, expanded_taus)


class ContinuousQRQFunction(nn.Module):
    """qr_q_function.py:97-161."""

    def __init__(self, encoder: VectorEncoderWithAction, n_quantiles: int):
        super().__init__()
        self._encoder = encoder
        self._n_quantiles = n_quantiles
        self._fc = nn.Linear(encoder.get_feature_size(), n_quantiles)

    def forward(self, x, action):
        quantiles = self._fc(self._encoder(x, action))
        return quantiles.mean(dim=1, keepdim=True)

    def compute_error(self, observations, actions, rewards, target, terminals, gamma=0.99,
                      reduction="mean"):
        assert target.shape == (observations.shape[0], self._n_quantiles)
        quantiles = self._fc(self._encoder(observations, actions))
        taus = make_taus(self._n_quantiles).to(quantiles.dtype)
        loss = compute_quantile_loss(quantiles, rewards, target, terminals, taus, gamma)
        return compute_reduce(loss, reduction)

    def compute_target(self, x, action):
        return self._fc(self._encoder(x, action))


class EnsembleQRQFunction(nn.Module):
    """ensemble_q_function.py:69-184 for quantile heads."""

    def __init__(self, q_funcs: List[ContinuousQRQFunction]):
        super().__init__()
        self._q_funcs = nn.ModuleList(q_funcs)

    def forward(self, x, action, reduction="mean"):
        assert reduction == "none"
        return torch.cat([q(x, action).view(1, x.shape[0], 1) for q in self._q_funcs], dim=0)

    def compute_error(self, observations, actions, rewards, target, terminals, gamma=0.99):
        td_sum = torch.tensor(0.0, dtype=torch.float32)
        for q_func in self._q_funcs:
            loss = q_func.compute_error(observations, actions, rewards, target, terminals,
                                        gamma=gamma, reduction="none")
            td_sum += loss.mean()
        return td_sum

    def compute_target(self, x, action, reduction="none"):
        assert reduction == "none"
        return torch.cat([q.compute_target(x, action).reshape(1, x.shape[0], -1)
                          for q in self._q_funcs], dim=0)

    @property
    def q_funcs(self):
        return self._q_funcs


def gather_quantiles_by_indices(y: torch.Tensor, indices: torch.Tensor) -> torch.Tensor:
    """ensemble_q_function.py:25-42 (the 3-D case: (N, batch, K) -> (batch, K))."""
    assert y.dim() == 3
    return y.transpose(0, 1)[torch.arange(y.shape[1]), indices]


def reduce_quantile_ensemble(y: torch.Tensor, reduction: str = "min", dim: int = 0,
                             lam: float = 0.75) -> torch.Tensor:
    """ensemble_q_function.py:45-66: pick each row's member by the mean of its
    quantiles (min / max), or mix the two picks."""
    mean = y.mean(dim=-1)
    if reduction == "min":
        return gather_quantiles_by_indices(y, mean.min(dim=dim).indices)
    if reduction == "max":
        return gather_quantiles_by_indices(y, mean.max(dim=dim).indices)
    if reduction == "none":
        return y
    if reduction == "mix":
        mn = gather_quantiles_by_indices(y, mean.min(dim=dim).indices)
        mx = gather_quantiles_by_indices(y, mean.max(dim=dim).indices)
        return lam * mn + (1.0 - lam) * mx
    raise ValueError("invalid reduction type.")


def compute_max_with_n_actions(x, actions, q_func: EnsembleQRQFunction, lam: float):
    """q_functions/__init__.py:8-72 (first return value)."""
    batch_size = actions.shape[0]
    n_critics = len(q_func.q_funcs)
    n_actions = actions.shape[1]
    expanded_x = x.expand(n_actions, *x.shape).transpose(0, 1)
    flat_x = expanded_x.reshape(-1, *x.shape[1:])
    flat_actions = actions.reshape(batch_size * n_actions, -1)
    flat_values = q_func.compute_target(flat_x, flat_actions, "none")
    transposed_values = flat_values.view(n_critics, batch_size, n_actions, -1)
    values = transposed_values.transpose(0, 1)
    mean_values = values.mean(dim=3)
    max_values, max_indices = mean_values.max(dim=1)
    min_values, min_indices = mean_values.min(dim=1)
    mix_values = (1.0 - lam) * max_values + lam * min_values
    action_indices = mix_values.argmax(dim=1)
    values_T = values.transpose(1, 2)
    flat_values = values_T.reshape(batch_size * n_actions, n_critics, -1)
    bn_indices = torch.arange(batch_size * n_actions)
    max_values = flat_values[bn_indices, max_indices.view(-1)]
    min_values = flat_values[bn_indices, min_indices.view(-1)]
    max_values = max_values.view(batch_size, n_actions, -1)
    min_values = min_values.view(batch_size, n_actions, -1)
    mix_values = (1.0 - lam) * max_values + lam * min_values
    return mix_values[torch.arange(x.shape[0]), action_indices]


class ConditionalVAE(nn.Module):
    """imitators.py:13-98 (rsample noise supplied)."""

    def __init__(self, encoder_encoder, decoder_encoder, action_size, latent_size, beta,
                 min_logstd=-20.0, max_logstd=2.0):
        super().__init__()
        self._encoder_encoder = encoder_encoder
        self._decoder_encoder = decoder_encoder
        self._beta = beta
        self._min_logstd = min_logstd
        self._max_logstd = max_logstd
        self._mu = nn.Linear(encoder_encoder.get_feature_size(), latent_size)
        self._logstd = nn.Linear(encoder_encoder.get_feature_size(), latent_size)
        self._fc = nn.Linear(decoder_encoder.get_feature_size(), action_size)

    def encode(self, x, action) -> Normal:
        h = self._encoder_encoder(x, action)
        mu = self._mu(h)
        logstd = self._logstd(h)
        clipped_logstd = logstd.clamp(self._min_logstd, self._max_logstd)
        return Normal(mu, clipped_logstd.exp())

    def decode(self, x, latent):
        h = self._decoder_encoder(x, latent)
        return torch.tanh(self._fc(h))

    def compute_error(self, x, action, eps):
        dist = self.encode(x, action)
        kl_loss = kl_divergence(dist, Normal(0.0, 1.0)).mean()
        z = dist.loc + eps * dist.scale  # Normal.rsample with the draw supplied
        y = self.decode(x, z)
        return F.mse_loss(y, action) + self._beta * kl_loss


class DeterministicResidualPolicy(nn.Module):
    """policies.py:82-97."""

    def __init__(self, encoder: VectorEncoderWithAction, action_size: int, scale: float):
        super().__init__()
        self._scale = scale
        self._encoder = encoder
        self._fc = nn.Linear(encoder.get_feature_size(), action_size)

    def forward(self, x, action):
        h = self._encoder(x, action)
        residual_action = self._scale * torch.tanh(self._fc(h))
        return (action + residual_action).clamp(-1.0, 1.0)


@dataclass
class BCQNoise:
    """The torch.randn draws of one BCQ._update:
    eps_vae (B, 2A)      ConditionalVAE.compute_error  dist.rsample()
    z_target (B*N, 2A)   _sample_repeated_action (target)
    z_actor (B, 2A)      compute_actor_loss latent"""
    eps_vae: torch.Tensor
    z_target: torch.Tensor
    z_actor: torch.Tensor

    @staticmethod
    def draw(gen: torch.Generator, B: int, A: int, N: int) -> "BCQNoise":
        return BCQNoise(torch.randn(B, 2 * A, generator=gen),
                        torch.randn(B * N, 2 * A, generator=gen),
                        torch.randn(B, 2 * A, generator=gen))


class BCQOracle:
    """BCQImpl with the K3 configuration (QR critics) and the reference defaults
    (algos/bcq.py:171-192)."""

    def __init__(self, observation_size: int, action_size: int,
                 actor_learning_rate: float = 1e-3, critic_learning_rate: float = 1e-3,
                 imitator_learning_rate: float = 1e-3, gamma: float = 0.99, tau: float = 0.005,
                 n_critics: int = 2, lam: float = 0.75, n_action_samples: int = 100,
                 action_flexibility: float = 0.05, beta: float = 0.5, n_quantiles: int = 200,
                 hidden_units: Sequence[int] = (256, 256), seed: int = 0):
        torch.manual_seed(seed)
        D, A = observation_size, action_size
        self._A = A
        self._gamma, self._tau, self._lam = gamma, tau, lam
        self._n_action_samples = n_action_samples
        # BCQImpl.build (bcq_impl.py:101-105): imitator, then DDPGBaseImpl.build
        self._imitator = ConditionalVAE(VectorEncoderWithAction(D, A, hidden_units),
                                        VectorEncoderWithAction(D, 2 * A, hidden_units),
                                        A, 2 * A, beta, min_logstd=-4.0, max_logstd=15.0)
        self._q_func = EnsembleQRQFunction([
            ContinuousQRQFunction(VectorEncoderWithAction(D, A, hidden_units), n_quantiles)
            for _ in range(n_critics)])
        self._policy = DeterministicResidualPolicy(VectorEncoderWithAction(D, A, hidden_units),
                                                   A, action_flexibility)
        self._targ_q_func = copy.deepcopy(self._q_func)
        self._targ_policy = copy.deepcopy(self._policy)
        self._critic_optim = torch.optim.Adam(self._q_func.parameters(), lr=critic_learning_rate)
        self._actor_optim = torch.optim.Adam(self._policy.parameters(), lr=actor_learning_rate)
        self._imitator_optim = torch.optim.Adam(self._imitator.parameters(),
                                                lr=imitator_learning_rate)

    def update_imitator(self, batch: Batch, eps_vae: torch.Tensor):
        """bcq_impl.py:148-161."""
        self._imitator_optim.zero_grad()
        loss = self._imitator.compute_error(batch.observations, batch.actions, eps_vae)
        loss.backward()
        self._imitator_optim.step()
        return loss.detach().numpy()

    def _sample_repeated_action(self, repeated_x, z, target: bool):
        """bcq_impl.py:169-187."""
        flattened_x = repeated_x.reshape(-1, repeated_x.shape[-1])
        clipped_latent = z.clamp(-0.5, 0.5)
        sampled_action = self._imitator.decode(flattened_x, clipped_latent)
        policy = self._targ_policy if target else self._policy
        action = policy(flattened_x, sampled_action)
        return action.view(-1, self._n_action_samples, self._A)

    def compute_target(self, batch: Batch, z_target: torch.Tensor):
        """bcq_impl.py:215-226."""
        with torch.no_grad():
            x = batch.next_observations
            repeated_x = x.view(x.shape[0], 1, *x.shape[1:]).expand(
                x.shape[0], self._n_action_samples, *x.shape[1:])
            actions = self._sample_repeated_action(repeated_x, z_target, True)
            return compute_max_with_n_actions(x, actions, self._targ_q_func, self._lam)

    def update_critic(self, batch: Batch, z_target: torch.Tensor):
        """ddpg_impl.py:138-165."""
        self._critic_optim.zero_grad()
        q_tpn = self.compute_target(batch, z_target)
        loss = self._q_func.compute_error(batch.observations, batch.actions, batch.rewards, q_tpn,
                                          batch.terminals, gamma=self._gamma ** batch.n_steps)
        loss.backward()
        self._critic_optim.step()
        return loss.detach().numpy()

    def compute_actor_loss(self, batch: Batch, z_actor: torch.Tensor):
        """bcq_impl.py:132-146."""
        clipped_latent = z_actor.clamp(-0.5, 0.5)
        sampled_action = self._imitator.decode(batch.observations, clipped_latent)
        action = self._policy(batch.observations, sampled_action)
        return -self._q_func(batch.observations, action, "none")[0].mean()

    def update_actor(self, batch: Batch, z_actor: torch.Tensor):
        """ddpg_impl.py:167-183."""
        self._actor_optim.zero_grad()
        loss = self.compute_actor_loss(batch, z_actor)
        loss.backward()
        self._actor_optim.step()
        return loss.detach().numpy()

    def update(self, batch: Batch, noise: BCQNoise) -> Dict[str, float]:
        """algos/bcq.py:261-279 with rl_start_step 0, update_actor_interval 1."""
        m = {"imitator_loss": float(self.update_imitator(batch, noise.eps_vae))}
        m["critic_loss"] = float(self.update_critic(batch, noise.z_target))
        m["actor_loss"] = float(self.update_actor(batch, noise.z_actor))
        soft_sync(self._targ_policy, self._policy, self._tau)
        soft_sync(self._targ_q_func, self._q_func, self._tau)
        return m
