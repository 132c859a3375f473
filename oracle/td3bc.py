"""CPU restatement of TD3PlusBCImpl updates — TEST INFRASTRUCTURE.

Follows, op for op and in the same order:
  d3rlpy/algos/torch/ddpg_impl.py:95-209   (build, update_critic, update_actor, targets)
  d3rlpy/algos/torch/td3_impl.py:61-78     (target smoothing)
  d3rlpy/algos/torch/td3_plus_bc_impl.py:64-70 (BC actor loss)
  d3rlpy/algos/td3_plus_bc.py:177-192      (TD3PlusBC._update schedule)
  d3rlpy/torch_utility.py:179-181 + preprocessing/scalers.py:350-354 (standard scaler)
with the target-smoothing noise passed in explicitly.  TD3Oracle / DDPGOracle
restate the parents: DDPGImpl.compute_actor_loss (ddpg_impl.py:244-249) and,
for DDPG, DDPGImpl.compute_target (ddpg_impl.py:251-260) with the schedules of
algos/td3.py:182-203 and algos/ddpg.py:167-174.
"""
from __future__ import annotations

import copy
from typing import Dict, Optional, Sequence

import numpy as np
import torch

from .cql import Batch
from .models import DeterministicPolicy, VectorEncoder, create_continuous_q_function, soft_sync


class StandardScalerT:
    """scalers.py:350-354 transform with fixed mean / std arrays."""

    def __init__(self, mean: np.ndarray, std: np.ndarray, eps: float = 1e-3):
        self._mean = np.asarray(mean).reshape(1, -1)
        self._std = np.asarray(std).reshape(1, -1)
        self._eps = eps

    def transform(self, x: torch.Tensor) -> torch.Tensor:
        mean = torch.tensor(self._mean, dtype=torch.float32, device=x.device)
        std = torch.tensor(self._std, dtype=torch.float32, device=x.device)
        return (x - mean) / (std + self._eps)


def fit_standard_scaler(observations: np.ndarray):
    """scalers.py:320-341 (two passes, float64 accumulation as numpy does)."""
    total_sum = np.zeros(observations.shape[1:])
    for o in observations:
        total_sum += np.asarray(o)
    mean = total_sum / len(observations)
    total_sqsum = np.zeros(observations.shape[1:])
    for o in observations:
        total_sqsum += (np.asarray(o) - mean) ** 2
    std = np.sqrt(total_sqsum / len(observations))
    return mean, std


class TD3PlusBCOracle:
    _BC = True

    def __init__(self, observation_size: int, action_size: int,
                 actor_learning_rate: float = 3e-4, critic_learning_rate: float = 3e-4,
                 gamma: float = 0.99, tau: float = 0.005, n_critics: int = 2,
                 target_smoothing_sigma: float = 0.2, target_smoothing_clip: float = 0.5,
                 alpha: float = 2.5, hidden_units: Sequence[int] = (256, 256),
                 scaler: Optional[StandardScalerT] = None, seed: int = 0):
        torch.manual_seed(seed)
        self._action_size = action_size
        self._gamma = gamma
        self._tau = tau
        self._sigma = target_smoothing_sigma
        self._clip = target_smoothing_clip
        self._alpha = alpha
        self._scaler = scaler
        # DDPGBaseImpl.build: critic, actor, deepcopy targets, optimisers
        self._q_func = create_continuous_q_function(observation_size, action_size, n_critics,
                                                    hidden_units)
        self._policy = DeterministicPolicy(VectorEncoder(observation_size, hidden_units),
                                           action_size)
        self._targ_q_func = copy.deepcopy(self._q_func)
        self._targ_policy = copy.deepcopy(self._policy)
        self._critic_optim = torch.optim.Adam(self._q_func.parameters(), lr=critic_learning_rate,
                                              betas=(0.9, 0.999), eps=1e-8)
        self._actor_optim = torch.optim.Adam(self._policy.parameters(), lr=actor_learning_rate,
                                             betas=(0.9, 0.999), eps=1e-8)

    def _scaled(self, batch: Batch) -> Batch:
        if self._scaler is None:
            return batch
        return Batch(self._scaler.transform(batch.observations), batch.actions, batch.rewards,
                     self._scaler.transform(batch.next_observations), batch.terminals,
                     batch.n_steps)

    def compute_target(self, batch: Batch, noise: torch.Tensor) -> torch.Tensor:
        """td3_impl.py:61-78 (torch.randn draw supplied)."""
        with torch.no_grad():
            action = self._targ_policy(batch.next_observations)
            scaled_noise = self._sigma * noise
            clipped_noise = scaled_noise.clamp(-self._clip, self._clip)
            smoothed_action = action + clipped_noise
            clipped_action = smoothed_action.clamp(-1.0, 1.0)
            return self._targ_q_func.compute_target(batch.next_observations, clipped_action,
                                                    reduction="min")

    def update_critic(self, batch: Batch, noise: torch.Tensor):
        """ddpg_impl.py:138-165."""
        batch = self._scaled(batch)
        self._critic_optim.zero_grad()
        q_tpn = self.compute_target(batch, noise)
        loss = self._q_func.compute_error(
            observations=batch.observations, actions=batch.actions, rewards=batch.rewards,
            target=q_tpn, terminals=batch.terminals, gamma=self._gamma ** batch.n_steps)
        loss.backward()
        self._critic_optim.step()
        return loss.cpu().detach().numpy()

    def compute_actor_loss(self, batch: Batch) -> torch.Tensor:
        """td3_plus_bc_impl.py:64-70."""
        action = self._policy(batch.observations)
        q_t = self._q_func(batch.observations, action, "none")[0]
        if not self._BC:
            return -q_t.mean()  # ddpg_impl.py:244-249
        lam = self._alpha / (q_t.abs().mean()).detach()
        return lam * -q_t.mean() + ((batch.actions - action) ** 2).mean()

    def update_actor(self, batch: Batch):
        """ddpg_impl.py:167-183."""
        batch = self._scaled(batch)
        self._actor_optim.zero_grad()
        loss = self.compute_actor_loss(batch)
        loss.backward()
        self._actor_optim.step()
        return loss.cpu().detach().numpy()

    def update_critic_target(self):
        soft_sync(self._targ_q_func, self._q_func, self._tau)

    def update_actor_target(self):
        soft_sync(self._targ_policy, self._policy, self._tau)

    def update(self, batch: Batch, noise: torch.Tensor, grad_step: int,
               update_actor_interval: int = 2) -> Dict[str, float]:
        """algos/td3_plus_bc.py:177-192."""
        metrics = {"critic_loss": float(self.update_critic(batch, noise))}
        if grad_step % update_actor_interval == 0:
            metrics["actor_loss"] = float(self.update_actor(batch))
            self.update_critic_target()
            self.update_actor_target()
        return metrics


class TD3Oracle(TD3PlusBCOracle):
    """TD3Impl (td3_impl.py:14-78): DDPG actor loss, smoothed target."""

    _BC = False

    def __init__(self, observation_size: int, action_size: int, **kw):
        kw.setdefault("alpha", 0.0)
        super().__init__(observation_size, action_size, **kw)


class DDPGOracle(TD3Oracle):
    """DDPGImpl (ddpg_impl.py:232-263) with the DDPG._update schedule."""

    def __init__(self, observation_size: int, action_size: int, n_critics: int = 1, **kw):
        super().__init__(observation_size, action_size, n_critics=n_critics,
                         target_smoothing_sigma=0.0, target_smoothing_clip=0.0, **kw)

    def compute_target(self, batch: Batch, noise: Optional[torch.Tensor] = None) -> torch.Tensor:
        """ddpg_impl.py:251-260 (no smoothing noise)."""
        with torch.no_grad():
            action = self._targ_policy(batch.next_observations)
            return self._targ_q_func.compute_target(batch.next_observations,
                                                    action.clamp(-1.0, 1.0), reduction="min")

    def update(self, batch: Batch, noise: Optional[torch.Tensor] = None, grad_step: int = 0,
               update_actor_interval: int = 1) -> Dict[str, float]:
        """algos/ddpg.py:167-174."""
        metrics = {"critic_loss": float(self.update_critic(batch, noise))}
        metrics["actor_loss"] = float(self.update_actor(batch))
        self.update_critic_target()
        self.update_actor_target()
        return metrics
