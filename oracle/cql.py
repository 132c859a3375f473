"""CPU restatement of CQLImpl / SACImpl / DDPGBaseImpl updates (continuous CQL).

TEST INFRASTRUCTURE (see oracle/__init__.py).  Follows, op for op and in the
same order:
  d3rlpy/algos/torch/cql_impl.py:95-243   (CQLImpl)
  d3rlpy/algos/torch/sac_impl.py:92-162   (SACImpl: build, actor loss, update_temp)
  d3rlpy/algos/torch/ddpg_impl.py:95-209  (update_critic / update_actor / targets)
  d3rlpy/algos/cql.py:234-258             (CQL._update schedule)
  d3rlpy/algos/torch/sac_impl.py:148-162  (SACImpl.compute_target: soft_q_backup, SACOracle)
  d3rlpy/algos/sac.py:195-214             (SAC._update schedule, SACOracle)
with every random draw passed in explicitly (``CQLNoise``).
"""
from __future__ import annotations

import copy
import math
from dataclasses import dataclass
from typing import Dict, Optional, Sequence

import numpy as np
import torch

from .models import (
    SquashedNormalPolicy,
    VectorEncoder,
    create_continuous_q_function,
    create_parameter,
    soft_sync,
)


@dataclass
class Batch:
    """TorchMiniBatch fields (torch_utility.py:152-193), fp32 CPU tensors."""

    observations: torch.Tensor
    actions: torch.Tensor
    rewards: torch.Tensor
    next_observations: torch.Tensor
    terminals: torch.Tensor
    n_steps: torch.Tensor

    @staticmethod
    def from_numpy(obs, act, rew, next_obs, term, n_steps) -> "Batch":
        f = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float32))  # noqa: E731
        return Batch(f(obs), f(act), f(rew).view(-1, 1), f(next_obs), f(term).view(-1, 1),
                     f(n_steps).view(-1, 1))


@dataclass
class CQLNoise:
    """All draws of one CQL._update call, in the reference's shapes.

    eps_temp:        (B, A)     update_temp        policy.sample_with_log_prob
    alpha_pi_t:      (N, B, A)  update_alpha       _compute_policy_is_values(obs_t)
    alpha_pi_tp1:    (N, B, A)  update_alpha       _compute_policy_is_values(obs_tp1)
    alpha_rand:      (B*N, A)   update_alpha       uniform_(-1, 1)
    critic_pi_t / critic_pi_tp1 / critic_rand:     same, inside update_critic
    eps_actor:       (B, A)     update_actor       policy.sample_with_log_prob
    eps_targ:        (B, A)     update_critic      soft target sample_with_log_prob(next_obs)
                                                   (soft_q_backup / SAC only; else None)
    """

    eps_temp: torch.Tensor
    alpha_pi_t: torch.Tensor
    alpha_pi_tp1: torch.Tensor
    alpha_rand: torch.Tensor
    critic_pi_t: torch.Tensor
    critic_pi_tp1: torch.Tensor
    critic_rand: torch.Tensor
    eps_actor: torch.Tensor
    eps_targ: Optional[torch.Tensor] = None

    def tensors(self) -> Dict[str, torch.Tensor]:
        """The draws that exist (eps_targ only for a soft target)."""
        return {k: getattr(self, k) for k in self.__dataclass_fields__
                if getattr(self, k) is not None}

    @staticmethod
    def draw(gen: torch.Generator, B: int, A: int, N: int,
             soft_target: bool = False) -> "CQLNoise":
        n = lambda *s: torch.randn(*s, generator=gen)  # noqa: E731
        u = lambda *s: torch.rand(*s, generator=gen) * 2.0 - 1.0  # noqa: E731
        nz = CQLNoise(n(B, A), n(N, B, A), n(N, B, A), u(B * N, A),
                      n(N, B, A), n(N, B, A), u(B * N, A), n(B, A))
        if soft_target:  # drawn last: the other draws keep their stream
            nz.eps_targ = n(B, A)
        return nz


class CQLOracle:
    """CQLImpl with the reference defaults (algos/cql.py:139-161)."""

    def __init__(
        self,
        observation_size: int,
        action_size: int,
        actor_learning_rate: float = 1e-4,
        critic_learning_rate: float = 3e-4,
        temp_learning_rate: float = 1e-4,
        alpha_learning_rate: float = 1e-4,
        gamma: float = 0.99,
        tau: float = 0.005,
        n_critics: int = 2,
        initial_temperature: float = 1.0,
        initial_alpha: float = 1.0,
        alpha_threshold: float = 10.0,
        conservative_weight: float = 5.0,
        n_action_samples: int = 10,
        soft_q_backup: bool = False,
        hidden_units: Sequence[int] = (256, 256),
        betas=(0.9, 0.999),
        eps: float = 1e-8,
        seed: int = 0,
    ):
        torch.manual_seed(seed)
        self._observation_size = observation_size
        self._action_size = action_size
        self._gamma = gamma
        self._tau = tau
        self._n_critics = n_critics
        self._alpha_threshold = alpha_threshold
        self._conservative_weight = conservative_weight
        self._n_action_samples = n_action_samples
        self._soft_q_backup = soft_q_backup
        self._temp_learning_rate = temp_learning_rate
        self._alpha_learning_rate = alpha_learning_rate
        # build order: CQLImpl.build -> _build_alpha, SACImpl.build -> _build_temperature,
        # DDPGBaseImpl.build -> critic, actor, deepcopy targets, optimizers
        self._log_alpha = create_parameter((1, 1), math.log(initial_alpha))
        self._log_temp = create_parameter((1, 1), math.log(initial_temperature))
        self._q_func = create_continuous_q_function(
            observation_size, action_size, n_critics, hidden_units)
        self._policy = SquashedNormalPolicy(VectorEncoder(observation_size, hidden_units),
                                            action_size)
        self._targ_q_func = copy.deepcopy(self._q_func)
        self._targ_policy = copy.deepcopy(self._policy)
        adam = lambda params, lr: torch.optim.Adam(params, lr=lr, betas=betas, eps=eps)  # noqa
        self._critic_optim = adam(self._q_func.parameters(), critic_learning_rate)
        self._actor_optim = adam(self._policy.parameters(), actor_learning_rate)
        self._temp_optim = adam(self._log_temp.parameters(), temp_learning_rate)
        self._alpha_optim = adam(self._log_alpha.parameters(), alpha_learning_rate)

    # ------------------------------------------------------------------ steps
    def update_temp(self, batch: Batch, eps: torch.Tensor):
        """sac_impl.py:123-146."""
        self._temp_optim.zero_grad()
        with torch.no_grad():
            _, log_prob = self._policy.sample_with_log_prob(batch.observations, eps)
            targ_temp = log_prob - self._action_size
        loss = -(self._log_temp().exp() * targ_temp).mean()
        loss.backward()
        self._temp_optim.step()
        cur_temp = self._log_temp().exp().cpu().detach().numpy()[0][0]
        return loss.cpu().detach().numpy(), cur_temp

    def _compute_policy_is_values(self, policy_obs, value_obs, eps_n):
        """cql_impl.py:143-171."""
        with torch.no_grad():
            policy_actions, n_log_probs = self._policy.sample_n_with_log_prob(policy_obs, eps_n)
        obs_shape = value_obs.shape
        repeated_obs = value_obs.expand(self._n_action_samples, *obs_shape)
        transposed_obs = repeated_obs.transpose(0, 1)
        flat_obs = transposed_obs.reshape(-1, *obs_shape[1:])
        flat_policy_acts = policy_actions.reshape(-1, self._action_size)
        policy_values = self._q_func(flat_obs, flat_policy_acts, "none")
        policy_values = policy_values.view(self._n_critics, obs_shape[0], self._n_action_samples)
        log_probs = n_log_probs.view(1, -1, self._n_action_samples)
        return policy_values - log_probs

    def _compute_random_is_values(self, obs, random_actions):
        """cql_impl.py:173-194 (uniform_(-1, 1) draw supplied)."""
        repeated_obs = obs.expand(self._n_action_samples, *obs.shape)
        transposed_obs = repeated_obs.transpose(0, 1)
        flat_obs = transposed_obs.reshape(-1, *obs.shape[1:])
        random_values = self._q_func(flat_obs, random_actions, "none")
        random_values = random_values.view(self._n_critics, obs.shape[0], self._n_action_samples)
        random_log_probs = math.log(0.5 ** self._action_size)
        return random_values - random_log_probs

    def _compute_conservative_loss(self, obs_t, act_t, obs_tp1, pi_t, pi_tp1, rand):
        """cql_impl.py:196-223."""
        policy_values_t = self._compute_policy_is_values(obs_t, obs_t, pi_t)
        policy_values_tp1 = self._compute_policy_is_values(obs_tp1, obs_t, pi_tp1)
        random_values = self._compute_random_is_values(obs_t, rand)
        target_values = torch.cat([policy_values_t, policy_values_tp1, random_values], dim=2)
        logsumexp = torch.logsumexp(target_values, dim=2, keepdim=True)
        data_values = self._q_func(obs_t, act_t, "none")
        loss = logsumexp.mean(dim=0).mean() - data_values.mean(dim=0).mean()
        scaled_loss = self._conservative_weight * loss
        clipped_alpha = self._log_alpha().exp().clamp(0, 1e6)[0][0]
        return clipped_alpha * (scaled_loss - self._alpha_threshold)

    def update_alpha(self, batch: Batch, noise: CQLNoise):
        """cql_impl.py:119-141."""
        self._alpha_optim.zero_grad()
        loss = -self._compute_conservative_loss(
            batch.observations, batch.actions, batch.next_observations,
            noise.alpha_pi_t, noise.alpha_pi_tp1, noise.alpha_rand)
        loss.backward()
        self._alpha_optim.step()
        cur_alpha = self._log_alpha().exp().cpu().detach().numpy()[0][0]
        return loss.cpu().detach().numpy(), cur_alpha

    def compute_target(self, batch: Batch, noise: Optional[CQLNoise] = None):
        """cql_impl.py:225-243."""
        if self._soft_q_backup:
            return self._compute_soft_target(batch, noise.eps_targ)
        with torch.no_grad():
            action = self._policy.best_action(batch.next_observations)
            return self._targ_q_func.compute_target(batch.next_observations, action,
                                                    reduction="min")

    def _compute_soft_target(self, batch: Batch, eps: torch.Tensor):
        """SACImpl.compute_target (sac_impl.py:148-162), sample noise supplied."""
        with torch.no_grad():
            action, log_prob = self._policy.sample_with_log_prob(batch.next_observations, eps)
            entropy = self._log_temp().exp() * log_prob
            target = self._targ_q_func.compute_target(batch.next_observations, action,
                                                      reduction="min")
            return target - entropy

    def compute_critic_loss(self, batch: Batch, q_tpn: torch.Tensor, noise: CQLNoise):
        """cql_impl.py:110-117 (DDPGBaseImpl's TD error + conservative loss)."""
        loss = self._q_func.compute_error(
            observations=batch.observations, actions=batch.actions, rewards=batch.rewards,
            target=q_tpn, terminals=batch.terminals, gamma=self._gamma ** batch.n_steps)
        return loss + self._compute_conservative_loss(
            batch.observations, batch.actions, batch.next_observations,
            noise.critic_pi_t, noise.critic_pi_tp1, noise.critic_rand)

    def update_critic(self, batch: Batch, noise: CQLNoise):
        """ddpg_impl.py:138-165."""
        self._critic_optim.zero_grad()
        q_tpn = self.compute_target(batch, noise)
        loss = self.compute_critic_loss(batch, q_tpn, noise)
        loss.backward()
        self._critic_optim.step()
        return loss.cpu().detach().numpy()

    def compute_actor_loss(self, batch: Batch, eps: torch.Tensor):
        """sac_impl.py:114-121."""
        action, log_prob = self._policy.sample_with_log_prob(batch.observations, eps)
        entropy = self._log_temp().exp() * log_prob
        q_t = self._q_func(batch.observations, action, "min")
        return (entropy - q_t).mean()

    def update_actor(self, batch: Batch, eps: torch.Tensor):
        """ddpg_impl.py:167-183."""
        self._actor_optim.zero_grad()
        loss = self.compute_actor_loss(batch, eps)
        loss.backward()
        self._actor_optim.step()
        return loss.cpu().detach().numpy()

    def update_critic_target(self):
        soft_sync(self._targ_q_func, self._q_func, self._tau)

    def update_actor_target(self):
        soft_sync(self._targ_policy, self._policy, self._tau)

    def update(self, batch: Batch, noise: CQLNoise) -> Dict[str, float]:
        """algos/cql.py:234-258 (CQL._update)."""
        metrics = {}
        if self._temp_learning_rate > 0:
            temp_loss, temp = self.update_temp(batch, noise.eps_temp)
            metrics.update({"temp_loss": float(temp_loss), "temp": float(temp)})
        if self._alpha_learning_rate > 0:
            alpha_loss, alpha = self.update_alpha(batch, noise)
            metrics.update({"alpha_loss": float(alpha_loss), "alpha": float(alpha)})
        metrics["critic_loss"] = float(self.update_critic(batch, noise))
        metrics["actor_loss"] = float(self.update_actor(batch, noise.eps_actor))
        self.update_critic_target()
        self.update_actor_target()
        return metrics

    # ------------------------------------------------------------- inspection
    def grads(self) -> Dict[str, torch.Tensor]:
        out = {}
        for name, p in self._q_func.named_parameters():
            out["q." + name] = p.grad.detach().clone() if p.grad is not None else None
        for name, p in self._policy.named_parameters():
            out["pi." + name] = p.grad.detach().clone() if p.grad is not None else None
        return out


class SACOracle(CQLOracle):
    """SACImpl (sac_impl.py:27-162) with the reference defaults
    (algos/sac.py:118-140): no conservative term, no alpha, soft target.
    Construction draws the same weights as CQLOracle with the same seed
    (the log_alpha parameter of CQLImpl consumes no random numbers)."""

    def __init__(self, observation_size: int, action_size: int,
                 actor_learning_rate: float = 3e-4, critic_learning_rate: float = 3e-4,
                 temp_learning_rate: float = 3e-4, **kw):
        super().__init__(observation_size, action_size, actor_learning_rate=actor_learning_rate,
                         critic_learning_rate=critic_learning_rate,
                         temp_learning_rate=temp_learning_rate, alpha_learning_rate=0.0,
                         n_action_samples=0, soft_q_backup=True, **kw)

    def compute_critic_loss(self, batch: Batch, q_tpn: torch.Tensor, noise: CQLNoise):
        """DDPGBaseImpl.compute_critic_loss (ddpg_impl.py:154-167)."""
        return self._q_func.compute_error(
            observations=batch.observations, actions=batch.actions, rewards=batch.rewards,
            target=q_tpn, terminals=batch.terminals, gamma=self._gamma ** batch.n_steps)

    def update(self, batch: Batch, noise: CQLNoise) -> Dict[str, float]:
        """algos/sac.py:195-214 (SAC._update)."""
        metrics = {}
        if self._temp_learning_rate > 0:
            temp_loss, temp = self.update_temp(batch, noise.eps_temp)
            metrics.update({"temp_loss": float(temp_loss), "temp": float(temp)})
        metrics["critic_loss"] = float(self.update_critic(batch, noise))
        metrics["actor_loss"] = float(self.update_actor(batch, noise.eps_actor))
        self.update_critic_target()
        self.update_actor_target()
        return metrics
