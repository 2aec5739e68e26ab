"""DroQ agent (reference: ``sheeprl/algos/droq/agent.py:16-200``): SAC with Dropout + LayerNorm
critics ("Dropout Q-Functions for Doubly Efficient RL", arXiv:2110.02034).

Layout: the reference keeps ``num_critics`` separate ``DROQCritic`` modules (Linear -> Dropout ->
LayerNorm -> ReLU, twice, then a Linear head, ``agent.py:16-56``) and updates them one after the other
(``droq.py:95-110``: critic i takes an optimiser step on loss_i, then its target gets its own EMA).
Here the critics are ONE stacked ensemble (``models/ensemble.py``: members' weights ``[n, out, in]``,
one GEMM / batched GEMM per layer for all members).  Member i only ever receives loss_i's gradient
and Adam is elementwise, so the batched update equals the reference's per-critic loop; the
per-critic API of the reference (``get_ith_q_value``, ``get_ith_target_q_value``, per-critic target
EMA) is kept as views of member i.
"""
from __future__ import annotations

from typing import Any, Dict, Optional, Union

import numpy as np
import torch
from torch import Tensor, nn

from sheeprl_prey_amd.algos.sac.agent import SACActor, SACAgent, SACCriticEnsemble


class DROQCritic(SACCriticEnsemble):
    """``num_critics`` DroQ critics, batched: Linear -> Dropout -> LayerNorm -> ReLU (x2) -> Linear
    (reference ``droq/agent.py:16-56``; ``forward`` returns ``[B, num_critics]``)."""

    def __init__(self, observation_dim: int, hidden_size: int = 256, num_critics: int = 2, dropout: float = 0.0):
        super().__init__(observation_dim, n=num_critics, hidden_size=hidden_size, dropout=dropout, layer_norm=True)
        self.dropout = float(dropout)


class DROQAgent(SACAgent):
    """Reference ``droq/agent.py:59-200`` over one batched critic ensemble (see the module docstring)."""

    def __init__(self, actor: SACActor, critic: DROQCritic, target_entropy: float, alpha: float = 1.0,
                 tau: float = 0.005, device: Union[str, torch.device] = "cpu"):
        if not isinstance(critic, DROQCritic):
            raise TypeError(f"DROQAgent needs a DROQCritic, got {type(critic).__name__}")
        super().__init__(actor, critic, target_entropy, alpha=alpha, tau=tau, device=device)

    @property
    def critics(self) -> nn.Module:
        """All critics (one stacked module; reference: a ``ModuleList`` of ``num_critics`` critics)."""
        return self.critic

    def get_ith_q_value(self, obs: Tensor, action: Tensor, critic_idx: int) -> Tensor:
        """Q_i(obs, action) ``[B, 1]`` (reference ``agent.py:172-173``)."""
        self._check_idx(critic_idx)
        return self.critic.member(obs, action, critic_idx)

    @torch.no_grad()
    def get_ith_target_q_value(self, obs: Tensor, action: Tensor, critic_idx: int) -> Tensor:
        """Target Q_i(obs, action) ``[B, 1]`` (reference ``agent.py:179-181``)."""
        self._check_idx(critic_idx)
        return self.critic_target.member(obs, action, critic_idx)

    @torch.no_grad()
    def qfs_target_ema(self, weight: Optional[Union[float, Tensor]] = None, critic_idx: Optional[int] = None) -> None:
        """theta'_i <- w theta_i + (1 - w) theta'_i for member ``critic_idx`` (reference ``agent.py:196-200``,
        called once per critic after its update), or for every member at once when ``critic_idx`` is None
        (what the batched trainer does: the members are independent, so it is the same update)."""
        if critic_idx is None:
            super().qfs_target_ema(weight)
            return
        self._check_idx(critic_idx)
        w = self.tau if weight is None else weight
        # every ensemble parameter is stacked over the members on dim 0: member i is the slice [i]
        for p, tp in zip(self.critic.parameters(), self.critic_target.parameters()):
            tp[critic_idx].lerp_(p[critic_idx], w)

    def _check_idx(self, critic_idx: int) -> None:
        if not 0 <= critic_idx < self.num_critics:
            raise ValueError(f"critic_idx {critic_idx} out of range for {self.num_critics} critics")


def build_agent(runner, cfg: Dict[str, Any], obs_dim: int, action_space, state: Optional[Dict[str, Any]] = None
                ) -> DROQAgent:
    """Actor + ``cfg.algo.critic.n`` DroQ critics (dropout ``cfg.algo.critic.dropout``) + target + log-alpha
    (reference ``droq/droq.py:200-225``); every rank starts from rank 0's weights."""
    act_dim = int(np.prod(action_space.shape))
    actor = SACActor(obs_dim, act_dim, cfg.distribution, cfg.algo.actor.hidden_size, action_space.low,
                     action_space.high)
    critic = DROQCritic(obs_dim + act_dim, hidden_size=cfg.algo.critic.hidden_size, num_critics=cfg.algo.critic.n,
                        dropout=float(cfg.algo.critic.get("dropout", 0.0)))
    agent = DROQAgent(actor, critic, target_entropy=-act_dim, alpha=cfg.algo.alpha.alpha, tau=cfg.algo.tau)
    if state is not None:
        agent.load_state_dict(state)
    agent = agent.to(runner.device)
    runner.setup_module(agent)
    return agent


__all__ = ["DROQAgent", "DROQCritic", "SACActor", "build_agent"]
