"""DroQ agent (reference: ``sheeprl/algos/droq/agent.py:16-200``): SAC with Dropout + LayerNorm
critics ("Dropout Q-Functions for Doubly Efficient RL", arXiv:2110.02034).

The critics are the SAC ``SACCriticEnsemble`` built with ``dropout=p, layer_norm=True``; the
reference's per-critic sequential updates and per-critic EMA (``droq.py:95-110``) are one batched
ensemble update (member i only receives loss_i's gradient - see ``models/ensemble.py``)."""
from __future__ import annotations

from sheeprl_prey_amd.algos.sac.agent import SACActor, SACAgent, SACCriticEnsemble, build_agent


class DROQCritic(SACCriticEnsemble):
    """``n`` DroQ critics: Linear -> Dropout -> LayerNorm -> ReLU (x2) -> Linear, batched."""

    def __init__(self, observation_dim: int, hidden_size: int = 256, num_critics: int = 2, dropout: float = 0.0):
        super().__init__(observation_dim, n=num_critics, hidden_size=hidden_size, dropout=dropout, layer_norm=True)


DROQAgent = SACAgent

__all__ = ["DROQAgent", "DROQCritic", "SACActor", "build_agent"]
