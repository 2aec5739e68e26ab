"""PPO agent (reference: ``sheeprl/algos/ppo/agent.py:14-196``).

MultiEncoder (NatureCNN for pixels, MLP for vectors) -> actor MLP + heads / critic MLP.
Continuous: Independent Normal(mean, exp(log_std)) from one head; discrete/multi-discrete:
one categorical per head.  The discrete log-prob/entropy path runs through
``sheeprl_prey_amd.algos.ppo.heads`` (fused on GPU)."""
from __future__ import annotations

from math import prod
from typing import Any, Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn
from torch import Tensor
from torch.distributions import Independent, Normal

from sheeprl_prey_amd.models.models import MLP, MultiEncoder, NatureCNN
from sheeprl_prey_amd.utils.distribution import OneHotCategoricalValidateArgs


def _act(name: str):
    from sheeprl_prey_amd.config.instantiate import get_class

    return get_class(name) if isinstance(name, str) else name


class CNNEncoder(nn.Module):
    def __init__(self, in_channels: int, features_dim: int, screen_size: int, keys: Sequence[str]) -> None:
        super().__init__()
        self.keys = keys
        self.input_dim = (in_channels, screen_size, screen_size)
        self.output_dim = features_dim
        self.model = NatureCNN(in_channels=in_channels, features_dim=features_dim, screen_size=screen_size)

    def forward(self, obs: Dict[str, Tensor]) -> Tensor:
        return self.model(torch.cat([obs[k] for k in self.keys], dim=-3))


class MLPEncoder(nn.Module):
    def __init__(self, input_dim: int, features_dim: int, keys: Sequence[str], dense_units: int = 64, mlp_layers: int = 2,
                 dense_act=nn.ReLU, layer_norm: bool = False) -> None:
        super().__init__()
        self.keys = keys
        self.input_dim = input_dim
        self.output_dim = features_dim
        self.model = MLP(
            input_dim, features_dim, [dense_units] * mlp_layers, activation=dense_act,
            norm_layer=[nn.LayerNorm for _ in range(mlp_layers)] if layer_norm else None,
            norm_args=[{"normalized_shape": dense_units} for _ in range(mlp_layers)] if layer_norm else None,
        )

    def forward(self, obs: Dict[str, Tensor]) -> Tensor:
        return self.model(torch.cat([obs[k] for k in self.keys], dim=-1))


def _mlp(input_dim, output_dim, cfg) -> MLP:
    n = cfg.mlp_layers
    return MLP(
        input_dims=input_dim, output_dim=output_dim, hidden_sizes=[cfg.dense_units] * n, activation=_act(cfg.dense_act),
        flatten_dim=None,
        norm_layer=[nn.LayerNorm for _ in range(n)] if cfg.layer_norm else None,
        norm_args=[{"normalized_shape": cfg.dense_units} for _ in range(n)] if cfg.layer_norm else None,
    )


class PPOAgent(nn.Module):
    def __init__(self, actions_dim: List[int], obs_space, encoder_cfg: Dict[str, Any], actor_cfg: Dict[str, Any],
                 critic_cfg: Dict[str, Any], cnn_keys: Sequence[str], mlp_keys: Sequence[str], screen_size: int,
                 distribution_cfg: Dict[str, Any], is_continuous: bool = False):
        super().__init__()
        self.distribution_cfg = distribution_cfg
        self.actions_dim = list(actions_dim)
        in_channels = sum(prod(obs_space[k].shape[:-2]) for k in cnn_keys)
        mlp_input_dim = sum(obs_space[k].shape[0] for k in mlp_keys)
        cnn_encoder = CNNEncoder(in_channels, encoder_cfg.cnn_features_dim, screen_size, cnn_keys) if cnn_keys else None
        mlp_encoder = (
            MLPEncoder(mlp_input_dim, encoder_cfg.mlp_features_dim, mlp_keys, encoder_cfg.dense_units,
                       encoder_cfg.mlp_layers, _act(encoder_cfg.dense_act), encoder_cfg.layer_norm)
            if mlp_keys else None
        )
        self.feature_extractor = MultiEncoder(cnn_encoder, mlp_encoder)
        self.is_continuous = is_continuous
        features_dim = self.feature_extractor.output_dim
        self.critic = _mlp(features_dim, 1, critic_cfg)
        self.actor_backbone = _mlp(features_dim, None, actor_cfg)
        if is_continuous:
            self.actor_heads = nn.ModuleList([nn.Linear(actor_cfg.dense_units, sum(actions_dim) * 2)])
        else:
            self.actor_heads = nn.ModuleList([nn.Linear(actor_cfg.dense_units, a) for a in actions_dim])

    def forward(self, obs: Dict[str, Tensor], actions: Optional[List[Tensor]] = None) -> Tuple[Sequence[Tensor], Tensor, Tensor, Tensor]:
        feat = self.feature_extractor(obs)
        out = self.actor_backbone(feat)
        pre_dist = [head(out) for head in self.actor_heads]
        values = self.critic(feat)
        va = self.distribution_cfg.validate_args
        if self.is_continuous:
            mean, log_std = torch.chunk(pre_dist[0], chunks=2, dim=-1)
            std = log_std.exp()
            normal = Independent(Normal(mean, std, validate_args=va), 1, validate_args=va)
            # reparameterised draw (same law as Normal.sample; torch.normal on expanded operands is
            # not capturable in a hipGraph)
            act = (mean + std * torch.randn_like(mean)).detach() if actions is None else actions[0]
            return (act,), normal.log_prob(act).unsqueeze(-1), normal.entropy().unsqueeze(-1), values
        from sheeprl_prey_amd.algos.ppo.heads import categorical_heads

        acts, logp, ent = categorical_heads(pre_dist, actions)
        return acts, logp, ent, values

    def get_value(self, obs: Dict[str, Tensor]) -> Tensor:
        return self.critic(self.feature_extractor(obs))

    def get_greedy_actions(self, obs: Dict[str, Tensor]) -> Sequence[Tensor]:
        out = self.actor_backbone(self.feature_extractor(obs))
        pre_dist = [head(out) for head in self.actor_heads]
        if self.is_continuous:
            return [torch.chunk(pre_dist[0], 2, -1)[0]]
        return tuple(OneHotCategoricalValidateArgs(logits=l, validate_args=False).mode for l in pre_dist)
