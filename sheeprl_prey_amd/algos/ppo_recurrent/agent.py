"""Recurrent PPO agent (reference: ``sheeprl/algos/ppo_recurrent/agent.py:16-318``).

features(obs) || prev_action -> [pre-MLP] -> LSTM -> [post-MLP] -> actor heads / critic.

Padded training sequences are run straight through the LSTM instead of ``pack_padded_sequence``:
the padding sits at the END of every sequence, so each valid step's output is computed before any
padded input is seen (identical to the packed result), only the final state differs - and the
training loss never uses it.  That removes the per-minibatch device->host ``lengths`` copy the
packed path needs.
"""
from __future__ import annotations

from math import prod
from typing import Any, Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn
from torch import Tensor
from torch.distributions import Independent, Normal

from sheeprl_prey_amd import ops
from sheeprl_prey_amd.algos.ppo.agent import CNNEncoder, MLPEncoder, _act
from sheeprl_prey_amd.models.models import MLP, MultiEncoder
from sheeprl_prey_amd.utils.distribution import OneHotCategoricalValidateArgs


def _opt_mlp(input_dim: int, cfg) -> Tuple[nn.Module, int]:
    if not cfg.apply:
        return nn.Identity(), input_dim
    m = MLP(input_dims=input_dim, output_dim=None, hidden_sizes=[cfg.dense_units], activation=_act(cfg.activation),
            layer_args={"bias": cfg.bias}, norm_layer=[nn.LayerNorm] if cfg.layer_norm else None,
            norm_args=[{"normalized_shape": cfg.dense_units, "eps": 1e-3}] if cfg.layer_norm else None)
    return m, cfg.dense_units


class RecurrentModel(nn.Module):
    def __init__(self, input_size: int, lstm_hidden_size: int, pre_rnn_mlp_cfg, post_rnn_mlp_cfg) -> None:
        super().__init__()
        self._pre_mlp, d = _opt_mlp(input_size, pre_rnn_mlp_cfg)
        self._lstm = nn.LSTM(input_size=d, hidden_size=lstm_hidden_size, batch_first=False)
        self._post_mlp, self._output_dim = _opt_mlp(lstm_hidden_size, post_rnn_mlp_cfg)

    @property
    def output_dim(self) -> int:
        return self._output_dim

    def forward(self, input: Tensor, states: Tuple[Tensor, Tensor], mask: Optional[Tensor] = None):
        x = self._pre_mlp(input)
        if ops.lstm_supported(self._lstm, x):  # persistent HIP LSTM, one launch per direction (K18)
            out, states = ops.lstm_seq(self._lstm, x, states)
        else:
            out, states = self._lstm(x, states)
        shape = out.shape
        return self._post_mlp(out.reshape(-1, shape[-1])).view(*shape[:-1], -1), states


class _SeqCNNEncoder(CNNEncoder):
    """NatureCNN over ``[T, B, C, H, W]`` (leading dims folded into the batch)."""

    def forward(self, obs: Dict[str, Tensor]) -> Tensor:
        x = torch.cat([obs[k] for k in self.keys], dim=-3)
        lead = x.shape[:-3]
        return self.model(x.reshape(-1, *x.shape[-3:])).view(*lead, -1)


class RecurrentPPOAgent(nn.Module):
    def __init__(self, actions_dim: Sequence[int], obs_space, encoder_cfg, rnn_cfg, actor_cfg, critic_cfg,
                 cnn_keys: Sequence[str], mlp_keys: Sequence[str], is_continuous: bool,
                 distribution_cfg: Dict[str, Any], num_envs: int = 1, screen_size: int = 64, device="cpu"):
        super().__init__()
        self.num_envs = num_envs
        self.actions_dim = list(actions_dim)
        self.distribution_cfg = distribution_cfg
        self.rnn_hidden_size = rnn_cfg.lstm.hidden_size
        self.device = torch.device(device) if isinstance(device, str) else device
        in_channels = sum(prod(obs_space[k].shape[:-2]) for k in cnn_keys)
        mlp_input_dim = sum(obs_space[k].shape[0] for k in mlp_keys)
        cnn_encoder = _SeqCNNEncoder(in_channels, encoder_cfg.cnn_features_dim, screen_size, cnn_keys) if cnn_keys else None
        mlp_encoder = (MLPEncoder(mlp_input_dim, encoder_cfg.mlp_features_dim, mlp_keys, encoder_cfg.dense_units,
                                  encoder_cfg.mlp_layers, _act(encoder_cfg.dense_act), encoder_cfg.layer_norm)
                       if mlp_keys else None)
        self.feature_extractor = MultiEncoder(cnn_encoder, mlp_encoder)
        self.is_continuous = is_continuous
        features_dim = self.feature_extractor.output_dim
        self.rnn = RecurrentModel(int(features_dim + sum(actions_dim)), rnn_cfg.lstm.hidden_size,
                                  rnn_cfg.pre_rnn_mlp, rnn_cfg.post_rnn_mlp)

        def mlp(out, cfg):
            n = cfg.mlp_layers
            return MLP(input_dims=self.rnn_hidden_size, output_dim=out, hidden_sizes=[cfg.dense_units] * n,
                       activation=_act(cfg.dense_act), flatten_dim=None,
                       norm_layer=[nn.LayerNorm] * n if cfg.layer_norm else None,
                       norm_args=[{"normalized_shape": cfg.dense_units} for _ in range(n)] if cfg.layer_norm else None)

        self.critic = mlp(1, critic_cfg)
        self.actor_backbone = mlp(None, actor_cfg)
        if is_continuous:
            self.actor_heads = nn.ModuleList([nn.Linear(actor_cfg.dense_units, int(sum(actions_dim)) * 2)])
        else:
            self.actor_heads = nn.ModuleList([nn.Linear(actor_cfg.dense_units, a) for a in actions_dim])
        self._initial_states = self.reset_hidden_states()

    @property
    def initial_states(self) -> Tuple[Tensor, Tensor]:
        return self._initial_states

    @initial_states.setter
    def initial_states(self, value) -> None:
        self._initial_states = value

    def reset_hidden_states(self) -> Tuple[Tensor, Tensor]:
        z = torch.zeros(1, self.num_envs, self.rnn_hidden_size, device=self.device)
        return (z, z.clone())

    def get_pre_dist(self, x: Tensor):
        feat = self.actor_backbone(x)
        pre = [h(feat) for h in self.actor_heads]
        if self.is_continuous:
            mean, log_std = torch.chunk(pre[0], 2, -1)
            return (mean, log_std.exp())
        return tuple(pre)

    def get_values(self, x: Tensor) -> Tensor:
        return self.critic(x)

    def get_sampled_actions(self, pre_dist, actions: Optional[List[Tensor]] = None):
        va = self.distribution_cfg.validate_args
        if self.is_continuous:
            dist = Independent(Normal(*pre_dist, validate_args=va), 1, validate_args=va)
            a = dist.sample() if actions is None else actions[0]
            return (a,), dist.log_prob(a).unsqueeze(-1), dist.entropy().unsqueeze(-1)
        from sheeprl_prey_amd.algos.ppo.heads import categorical_heads

        return categorical_heads(list(pre_dist), actions)

    def forward(self, obs: Dict[str, Tensor], prev_actions: Tensor, prev_states: Tuple[Tensor, Tensor],
                actions: Optional[List[Tensor]] = None, mask: Optional[Tensor] = None):
        emb = self.feature_extractor(obs)
        out, states = self.rnn(torch.cat((emb, prev_actions), -1), prev_states, mask)
        values = self.get_values(out)
        acts, logp, ent = self.get_sampled_actions(self.get_pre_dist(out), actions)
        return acts, logp, ent, values, states

    def get_greedy_actions(self, obs: Dict[str, Tensor], prev_states, prev_actions: Tensor, mask=None):
        emb = self.feature_extractor(obs)
        out, states = self.rnn(torch.cat((emb, prev_actions), -1), prev_states, mask)
        pre = self.get_pre_dist(out)
        if self.is_continuous:
            return (pre[0],), states
        return tuple(OneHotCategoricalValidateArgs(logits=l, validate_args=False).mode for l in pre), states
