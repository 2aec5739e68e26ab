"""DreamerV1 agent (reference: ``sheeprl/algos/dreamer_v1/agent.py:23-529``).

Continuous Gaussian RSSM: recurrent model = Linear+ELU -> GRU; representation / transition MLPs
emit (mean, pre-std) and the state is a reparameterised Normal sample with
``std = softplus(pre) + min_std``.  Encoders / decoders / actor are the DreamerV2 ones (no LN).
"""
from __future__ import annotations

from typing import Any, Dict, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F
from torch import Tensor, nn
from torch.distributions import Normal

from sheeprl_prey_amd import ops
from sheeprl_prey_amd.algos.dreamer_v2.agent import Actor as DV2Actor
from sheeprl_prey_amd.algos.dreamer_v2.agent import CNNDecoder, CNNEncoder, MLPDecoder, MLPEncoder, _act
from sheeprl_prey_amd.algos.dreamer_v2.agent import MinedojoActor as DV2MinedojoActor
from sheeprl_prey_amd.config.instantiate import get_class
from sheeprl_prey_amd.models.models import MLP, MultiDecoder, MultiEncoder
from sheeprl_prey_amd.models.world_model import WorldModel
from sheeprl_prey_amd.utils.distribution import OneHotCategoricalValidateArgs
from sheeprl_prey_amd.utils.utils import init_weights

Actor = DV2Actor
MinedojoActor = DV2MinedojoActor


def compute_stochastic_state(state_information: Tensor, min_std: float = 0.1) -> Tuple[Tuple[Tensor, Tensor], Tensor]:
    """(mean, std), rsample of Normal(mean, softplus(pre_std) + min_std) (reference ``dreamer_v1/utils.py:50-74``)."""
    mean, std = torch.chunk(state_information, 2, -1)
    std = F.softplus(std) + min_std
    return (mean, std), mean + std * torch.randn_like(mean)


class RecurrentModel(nn.Module):
    def __init__(self, input_size: int, recurrent_state_size: int, activation=nn.ELU) -> None:
        super().__init__()
        self.mlp = nn.Sequential(nn.Linear(input_size, recurrent_state_size), activation())
        self.rnn = nn.GRU(recurrent_state_size, recurrent_state_size)

    def forward(self, input: Tensor, recurrent_state: Tensor) -> Tuple[Tensor, Tensor]:
        # GRU gate math fused in one kernel each way on the GPU (K19); projections stay library GEMMs
        return ops.gru_step(self.rnn, self.mlp(input), recurrent_state)


class RSSM(nn.Module):
    def __init__(self, recurrent_model: nn.Module, representation_model: nn.Module, transition_model: nn.Module,
                 distribution_cfg: Dict[str, Any], min_std: float = 0.1) -> None:
        super().__init__()
        self.recurrent_model = recurrent_model
        self.representation_model = representation_model
        self.transition_model = transition_model
        self.min_std = min_std
        self.distribution_cfg = distribution_cfg

    def dynamic(self, posterior: Tensor, recurrent_state: Tensor, action: Tensor, embedded_obs: Tensor):
        recurrent_out, recurrent_state = self.recurrent_model(torch.cat((posterior, action), -1), recurrent_state)
        prior_mean_std, prior = self._transition(recurrent_out)
        posterior_mean_std, posterior = self._representation(recurrent_state, embedded_obs)
        return recurrent_state, posterior, prior, posterior_mean_std, prior_mean_std

    def _representation(self, recurrent_state: Tensor, embedded_obs: Tensor):
        return compute_stochastic_state(self.representation_model(torch.cat((recurrent_state, embedded_obs), -1)),
                                        self.min_std)

    def _transition(self, recurrent_out: Tensor):
        return compute_stochastic_state(self.transition_model(recurrent_out), self.min_std)

    def imagination(self, stochastic_state: Tensor, recurrent_state: Tensor, actions: Tensor) -> Tuple[Tensor, Tensor]:
        out, recurrent_state = self.recurrent_model(torch.cat((stochastic_state, actions), -1), recurrent_state)
        _, prior = self._transition(out)
        return prior, recurrent_state


class PlayerDV1(nn.Module):
    def __init__(self, encoder: nn.Module, recurrent_model: nn.Module, representation_model: nn.Module,
                 actor: nn.Module, actions_dim: Sequence[int], expl_amount: float, num_envs: int, stochastic_size: int,
                 recurrent_state_size: int, device, min_std: float = 0.1) -> None:
        super().__init__()
        self.encoder = encoder
        self.recurrent_model = recurrent_model
        self.representation_model = representation_model
        self.actor = actor
        self.device = device
        self.expl_amount = expl_amount
        self.actions_dim = actions_dim
        self.stochastic_size = stochastic_size
        self.recurrent_state_size = recurrent_state_size
        self.num_envs = num_envs
        self.min_std = min_std
        self.init_states()

    def init_states(self, reset_envs: Optional[Sequence[int]] = None) -> None:
        if reset_envs is None or len(reset_envs) == 0:
            self.actions = torch.zeros(1, self.num_envs, int(np.sum(self.actions_dim)), device=self.device)
            self.recurrent_state = torch.zeros(1, self.num_envs, self.recurrent_state_size, device=self.device)
            self.stochastic_state = torch.zeros(1, self.num_envs, self.stochastic_size, device=self.device)
        else:
            self.actions[:, reset_envs] = 0
            self.recurrent_state[:, reset_envs] = 0
            self.stochastic_state[:, reset_envs] = 0

    def get_exploration_action(self, obs: Dict[str, Tensor], is_continuous: bool, mask=None):
        actions = self.get_greedy_action(obs, mask=mask)
        if is_continuous:
            self.actions = torch.cat(actions, -1)
            if self.expl_amount > 0.0:
                self.actions = torch.clip(Normal(self.actions, self.expl_amount).sample(), -1, 1)
            expl = [self.actions]
        else:
            expl = []
            for act in actions:
                sample = OneHotCategoricalValidateArgs(logits=torch.zeros_like(act), validate_args=False).sample()
                expl.append(torch.where(torch.rand(act.shape[:1], device=self.device) < self.expl_amount, sample, act))
            self.actions = torch.cat(expl, -1)
        return tuple(expl)

    def get_greedy_action(self, obs: Dict[str, Tensor], is_training: bool = True, mask=None):
        embedded_obs = self.encoder(obs)
        _, self.recurrent_state = self.recurrent_model(torch.cat((self.stochastic_state, self.actions), -1),
                                                       self.recurrent_state)
        _, self.stochastic_state = compute_stochastic_state(
            self.representation_model(torch.cat((self.recurrent_state, embedded_obs), -1)), self.min_std)
        actions, _ = self.actor(torch.cat((self.stochastic_state, self.recurrent_state), -1), is_training, mask)
        self.actions = torch.cat(actions, -1)
        return actions


def build_models(runner, actions_dim: Sequence[int], is_continuous: bool, cfg: Dict[str, Any], obs_space,
                 world_model_state=None, actor_state=None, critic_state=None):
    wm = cfg.algo.world_model
    latent_state_size = wm.stochastic_size + wm.recurrent_model.recurrent_state_size
    cnn_encoder = (CNNEncoder(cfg.cnn_keys.encoder, [int(np.prod(obs_space[k].shape[:-2])) for k in cfg.cnn_keys.encoder],
                              obs_space[cfg.cnn_keys.encoder[0]].shape[-2:], wm.encoder.cnn_channels_multiplier, False,
                              _act(wm.encoder.cnn_act)) if cfg.cnn_keys.encoder else None)
    mlp_encoder = (MLPEncoder(cfg.mlp_keys.encoder, [obs_space[k].shape[0] for k in cfg.mlp_keys.encoder],
                              wm.encoder.mlp_layers, wm.encoder.dense_units, False, _act(wm.encoder.dense_act))
                   if cfg.mlp_keys.encoder else None)
    encoder = MultiEncoder(cnn_encoder, mlp_encoder)
    recurrent_model = RecurrentModel(int(sum(actions_dim) + wm.stochastic_size), wm.recurrent_model.recurrent_state_size,
                                     _act(wm.recurrent_model.dense_act))
    representation_model = MLP(input_dims=wm.recurrent_model.recurrent_state_size + encoder.output_dim,
                               output_dim=wm.stochastic_size * 2, hidden_sizes=[wm.representation_model.hidden_size],
                               activation=_act(wm.representation_model.dense_act), flatten_dim=None)
    transition_model = MLP(input_dims=wm.recurrent_model.recurrent_state_size, output_dim=wm.stochastic_size * 2,
                           hidden_sizes=[wm.transition_model.hidden_size],
                           activation=_act(wm.transition_model.dense_act), flatten_dim=None)
    rssm = RSSM(recurrent_model.apply(init_weights), representation_model.apply(init_weights),
                transition_model.apply(init_weights), cfg.distribution, min_std=wm.min_std)
    cnn_decoder = (CNNDecoder(cfg.cnn_keys.decoder, [int(np.prod(obs_space[k].shape[:-2])) for k in cfg.cnn_keys.decoder],
                              wm.observation_model.cnn_channels_multiplier, latent_state_size, cnn_encoder.output_dim,
                              obs_space[cfg.cnn_keys.decoder[0]].shape[-2:], _act(wm.observation_model.cnn_act), False)
                   if cfg.cnn_keys.decoder else None)
    mlp_decoder = (MLPDecoder(cfg.mlp_keys.decoder, [obs_space[k].shape[0] for k in cfg.mlp_keys.decoder],
                              latent_state_size, wm.observation_model.mlp_layers, wm.observation_model.dense_units,
                              _act(wm.observation_model.dense_act), False) if cfg.mlp_keys.decoder else None)
    observation_model = MultiDecoder(cnn_decoder, mlp_decoder)
    reward_model = MLP(input_dims=latent_state_size, output_dim=1,
                       hidden_sizes=[wm.reward_model.dense_units] * wm.reward_model.mlp_layers,
                       activation=_act(wm.reward_model.dense_act), flatten_dim=None)
    continue_model = None
    if wm.use_continues:
        continue_model = MLP(input_dims=latent_state_size, output_dim=1,
                             hidden_sizes=[wm.discount_model.dense_units] * wm.discount_model.mlp_layers,
                             activation=_act(wm.discount_model.dense_act), flatten_dim=None)
    world_model = WorldModel(encoder.apply(init_weights), rssm, observation_model.apply(init_weights),
                             reward_model.apply(init_weights),
                             continue_model.apply(init_weights) if continue_model is not None else None)
    ac = cfg.algo.actor
    actor = get_class(ac.cls)(latent_state_size=latent_state_size, actions_dim=actions_dim, is_continuous=is_continuous,
                              init_std=ac.init_std, min_std=ac.min_std, mlp_layers=ac.mlp_layers,
                              dense_units=ac.dense_units, activation=_act(ac.dense_act),
                              distribution_cfg=cfg.distribution, layer_norm=False)
    cc = cfg.algo.critic
    critic = MLP(input_dims=latent_state_size, output_dim=1, hidden_sizes=[cc.dense_units] * cc.mlp_layers,
                 activation=_act(cc.dense_act), flatten_dim=None)
    actor.apply(init_weights)
    critic.apply(init_weights)
    if world_model_state:
        world_model.load_state_dict(world_model_state)
    if actor_state:
        actor.load_state_dict(actor_state)
    if critic_state:
        critic.load_state_dict(critic_state)
    return runner.setup_module(world_model), runner.setup_module(actor), runner.setup_module(critic)
