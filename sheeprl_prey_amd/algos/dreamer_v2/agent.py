"""DreamerV2 agent (reference: ``sheeprl/algos/dreamer_v2/agent.py:28-1024``).

* encoder: 4 x Conv(k4, s2, no padding) with [1,2,4,8]*mult channels, ELU (optional channel LN);
  MLP encoder; decoder: Linear -> 1x1 -> 4 x ConvT(k5,5,6,6 s2) to the image; MLP decoder.
* RSSM: recurrent model = MLP(ELU) -> LayerNorm-GRU (fused ``ln_gru`` kernel); representation /
  transition MLPs -> 32x32 categorical logits; straight-through one-hot sampling runs through the
  fused ``unimix_sample`` kernel with mixing 0 (plain categorical).
* actor: the shared Dreamer actor (trunc_normal / tanh_normal / normal / discrete ST heads).
"""
from __future__ import annotations

import copy
from typing import Any, Dict, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn as nn
from torch import Tensor
from torch.distributions import Normal

from sheeprl_prey_amd import ops
from sheeprl_prey_amd.algos.dreamer_v3.agent import Actor as _DreamerActor
from sheeprl_prey_amd.algos.dreamer_v3.agent import MinedojoActor as _DreamerMinedojoActor
from sheeprl_prey_amd.config.instantiate import get_class
from sheeprl_prey_amd.models.models import CNN, MLP, DeCNN, LayerNormGRUCell, MultiDecoder, MultiEncoder
from sheeprl_prey_amd.models.world_model import WorldModel
from sheeprl_prey_amd.utils.distribution import OneHotCategoricalValidateArgs
from sheeprl_prey_amd.utils.model import LayerNormChannelLast, ModuleType, cnn_forward


def _act(name):
    return get_class(name) if isinstance(name, str) else name


def init_weights(m: nn.Module, mode: str = "normal") -> None:
    """Xavier init, zero bias (reference ``dreamer_v2/utils.py:44-66``)."""
    if isinstance(m, (nn.Conv2d, nn.ConvTranspose2d, nn.Linear)):
        if mode == "normal":
            nn.init.xavier_normal_(m.weight.data)
        elif mode == "uniform":
            nn.init.xavier_uniform_(m.weight.data)
        elif mode == "zero":
            nn.init.constant_(m.weight.data, 0)
        else:
            raise RuntimeError(f"Unrecognized initialization: {mode}. Choose between: `normal`, `uniform` and `zero`")
        if m.bias is not None:
            nn.init.constant_(m.bias.data, 0)


def compute_stochastic_state(logits: Tensor, discrete: int = 32, sample: bool = True, validate_args: bool = False) -> Tensor:
    """One-hot straight-through sample (or mode) of ``logits[..., S*discrete]`` -> ``[..., S, discrete]``."""
    _, st = ops.unimix_sample(logits, discrete, 0.0, sample=sample)
    return st.view(*logits.shape[:-1], -1, discrete)


def _mlp(input_dim, output_dim, hidden, layers, act, layer_norm, bias=True):
    return MLP(input_dims=input_dim, output_dim=output_dim, hidden_sizes=[hidden] * layers, activation=act,
               flatten_dim=None, layer_args={"bias": bias},
               norm_layer=[nn.LayerNorm for _ in range(layers)] if layer_norm else None,
               norm_args=[{"normalized_shape": hidden} for _ in range(layers)] if layer_norm else None)


class CNNEncoder(nn.Module):
    def __init__(self, keys: Sequence[str], input_channels: Sequence[int], image_size: Tuple[int, int],
                 channels_multiplier: int, layer_norm: bool = False, activation: ModuleType = nn.ELU) -> None:
        super().__init__()
        self.keys = keys
        self.input_dim = (sum(input_channels), *image_size)
        self.model = nn.Sequential(
            CNN(input_channels=sum(input_channels), hidden_channels=[m * channels_multiplier for m in (1, 2, 4, 8)],
                layer_args={"kernel_size": 4, "stride": 2}, activation=activation,
                norm_layer=[LayerNormChannelLast for _ in range(4)] if layer_norm else None,
                norm_args=[{"normalized_shape": (2**i) * channels_multiplier} for i in range(4)] if layer_norm else None),
            nn.Flatten(-3, -1),
        )
        with torch.no_grad():
            self.output_dim = self.model(torch.zeros(1, *self.input_dim)).shape[-1]

    def forward(self, obs: Dict[str, Tensor]) -> Tensor:
        x = torch.cat([obs[k] for k in self.keys], -3)
        return cnn_forward(self.model, x, x.shape[-3:], (-1,))


class MLPEncoder(nn.Module):
    def __init__(self, keys: Sequence[str], input_dims: Sequence[int], mlp_layers: int = 4, dense_units: int = 512,
                 layer_norm: bool = False, activation: ModuleType = nn.ELU) -> None:
        super().__init__()
        self.keys = keys
        self.input_dim = sum(input_dims)
        self.model = MLP(self.input_dim, None, [dense_units] * mlp_layers, activation=activation,
                         norm_layer=[nn.LayerNorm for _ in range(mlp_layers)] if layer_norm else None,
                         norm_args=[{"normalized_shape": dense_units} for _ in range(mlp_layers)] if layer_norm else None)
        self.output_dim = dense_units

    def forward(self, obs: Dict[str, Tensor]) -> Tensor:
        return self.model(torch.cat([obs[k] for k in self.keys], -1).float())


class CNNDecoder(nn.Module):
    def __init__(self, keys: Sequence[str], output_channels: Sequence[int], channels_multiplier: int,
                 latent_state_size: int, cnn_encoder_output_dim: int, image_size: Tuple[int, int],
                 activation: ModuleType = nn.ELU, layer_norm: bool = False) -> None:
        super().__init__()
        self.keys = keys
        self.output_channels = list(output_channels)
        self.cnn_encoder_output_dim = cnn_encoder_output_dim
        self.image_size = image_size
        self.output_dim = (sum(output_channels), *image_size)
        self.model = nn.Sequential(
            nn.Linear(latent_state_size, cnn_encoder_output_dim),
            nn.Unflatten(1, (cnn_encoder_output_dim, 1, 1)),
            DeCNN(input_channels=cnn_encoder_output_dim,
                  hidden_channels=[m * channels_multiplier for m in (4, 2, 1)] + [self.output_dim[0]],
                  layer_args=[{"kernel_size": 5, "stride": 2}, {"kernel_size": 5, "stride": 2},
                              {"kernel_size": 6, "stride": 2}, {"kernel_size": 6, "stride": 2}],
                  activation=[activation, activation, activation, None],
                  norm_layer=[LayerNormChannelLast for _ in range(3)] + [None] if layer_norm else None,
                  norm_args=[{"normalized_shape": m * channels_multiplier} for m in (4, 2, 1)] + [None]
                  if layer_norm else None),
        )

    def forward(self, latent_states: Tensor) -> Dict[str, Tensor]:
        x = cnn_forward(self.model, latent_states, (latent_states.shape[-1],), self.output_dim)
        return {k: r for k, r in zip(self.keys, torch.split(x, self.output_channels, -3))}


class MLPDecoder(nn.Module):
    def __init__(self, keys: Sequence[str], output_dims: Sequence[int], latent_state_size: int, mlp_layers: int = 4,
                 dense_units: int = 512, activation: ModuleType = nn.ELU, layer_norm: bool = False) -> None:
        super().__init__()
        self.output_dims = list(output_dims)
        self.keys = keys
        self.model = MLP(latent_state_size, None, [dense_units] * mlp_layers, activation=activation,
                         norm_layer=[nn.LayerNorm for _ in range(mlp_layers)] if layer_norm else None,
                         norm_args=[{"normalized_shape": dense_units} for _ in range(mlp_layers)] if layer_norm else None)
        self.heads = nn.ModuleList([nn.Linear(dense_units, d) for d in self.output_dims])

    def forward(self, latent_states: Tensor) -> Dict[str, Tensor]:
        x = self.model(latent_states)
        return {k: h(x) for k, h in zip(self.keys, self.heads)}


class RecurrentModel(nn.Module):
    """MLP(ELU) -> LayerNorm GRU (reference ``dreamer_v2/agent.py:230-271``)."""

    def __init__(self, input_size: int, recurrent_state_size: int, dense_units: int, activation: ModuleType = nn.ELU,
                 layer_norm: bool = False) -> None:
        super().__init__()
        self.mlp = MLP(input_dims=input_size, output_dim=None, hidden_sizes=[dense_units], activation=activation,
                       norm_layer=[nn.LayerNorm] if layer_norm else None,
                       norm_args=[{"normalized_shape": dense_units}] if layer_norm else None)
        self.rnn = LayerNormGRUCell(dense_units, recurrent_state_size, bias=True, batch_first=False, layer_norm=True)

    def forward(self, input: Tensor, recurrent_state: Tensor) -> Tensor:
        return self.rnn(self.mlp(input), recurrent_state)


class RSSM(nn.Module):
    """Reference ``dreamer_v2/agent.py:274-380``."""

    def __init__(self, recurrent_model: nn.Module, representation_model: nn.Module, transition_model: nn.Module,
                 distribution_cfg: Dict[str, Any], discrete: int = 32) -> None:
        super().__init__()
        self.recurrent_model = recurrent_model
        self.representation_model = representation_model
        self.transition_model = transition_model
        self.discrete = discrete
        self.distribution_cfg = distribution_cfg

    def dynamic(self, posterior: Tensor, recurrent_state: Tensor, action: Tensor, embedded_obs: Tensor,
                is_first: Tensor):
        action = (1 - is_first) * action
        posterior = (1 - is_first) * posterior.view(*posterior.shape[:-2], -1)
        recurrent_state = (1 - is_first) * recurrent_state
        recurrent_state = self.recurrent_model(torch.cat((posterior, action), -1), recurrent_state)
        prior_logits, prior = self._transition(recurrent_state)
        posterior_logits, posterior = self._representation(recurrent_state, embedded_obs)
        return recurrent_state, posterior, prior, posterior_logits, prior_logits

    def _representation(self, recurrent_state: Tensor, embedded_obs: Tensor) -> Tuple[Tensor, Tensor]:
        logits = self.representation_model(torch.cat((recurrent_state, embedded_obs), -1))
        return logits, compute_stochastic_state(logits, self.discrete)

    def _transition(self, recurrent_out: Tensor) -> Tuple[Tensor, Tensor]:
        logits = self.transition_model(recurrent_out)
        return logits, compute_stochastic_state(logits, self.discrete)

    def imagination(self, prior: Tensor, recurrent_state: Tensor, actions: Tensor) -> Tuple[Tensor, Tensor]:
        recurrent_state = self.recurrent_model(torch.cat((prior, actions), -1), recurrent_state)
        _, imagined_prior = self._transition(recurrent_state)
        return imagined_prior, recurrent_state


class Actor(_DreamerActor):
    """DreamerV2 actor: biased MLP layers (LN eps 1e-5 when enabled), no unimix (reference
    ``dreamer_v2/agent.py:383-510``)."""

    def __init__(self, latent_state_size: int, actions_dim: Sequence[int], is_continuous: bool,
                 distribution_cfg: Dict[str, Any], init_std: float = 0.0, min_std: float = 0.1, dense_units: int = 400,
                 activation: ModuleType = nn.ELU, mlp_layers: int = 4, layer_norm: bool = False) -> None:
        super().__init__(latent_state_size, actions_dim, is_continuous, distribution_cfg, init_std, min_std, dense_units,
                         activation, mlp_layers, layer_norm, unimix=0.0, ln_eps=1e-5, bias=True)


class MinedojoActor(_DreamerMinedojoActor):
    def __init__(self, latent_state_size: int, actions_dim: Sequence[int], is_continuous: bool,
                 distribution_cfg: Dict[str, Any], init_std: float = 0.0, min_std: float = 0.1, dense_units: int = 400,
                 activation: ModuleType = nn.ELU, mlp_layers: int = 4, layer_norm: bool = False) -> None:
        super().__init__(latent_state_size, actions_dim, is_continuous, distribution_cfg, init_std, min_std, dense_units,
                         activation, mlp_layers, layer_norm, unimix=0.0, ln_eps=1e-5, bias=True)


class PlayerDV2(nn.Module):
    """Env-interaction wrapper (reference ``dreamer_v2/agent.py:658-800``)."""

    def __init__(self, encoder: nn.Module, recurrent_model: nn.Module, representation_model: nn.Module,
                 actor: nn.Module, actions_dim: Sequence[int], expl_amount: float, num_envs: int, stochastic_size: int,
                 recurrent_state_size: int, device, discrete_size: int = 32) -> None:
        super().__init__()
        self.encoder = encoder
        self.recurrent_model = recurrent_model
        self.representation_model = representation_model
        self.actor = actor
        self.device = device
        self.expl_amount = expl_amount
        self.actions_dim = actions_dim
        self.stochastic_size = stochastic_size
        self.discrete_size = discrete_size
        self.recurrent_state_size = recurrent_state_size
        self.num_envs = num_envs
        self.validate_args = self.actor.distribution_cfg.get("validate_args", False)

    def init_states(self, reset_envs: Optional[Sequence[int]] = None) -> None:
        if reset_envs is None or len(reset_envs) == 0:
            self.actions = torch.zeros(1, self.num_envs, int(np.sum(self.actions_dim)), device=self.device)
            self.recurrent_state = torch.zeros(1, self.num_envs, self.recurrent_state_size, device=self.device)
            self.stochastic_state = torch.zeros(1, self.num_envs, self.stochastic_size * self.discrete_size,
                                                device=self.device)
        else:
            self.actions[:, reset_envs] = 0
            self.recurrent_state[:, reset_envs] = 0
            self.stochastic_state[:, reset_envs] = 0

    def _stoch(self, logits: Tensor) -> Tensor:
        return compute_stochastic_state(logits, self.discrete_size).view(*logits.shape[:-1], -1)

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
        self.recurrent_state = self.recurrent_model(torch.cat((self.stochastic_state, self.actions), -1),
                                                    self.recurrent_state)
        posterior_logits = self.representation_model(torch.cat((self.recurrent_state, embedded_obs), -1))
        self.stochastic_state = self._stoch(posterior_logits)
        actions, _ = self.actor(torch.cat((self.stochastic_state, self.recurrent_state), -1), is_training, mask)
        self.actions = torch.cat(actions, -1)
        return actions


def build_models(runner, actions_dim: Sequence[int], is_continuous: bool, cfg: Dict[str, Any], obs_space,
                 world_model_state: Optional[Dict[str, Tensor]] = None, actor_state: Optional[Dict[str, Tensor]] = None,
                 critic_state: Optional[Dict[str, Tensor]] = None,
                 target_critic_state: Optional[Dict[str, Tensor]] = None):
    """Reference ``dreamer_v2/agent.py:803-1024``."""
    wm = cfg.algo.world_model
    stochastic_size = wm.stochastic_size * wm.discrete_size
    latent_state_size = stochastic_size + wm.recurrent_model.recurrent_state_size
    cnn_encoder = (CNNEncoder(cfg.cnn_keys.encoder, [int(np.prod(obs_space[k].shape[:-2])) for k in cfg.cnn_keys.encoder],
                              obs_space[cfg.cnn_keys.encoder[0]].shape[-2:], wm.encoder.cnn_channels_multiplier,
                              wm.encoder.layer_norm, _act(wm.encoder.cnn_act)) if cfg.cnn_keys.encoder else None)
    mlp_encoder = (MLPEncoder(cfg.mlp_keys.encoder, [obs_space[k].shape[0] for k in cfg.mlp_keys.encoder],
                              wm.encoder.mlp_layers, wm.encoder.dense_units, wm.encoder.layer_norm,
                              _act(wm.encoder.dense_act)) if cfg.mlp_keys.encoder else None)
    encoder = MultiEncoder(cnn_encoder, mlp_encoder)
    rm = dict(wm.recurrent_model)
    recurrent_model = RecurrentModel(input_size=int(sum(actions_dim) + stochastic_size),
                                     recurrent_state_size=rm["recurrent_state_size"], dense_units=rm["dense_units"],
                                     activation=_act(rm.get("dense_act", "torch.nn.ELU")),
                                     layer_norm=rm.get("layer_norm", False))
    representation_model = _mlp(wm.recurrent_model.recurrent_state_size + encoder.output_dim, stochastic_size,
                                wm.representation_model.hidden_size, 1, _act(wm.representation_model.dense_act),
                                wm.representation_model.layer_norm)
    transition_model = _mlp(wm.recurrent_model.recurrent_state_size, stochastic_size, wm.transition_model.hidden_size,
                            1, _act(wm.transition_model.dense_act), wm.transition_model.layer_norm)
    rssm = RSSM(recurrent_model.apply(init_weights), representation_model.apply(init_weights),
                transition_model.apply(init_weights), cfg.distribution, discrete=wm.discrete_size)
    cnn_decoder = (CNNDecoder(cfg.cnn_keys.decoder, [int(np.prod(obs_space[k].shape[:-2])) for k in cfg.cnn_keys.decoder],
                              wm.observation_model.cnn_channels_multiplier, latent_state_size, cnn_encoder.output_dim,
                              obs_space[cfg.cnn_keys.decoder[0]].shape[-2:], _act(wm.observation_model.cnn_act),
                              wm.observation_model.layer_norm) if cfg.cnn_keys.decoder else None)
    mlp_decoder = (MLPDecoder(cfg.mlp_keys.decoder, [obs_space[k].shape[0] for k in cfg.mlp_keys.decoder],
                              latent_state_size, wm.observation_model.mlp_layers, wm.observation_model.dense_units,
                              _act(wm.observation_model.dense_act), wm.observation_model.layer_norm)
                   if cfg.mlp_keys.decoder else None)
    observation_model = MultiDecoder(cnn_decoder, mlp_decoder)
    reward_model = _mlp(latent_state_size, 1, wm.reward_model.dense_units, wm.reward_model.mlp_layers,
                        _act(wm.reward_model.dense_act), wm.reward_model.layer_norm)
    continue_model = None
    if wm.use_continues:
        continue_model = _mlp(latent_state_size, 1, wm.discount_model.dense_units, wm.discount_model.mlp_layers,
                              _act(wm.discount_model.dense_act), wm.discount_model.layer_norm)
    world_model = WorldModel(encoder.apply(init_weights), rssm, observation_model.apply(init_weights),
                             reward_model.apply(init_weights),
                             continue_model.apply(init_weights) if continue_model is not None else None)
    ac = cfg.algo.actor
    actor_cls = get_class(ac.cls)
    actor = actor_cls(latent_state_size=latent_state_size, actions_dim=actions_dim, is_continuous=is_continuous,
                      init_std=ac.init_std, min_std=ac.min_std, mlp_layers=ac.mlp_layers, dense_units=ac.dense_units,
                      activation=_act(ac.dense_act), distribution_cfg=cfg.distribution, layer_norm=ac.layer_norm)
    cc = cfg.algo.critic
    critic = _mlp(latent_state_size, 1, cc.dense_units, cc.mlp_layers, _act(cc.dense_act), cc.layer_norm)
    actor.apply(init_weights)
    critic.apply(init_weights)
    if world_model_state:
        world_model.load_state_dict(world_model_state)
    if actor_state:
        actor.load_state_dict(actor_state)
    if critic_state:
        critic.load_state_dict(critic_state)
    world_model = runner.setup_module(world_model)
    actor = runner.setup_module(actor)
    critic = runner.setup_module(critic)
    target_critic = copy.deepcopy(critic)
    for p in target_critic.parameters():
        p.requires_grad = False
    if target_critic_state:
        target_critic.load_state_dict(target_critic_state)
    return world_model, actor, critic, target_critic
