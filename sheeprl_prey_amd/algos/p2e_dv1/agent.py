"""Plan2Explore-DV1 models (reference: ``sheeprl/algos/p2e_dv1/agent.py:20-113``): the DreamerV1
world model + task actor/critic, plus an exploration actor/critic."""
from __future__ import annotations

from typing import Any, Dict, Sequence

from torch import nn

from sheeprl_prey_amd.algos.dreamer_v1.agent import Actor, MinedojoActor  # noqa: F401
from sheeprl_prey_amd.algos.dreamer_v1.agent import build_models as dv1_build_models
from sheeprl_prey_amd.algos.dreamer_v2.agent import _act
from sheeprl_prey_amd.config.instantiate import get_class
from sheeprl_prey_amd.models.models import MLP
from sheeprl_prey_amd.utils.utils import init_weights


def build_models(runner, actions_dim: Sequence[int], is_continuous: bool, cfg: Dict[str, Any], obs_space,
                 world_model_state=None, actor_task_state=None, critic_task_state=None, actor_exploration_state=None,
                 critic_exploration_state=None):
    wm = cfg.algo.world_model
    latent = wm.stochastic_size + wm.recurrent_model.recurrent_state_size
    world_model, actor_task, critic_task = dv1_build_models(runner, actions_dim, is_continuous, cfg, obs_space,
                                                            world_model_state, actor_task_state, critic_task_state)
    ac, cc = cfg.algo.actor, cfg.algo.critic
    actor_expl = get_class(ac.cls)(latent_state_size=latent, actions_dim=actions_dim, is_continuous=is_continuous,
                                   init_std=ac.init_std, min_std=ac.min_std, mlp_layers=ac.mlp_layers,
                                   dense_units=ac.dense_units, activation=_act(ac.dense_act),
                                   distribution_cfg=cfg.distribution, layer_norm=False)
    critic_expl = MLP(input_dims=latent, output_dim=1, hidden_sizes=[cc.dense_units] * cc.mlp_layers,
                      activation=_act(cc.dense_act), flatten_dim=None)
    actor_expl.apply(init_weights)
    critic_expl.apply(init_weights)
    if actor_exploration_state:
        actor_expl.load_state_dict(actor_exploration_state)
    if critic_exploration_state:
        critic_expl.load_state_dict(critic_exploration_state)
    return world_model, actor_task, critic_task, runner.setup_module(actor_expl), runner.setup_module(critic_expl)
