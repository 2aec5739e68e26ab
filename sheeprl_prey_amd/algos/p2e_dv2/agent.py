"""Plan2Explore-DV2 models (reference: ``sheeprl/algos/p2e_dv2/agent.py:21-142``): the DreamerV2
world model + exploration actor/critic, plus a task actor/critic (Kaiming init)."""
from __future__ import annotations

import copy
from typing import Any, Dict, Optional, Sequence

from torch import nn

from sheeprl_prey_amd.algos.dreamer_v2.agent import Actor, MinedojoActor, _act, _mlp  # noqa: F401
from sheeprl_prey_amd.algos.dreamer_v2.agent import build_models as dv2_build_models
from sheeprl_prey_amd.config.instantiate import get_class
from sheeprl_prey_amd.utils.utils import init_weights


def build_models(runner, actions_dim: Sequence[int], is_continuous: bool, cfg: Dict[str, Any], obs_space,
                 world_model_state=None, actor_task_state=None, critic_task_state=None, target_critic_task_state=None,
                 actor_exploration_state=None, critic_exploration_state=None, target_critic_exploration_state=None):
    wm = cfg.algo.world_model
    latent = wm.stochastic_size * wm.discrete_size + wm.recurrent_model.recurrent_state_size
    world_model, actor_expl, critic_expl, target_critic_expl = dv2_build_models(
        runner, actions_dim, is_continuous, cfg, obs_space, world_model_state, actor_exploration_state,
        critic_exploration_state, target_critic_exploration_state)
    ac, cc = cfg.algo.actor, cfg.algo.critic
    actor_task = get_class(ac.cls)(latent_state_size=latent, actions_dim=actions_dim, is_continuous=is_continuous,
                                   init_std=ac.init_std, min_std=ac.min_std, mlp_layers=ac.mlp_layers,
                                   dense_units=ac.dense_units, activation=_act(ac.dense_act),
                                   distribution_cfg=cfg.distribution, layer_norm=ac.layer_norm)
    critic_task = _mlp(latent, 1, cc.dense_units, cc.mlp_layers, _act(cc.dense_act), cc.layer_norm)
    actor_task.apply(init_weights)
    critic_task.apply(init_weights)
    if actor_task_state:
        actor_task.load_state_dict(actor_task_state)
    if critic_task_state:
        critic_task.load_state_dict(critic_task_state)
    actor_task = runner.setup_module(actor_task)
    critic_task = runner.setup_module(critic_task)
    target_critic_task = copy.deepcopy(critic_task)
    for p in target_critic_task.parameters():
        p.requires_grad = False
    if target_critic_task_state:
        target_critic_task.load_state_dict(target_critic_task_state)
    return world_model, actor_task, critic_task, target_critic_task, actor_expl, critic_expl, target_critic_expl
