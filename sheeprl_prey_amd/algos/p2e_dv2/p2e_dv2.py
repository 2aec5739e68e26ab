"""Plan2Explore with DreamerV2 (reference: ``sheeprl/algos/p2e_dv2/p2e_dv2.py:36-1081``).
The exploration / task phases live in ``algos/p2e_common.py``; the loop is ``algos/dreamer_loop.py``."""
from __future__ import annotations

import copy
from typing import Any, Dict

from sheeprl_prey_amd.algos.common import action_info, build_envs, check_obs_keys, load_resume, setup_logger
from sheeprl_prey_amd.algos.dreamer_loop import DreamerSpec, build_replay, restore_rb, run_dreamer_loop
from sheeprl_prey_amd.algos.dreamer_v2.agent import PlayerDV2
from sheeprl_prey_amd.algos.dreamer_v2.dreamer_v2 import DreamerV2Trainer, check_keys
from sheeprl_prey_amd.algos.dreamer_v2.utils import test
from sheeprl_prey_amd.algos.p2e_common import P2E_METRICS, P2EMixin, build_ensembles
from sheeprl_prey_amd.algos.p2e_dv2.agent import build_models
from sheeprl_prey_amd.parallel.flat_optim import build_optimizer
from sheeprl_prey_amd.utils.metric import MeanMetric, MetricAggregator
from sheeprl_prey_amd.utils.registry import register_algorithm


class P2EDV2Trainer(P2EMixin, DreamerV2Trainer):
    pass


@register_algorithm()
def main(runner, cfg: Dict[str, Any]):
    cfg, state = load_resume(runner, cfg)
    device = runner.device
    rank, world_size = runner.global_rank, runner.world_size
    runner.seed_everything(cfg.seed + rank)
    cfg.env.screen_size = 64
    cfg.env.frame_stack = 1

    logger, log_dir = setup_logger(runner, cfg)
    envs = build_envs(runner, cfg, log_dir)
    obs_space = envs.single_observation_space
    is_continuous, _, actions_dim = action_info(envs.single_action_space)
    check_obs_keys(cfg, obs_space)
    check_keys(cfg)
    g = (lambda k: state[k] if state else None)
    (world_model, actor_task, critic_task, target_critic_task, actor_expl, critic_expl,
     target_critic_expl) = build_models(runner, actions_dim, is_continuous, cfg, obs_space, g("world_model"),
                                        g("actor_task"), g("critic_task"), g("target_critic_task"),
                                        g("actor_exploration"), g("critic_exploration"), g("target_critic_exploration"))
    wm = cfg.algo.world_model
    stoch = wm.stochastic_size * wm.discrete_size
    ensembles = build_ensembles(cfg, int(sum(actions_dim)) + wm.recurrent_model.recurrent_state_size + stoch, stoch,
                                device)
    if state:
        ensembles.load_state_dict(state["ensembles"])
    runner.setup_module(ensembles)
    player = PlayerDV2(world_model.encoder, world_model.rssm.recurrent_model, world_model.rssm.representation_model,
                       actor_expl, actions_dim, cfg.algo.player.expl_amount, cfg.env.num_envs, wm.stochastic_size,
                       wm.recurrent_model.recurrent_state_size, device, discrete_size=wm.discrete_size)

    world_optimizer = build_optimizer(cfg.algo.world_model.optimizer, world_model.parameters())
    actor_expl_optimizer = build_optimizer(cfg.algo.actor.optimizer, actor_expl.parameters())
    critic_expl_optimizer = build_optimizer(cfg.algo.critic.optimizer, critic_expl.parameters())
    actor_task_optimizer = build_optimizer(cfg.algo.actor.optimizer, actor_task.parameters())
    critic_task_optimizer = build_optimizer(cfg.algo.critic.optimizer, critic_task.parameters())
    ensemble_optimizer = build_optimizer(cfg.algo.critic.optimizer, ensembles.parameters())
    opts = {"world_optimizer": world_optimizer, "actor_task_optimizer": actor_task_optimizer,
            "critic_task_optimizer": critic_task_optimizer, "ensemble_optimizer": ensemble_optimizer,
            "actor_exploration_optimizer": actor_expl_optimizer, "critic_exploration_optimizer": critic_expl_optimizer}
    if state:
        for k, o in opts.items():
            o.load_state_dict(state[k])
    trainer = P2EDV2Trainer(runner, cfg, world_model, actor_task, critic_task, target_critic_task, world_optimizer,
                            actor_task_optimizer, critic_task_optimizer, is_continuous, actions_dim)
    trainer.setup_p2e("dv2", actor_expl, critic_expl, target_critic_expl, ensembles, ensemble_optimizer,
                      actor_expl_optimizer, critic_expl_optimizer)
    aggregator = MetricAggregator({n: MeanMetric(sync_on_compute=cfg.metric.sync_on_compute) for n in P2E_METRICS})
    buffer_size = cfg.buffer.size // int(cfg.env.num_envs * world_size) if not cfg.dry_run else 4
    rb, btype = build_replay(cfg, runner, log_dir, buffer_size)
    if state and cfg.buffer.checkpoint:
        restore_rb(rb, state, runner)

    policy_steps_per_update = int(cfg.env.num_envs * world_size)
    num_updates = cfg.total_steps // policy_steps_per_update if not cfg.dry_run else 1
    exploration_updates = min(num_updates, int(cfg.exploration_steps // policy_steps_per_update)
                              if not cfg.dry_run else 4)

    def before_update(update: int) -> None:
        if update == exploration_updates:
            trainer.is_exploring = False
            player.actor = actor_task
            if runner.is_global_zero:
                test(copy.deepcopy(player), runner, cfg, log_dir, "zero-shot")

    def final_test():
        player.actor = actor_task
        test(player, runner, cfg, log_dir, "few-shot")

    spec = DreamerSpec(
        variant="dv2", player=player, train_step=trainer.train_step, update_target=trainer.update_targets,
        target_every=cfg.algo.critic.target_network_update_freq, before_update=before_update,
        checkpoint_state=lambda: {
            "world_model": world_model.state_dict(), "actor_task": actor_task.state_dict(),
            "critic_task": critic_task.state_dict(), "target_critic_task": target_critic_task.state_dict(),
            "ensembles": ensembles.state_dict(), "actor_exploration": actor_expl.state_dict(),
            "critic_exploration": critic_expl.state_dict(),
            "target_critic_exploration": target_critic_expl.state_dict(),
            **{k: o.state_dict() for k, o in opts.items()}},
        test=final_test, actor_cls_name=cfg.algo.actor.cls)
    run_dreamer_loop(runner, cfg, state, envs, spec, aggregator, rb, btype, actions_dim, is_continuous, log_dir,
                     expl_decay_steps=state["expl_decay_steps"] if state else 0)
