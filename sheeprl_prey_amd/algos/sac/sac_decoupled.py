"""SAC, decoupled actor-learner (reference: ``sheeprl/algos/sac/sac_decoupled.py:36-542``).

rank 0 (player): envs + replay buffer + actor; after ``learning_starts`` it samples
``G*B*(N-1)`` transitions per env step and sends one chunk to each trainer (packed P2P, see
``parallel/decoupled.py``), then receives the new actor weights from trainer rank 1.
ranks 1..N-1 (trainers): the captured ``SACTrainer`` updates with gradients averaged over the
optimisation group; trainer 1 returns actor weights, metrics and checkpoint state to the player.
"""
from __future__ import annotations

import os
from typing import Any, Dict

import numpy as np
import torch

from sheeprl_prey_amd.algos.common import build_envs, episode_stats, load_resume, restore_replay_buffer, setup_logger
from sheeprl_prey_amd.algos.sac.agent import SACActor, build_agent
from sheeprl_prey_amd.algos.sac.sac import SACTrainer, check_sac_spaces, real_next_obs
from sheeprl_prey_amd.algos.sac.utils import obs_to_tensor, test
from sheeprl_prey_amd.data.buffers import ReplayBuffer
from sheeprl_prey_amd.data.tensordict import TensorDict
from sheeprl_prey_amd.parallel.decoupled import DecoupledComm, params_to_vector, vector_to_params
from sheeprl_prey_amd.parallel.flat_optim import build_optimizer
from sheeprl_prey_amd.utils.metric import MeanMetric, MetricAggregator
from sheeprl_prey_amd.utils.registry import register_algorithm
from sheeprl_prey_amd.utils.timer import timer

_KEYS = ("observations", "next_observations", "actions", "rewards", "dones")


def player(runner, cfg: Dict[str, Any], comm: DecoupledComm, log_dir: str):
    device = runner.device
    envs = build_envs(runner, cfg, log_dir)
    check_sac_spaces(cfg, envs)
    action_space = envs.single_action_space
    obs_space = envs.single_observation_space
    obs_dim = int(sum(int(np.prod(obs_space[k].shape)) for k in cfg.mlp_keys.encoder))
    act_dim = int(np.prod(action_space.shape))
    actor = SACActor(obs_dim, act_dim, cfg.distribution, cfg.algo.actor.hidden_size, action_space.low,
                     action_space.high).to(device)
    actor_params = list(actor.parameters())
    flat = torch.empty_like(params_to_vector(actor_params))
    comm.broadcast_params(flat)
    vector_to_params(flat, actor_params)

    aggregator = MetricAggregator({k: MeanMetric() for k in ("Rewards/rew_avg", "Game/ep_len_avg")})
    buffer_size = cfg.buffer.size // cfg.env.num_envs if not cfg.dry_run else 1
    rb = ReplayBuffer(buffer_size, cfg.env.num_envs, device=device if device.type == "cuda" else "cpu",
                      memmap=cfg.buffer.memmap and device.type == "cpu",
                      memmap_dir=os.path.join(log_dir, "memmap_buffer", "rank_0"))
    state = cfg.pop("_resume_state", None)
    if state is not None and cfg.buffer.checkpoint and "rb" in state:
        restore_replay_buffer(rb, state["rb"], _OneRank())
    step_data = TensorDict({}, batch_size=[cfg.env.num_envs], device=rb.device)

    start_step = state["update"] if state else 1
    policy_step = (state["update"] - 1) * cfg.env.num_envs if state else 0
    last_log = state["last_log"] if state else 0
    last_checkpoint = state["last_checkpoint"] if state else 0
    policy_steps_per_update = int(cfg.env.num_envs)
    num_updates = int(cfg.total_steps // policy_steps_per_update) if not cfg.dry_run else 1
    learning_starts = cfg.algo.learning_starts // policy_steps_per_update if not cfg.dry_run else 0
    if state and not cfg.buffer.checkpoint:
        learning_starts += start_step
    n_tr = comm.world_size - 1
    first_info_sent = False

    o = envs.reset(seed=cfg.seed)[0]
    obs = obs_to_tensor(o, cfg.mlp_keys.encoder, rb.device, cfg.env.num_envs)
    for update in range(start_step, num_updates + 1):
        policy_step += cfg.env.num_envs
        with timer("Time/env_interaction_time"):
            if update <= learning_starts:
                actions = envs.action_space.sample()
            else:
                with torch.no_grad():
                    actions = actor(obs.to(device))[0].cpu().numpy()
            next_o, rewards, dones, truncated, infos = envs.step(actions.reshape(envs.action_space.shape))
            dones = np.logical_or(dones, truncated)
        for i, ep_rew, ep_len in episode_stats(infos):
            aggregator.update("Rewards/rew_avg", ep_rew)
            aggregator.update("Game/ep_len_avg", ep_len)
            runner.print(f"Rank-0: policy_step={policy_step}, reward_env_{i}={ep_rew[-1]}")

        next_obs = obs_to_tensor(next_o, cfg.mlp_keys.encoder, rb.device, cfg.env.num_envs)
        n = cfg.env.num_envs
        step_data["dones"] = torch.as_tensor(dones, dtype=torch.float32).view(n, -1).to(rb.device)
        step_data["actions"] = torch.as_tensor(actions, dtype=torch.float32).view(n, -1).to(rb.device)
        step_data["observations"] = obs
        if not cfg.buffer.sample_next_obs:
            step_data["next_observations"] = obs_to_tensor(real_next_obs(next_o, infos), cfg.mlp_keys.encoder,
                                                           rb.device, n)
        step_data["rewards"] = torch.as_tensor(rewards, dtype=torch.float32).view(n, -1).to(rb.device)
        rb.add(step_data.unsqueeze(0))
        obs = next_obs

        if update >= learning_starts:
            if not first_info_sent:
                comm.broadcast_object_world({"update": update, "last_log": last_log, "last_checkpoint": last_checkpoint})
                first_info_sent = True
            training_steps = learning_starts if update == learning_starts else 1
            per = max(training_steps, 1) * cfg.algo.per_rank_gradient_steps * cfg.per_rank_batch_size
            sample = rb.sample(per * n_tr, sample_next_obs=cfg.buffer.sample_next_obs)
            chunks = [{k: sample[k][i * per : (i + 1) * per].reshape(per, *sample[k].shape[2:]) for k in _KEYS}
                      for i in range(n_tr)]
            comm.send_chunks(chunks)
            comm.broadcast_params(flat)
            vector_to_params(flat, actor_params)
            if policy_step - last_log >= cfg.metric.log_every or cfg.dry_run:
                runner.log_dict(comm.player_trainer_object(None), policy_step)

        if policy_step - last_log >= cfg.metric.log_every or cfg.dry_run:
            runner.log_dict(aggregator.compute(), policy_step)
            aggregator.reset()
            tm = timer.compute()
            if tm.get("Time/env_interaction_time", 0) > 0:
                runner.log("Time/sps_env_interaction",
                           ((policy_step - last_log) * cfg.env.action_repeat) / tm["Time/env_interaction_time"],
                           policy_step)
            timer.reset()
            last_log = policy_step

        if (update >= learning_starts and cfg.checkpoint.every > 0
                and policy_step - last_checkpoint >= cfg.checkpoint.every) or cfg.dry_run:
            last_checkpoint = policy_step
            runner.call("on_checkpoint_player", comm=comm,
                        ckpt_path=os.path.join(log_dir, f"checkpoint/ckpt_{policy_step}_0.ckpt"),
                        replay_buffer=rb if cfg.buffer.checkpoint else None)

    comm.send_chunks(None)
    runner.call("on_checkpoint_player", comm=comm, ckpt_path=os.path.join(log_dir, f"checkpoint/ckpt_{policy_step}_0.ckpt"),
                replay_buffer=rb if cfg.buffer.checkpoint else None)
    envs.close()
    test(actor, runner, cfg, log_dir)


class _OneRank:
    world_size = 1
    global_rank = 0


def trainer(runner, cfg: Dict[str, Any], comm: DecoupledComm, log_dir: str):
    tr = comm.trainer_runner()
    device = runner.device
    is_first_trainer = comm.rank == 1
    envs = build_envs(tr, cfg, None)
    obs_space = envs.single_observation_space
    action_space = envs.single_action_space
    obs_dim = int(sum(int(np.prod(obs_space[k].shape)) for k in cfg.mlp_keys.encoder))
    envs.close()
    state = cfg.pop("_resume_state", None)
    agent = build_agent(tr, cfg, obs_dim, action_space, state["agent"] if state else None)
    qf_optimizer = build_optimizer(cfg.algo.critic.optimizer, agent.critic.parameters())
    actor_optimizer = build_optimizer(cfg.algo.actor.optimizer, agent.actor.parameters())
    alpha_optimizer = build_optimizer(cfg.algo.alpha.optimizer, [agent.log_alpha])
    if state:
        qf_optimizer.load_state_dict(state["qf_optimizer"])
        actor_optimizer.load_state_dict(state["actor_optimizer"])
        alpha_optimizer.load_state_dict(state["alpha_optimizer"])
    sac = SACTrainer(tr, cfg, agent, actor_optimizer, qf_optimizer, alpha_optimizer)
    actor_params = list(agent.actor.parameters())
    if is_first_trainer:
        comm.broadcast_params(params_to_vector(actor_params))
    aggregator = MetricAggregator({k: MeanMetric(sync_on_compute=cfg.metric.sync_on_compute)
                                   for k in ("Loss/value_loss", "Loss/policy_loss", "Loss/alpha_loss")})

    info = comm.broadcast_object_world(None)
    update, last_log, last_checkpoint = info["update"], info["last_log"], info["last_checkpoint"]
    train_step, last_train = 0, 0
    policy_steps_per_update = cfg.env.num_envs
    policy_step = update * policy_steps_per_update
    ema_every = cfg.algo.critic.target_network_frequency // policy_steps_per_update + 1
    n_tr = comm.world_size - 1

    def ckpt_state():
        return {
            "agent": agent.state_dict(),
            "qf_optimizer": qf_optimizer.state_dict(),
            "actor_optimizer": actor_optimizer.state_dict(),
            "alpha_optimizer": alpha_optimizer.state_dict(),
            "update": update,
            "batch_size": cfg.per_rank_batch_size * n_tr,
            "last_log": last_log,
            "last_checkpoint": last_checkpoint,
        }

    while True:
        data = comm.recv_chunk()
        if data is None:
            if is_first_trainer:
                runner.call("on_checkpoint_trainer", comm=comm, state=ckpt_state())
            return
        B = cfg.per_rank_batch_size
        with timer("Time/train_time"):
            n = data["rewards"].shape[0]
            for start in range(0, n, B):
                bd = {k: data[k][start : start + B] for k in _KEYS}
                if bd["rewards"].shape[0] != B and sac.critic_step.enabled:
                    from sheeprl_prey_amd.algos.sac.sac import _eager_train

                    _eager_train(sac, bd, update % ema_every == 0, aggregator)
                else:
                    sac.train(bd, update % ema_every == 0, aggregator)
            train_step += n_tr
        if is_first_trainer:
            comm.broadcast_params(params_to_vector(actor_params))
        if policy_step - last_log >= cfg.metric.log_every or cfg.dry_run:
            metrics = aggregator.compute()
            aggregator.reset()
            tm = timer.compute()
            if tm.get("Time/train_time", 0) > 0:
                metrics["Time/sps_train"] = (train_step - last_train) / tm["Time/train_time"]
            timer.reset()
            if is_first_trainer:
                comm.player_trainer_object(metrics)
            last_log = policy_step
            last_train = train_step
        if (cfg.checkpoint.every > 0 and policy_step - last_checkpoint >= cfg.checkpoint.every) or cfg.dry_run:
            last_checkpoint = policy_step
            if is_first_trainer:
                runner.call("on_checkpoint_trainer", comm=comm, state=ckpt_state())
        update += 1
        policy_step += policy_steps_per_update


@register_algorithm(decoupled=True)
def main(runner, cfg: Dict[str, Any]):
    comm = DecoupledComm(runner)
    cfg, state = load_resume(runner, cfg)
    runner.seed_everything(cfg.seed)
    if "minedojo" in str(cfg.env.wrapper.get("_target_", "")).lower():
        raise ValueError("MineDojo is not currently supported by SAC agent, since it does not take into consideration "
                         "the action masks provided by the environment, but needed in order to play correctly the game.")
    if len(cfg.cnn_keys.encoder) > 0:
        import warnings

        warnings.warn("SAC algorithm cannot allow to use images as observations, the CNN keys will be ignored")
        cfg.cnn_keys.encoder = []
    # the player's (possibly resumed) config is the source of truth (reference ``sac_decoupled.py:81``)
    cfg = comm.broadcast_object_world(cfg if comm.is_player else None)
    logger, log_dir = setup_logger(runner, cfg)
    if state is not None:
        cfg["_resume_state"] = state
    if comm.is_player:
        player(runner, cfg, comm, log_dir)
    else:
        trainer(runner, cfg, comm, log_dir)
