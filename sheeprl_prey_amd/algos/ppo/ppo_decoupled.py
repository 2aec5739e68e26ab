"""PPO, decoupled actor-learner (reference: ``sheeprl/algos/ppo/ppo_decoupled.py:36-633``).

rank 0 (player) collects ``rollout_steps x num_envs`` transitions, computes GAE with the HIP scan,
shuffles and splits the rollout almost evenly into one chunk per trainer (packed P2P over
RCCL/xGMI, ``parallel/decoupled.py``), then receives the updated weights from trainer 1.
ranks 1..N-1 (trainers) run ``update_epochs`` x minibatch PPO with gradients averaged over the
optimisation group (flat-slab all-reduce); trainer 1 also ships metrics and checkpoint state.
"""
from __future__ import annotations

import copy
import os
import warnings
from typing import Any, Dict

import numpy as np
import torch

from sheeprl_prey_amd.algos.common import (
    PolynomialLR,
    action_info,
    build_envs,
    check_obs_keys,
    episode_stats,
    load_resume,
    setup_logger,
)
from sheeprl_prey_amd.algos.ppo.agent import PPOAgent
from sheeprl_prey_amd.algos.ppo.loss import entropy_loss, policy_loss, value_loss
from sheeprl_prey_amd.algos.ppo.utils import test
from sheeprl_prey_amd.data.buffers import ReplayBuffer
from sheeprl_prey_amd.data.tensordict import TensorDict
from sheeprl_prey_amd.parallel.decoupled import DecoupledComm, params_to_vector, vector_to_params
from sheeprl_prey_amd.parallel.flat_optim import build_optimizer
from sheeprl_prey_amd.utils.metric import MeanMetric, MetricAggregator
from sheeprl_prey_amd.utils.registry import register_algorithm
from sheeprl_prey_amd.utils.timer import timer
from sheeprl_prey_amd.utils.utils import gae, normalize_tensor, polynomial_decay


def _agent(cfg, envs) -> PPOAgent:
    obs_space = envs.single_observation_space
    is_continuous, _, actions_dim = action_info(envs.single_action_space)
    return PPOAgent(actions_dim, obs_space, cfg.algo.encoder, cfg.algo.actor, cfg.algo.critic, cfg.cnn_keys.encoder,
                    cfg.mlp_keys.encoder, cfg.env.screen_size, cfg.distribution, is_continuous)


def _norm(obs, cnn_keys, keys):
    return {k: obs[k] / 255.0 - 0.5 if k in cnn_keys else obs[k] for k in keys}


def player(runner, cfg: Dict[str, Any], comm: DecoupledComm, log_dir: str):
    device = runner.device
    envs = build_envs(runner, cfg, log_dir)
    obs_space = envs.single_observation_space
    check_obs_keys(cfg, obs_space)
    obs_keys = list(cfg.cnn_keys.encoder) + list(cfg.mlp_keys.encoder)
    is_continuous, _, _ = action_info(envs.single_action_space)
    agent = _agent(cfg, envs).to(device)
    params = list(agent.parameters())
    flat = torch.empty_like(params_to_vector(params))
    comm.broadcast_params(flat)
    vector_to_params(flat, params)

    aggregator = MetricAggregator({k: MeanMetric() for k in ("Rewards/rew_avg", "Game/ep_len_avg")})
    rb = ReplayBuffer(cfg.algo.rollout_steps, cfg.env.num_envs, device=device,
                      memmap=cfg.buffer.memmap and device.type == "cpu",
                      memmap_dir=os.path.join(log_dir, "memmap_buffer", "rank_0"), obs_keys=obs_keys)
    step_data = TensorDict({}, batch_size=[cfg.env.num_envs], device=device)

    state = cfg.pop("_resume_state", None)
    start_step = state["update"] if state else 1
    policy_step = (state["update"] - 1) * cfg.env.num_envs * cfg.algo.rollout_steps if state else 0
    last_log = state["last_log"] if state else 0
    last_checkpoint = state["last_checkpoint"] if state else 0
    policy_steps_per_update = int(cfg.env.num_envs * cfg.algo.rollout_steps)
    num_updates = cfg.total_steps // policy_steps_per_update if not cfg.dry_run else 1
    comm.broadcast_object_world({"update": start_step, "last_log": last_log, "last_checkpoint": last_checkpoint,
                                 "num_updates": num_updates})
    n_tr = comm.world_size - 1

    def to_obs(o):
        out = {}
        for k in obs_keys:
            t = torch.as_tensor(np.asarray(o[k]), device=device)
            out[k] = t.view(cfg.env.num_envs, -1, *t.shape[-2:]) if k in cfg.cnn_keys.encoder else t.float()
        return out

    next_obs = to_obs(envs.reset(seed=cfg.seed)[0])
    for update in range(start_step, num_updates + 1):
        for _ in range(cfg.algo.rollout_steps):
            policy_step += cfg.env.num_envs
            with timer("Time/env_interaction_time"):
                with torch.no_grad():
                    actions, logprobs, _, values = agent(_norm(next_obs, cfg.cnn_keys.encoder, obs_keys))
                    if is_continuous:
                        real_actions = torch.cat(actions, -1).cpu().numpy()
                    else:
                        real_actions = np.stack([a.argmax(-1).cpu().numpy() for a in actions], -1)
                    actions = torch.cat(actions, -1)
                o, rewards, dones, truncated, info = envs.step(real_actions.reshape(envs.action_space.shape))
                trunc = np.nonzero(truncated)[0]
                if len(trunc) > 0:
                    final = {k: torch.as_tensor(np.stack([np.asarray(info["final_observation"][e][k]) for e in trunc]),
                                                dtype=torch.float32, device=device) for k in obs_keys}
                    for k in cfg.cnn_keys.encoder:
                        final[k] = final[k].view(len(trunc), -1, *final[k].shape[-2:]) / 255.0 - 0.5
                    with torch.no_grad():
                        v = agent.get_value(final).cpu().numpy()
                    rewards[trunc] += v.reshape(rewards[trunc].shape)
                dones = torch.as_tensor(np.logical_or(dones, truncated), dtype=torch.float32,
                                        device=device).view(cfg.env.num_envs, -1)
                rewards = torch.as_tensor(rewards, dtype=torch.float32, device=device).view(cfg.env.num_envs, -1)
            for k in obs_keys:
                step_data[k] = next_obs[k]
            step_data["dones"] = dones
            step_data["values"] = values
            step_data["actions"] = actions
            step_data["logprobs"] = logprobs
            step_data["rewards"] = rewards
            step_data["returns"] = torch.zeros_like(rewards)
            step_data["advantages"] = torch.zeros_like(rewards)
            rb.add(step_data.unsqueeze(0))
            next_obs = to_obs(o)
            for i, ep_rew, ep_len in episode_stats(info):
                aggregator.update("Rewards/rew_avg", ep_rew)
                aggregator.update("Game/ep_len_avg", ep_len)
                runner.print(f"Rank-0: policy_step={policy_step}, reward_env_{i}={ep_rew[-1]}")

        with torch.no_grad():
            next_values = agent.get_value(_norm(next_obs, cfg.cnn_keys.encoder, obs_keys))
            returns, advantages = gae(rb["rewards"], rb["values"], rb["dones"], next_values, cfg.algo.rollout_steps,
                                      cfg.algo.gamma, cfg.algo.gae_lambda)
            rb["returns"] = returns.float()
            rb["advantages"] = advantages.float()
        local = rb.buffer.view(-1)
        perm = torch.randperm(local.shape[0], device=local.device)
        sizes = [len(c) for c in np.array_split(np.arange(local.shape[0]), n_tr)]
        chunks, off = [], 0
        for s in sizes:
            idx = perm[off : off + s]
            chunks.append({k: v[idx] for k, v in local.items()})
            off += s
        comm.send_chunks(chunks)
        comm.broadcast_params(flat)
        vector_to_params(flat, params)

        if policy_step - last_log >= cfg.metric.log_every or cfg.dry_run:
            runner.log_dict(comm.player_trainer_object(None), policy_step)
            runner.log_dict(aggregator.compute(), policy_step)
            aggregator.reset()
            tm = timer.compute()
            if tm.get("Time/env_interaction_time", 0) > 0:
                runner.log("Time/sps_env_interaction",
                           ((policy_step - last_log) * cfg.env.action_repeat) / tm["Time/env_interaction_time"],
                           policy_step)
            timer.reset()
            last_log = policy_step

        if (cfg.checkpoint.every > 0 and policy_step - last_checkpoint >= cfg.checkpoint.every) or cfg.dry_run:
            last_checkpoint = policy_step
            runner.call("on_checkpoint_player", comm=comm,
                        ckpt_path=os.path.join(log_dir, f"checkpoint/ckpt_{policy_step}_0.ckpt"))

    comm.send_chunks(None)
    runner.call("on_checkpoint_player", comm=comm, ckpt_path=os.path.join(log_dir, f"checkpoint/ckpt_{policy_step}_0.ckpt"))
    envs.close()
    test(agent, runner, cfg, log_dir)


def trainer(runner, cfg: Dict[str, Any], comm: DecoupledComm):
    tr = comm.trainer_runner()
    is_first = comm.rank == 1
    envs = build_envs(tr, cfg, None)
    agent = _agent(cfg, envs)
    envs.close()
    state = cfg.pop("_resume_state", None)
    if state:
        agent.load_state_dict(state["agent"])
    agent = tr.setup_module(agent)
    optimizer = build_optimizer(cfg.algo.optimizer, agent.parameters())
    if state:
        optimizer.load_state_dict(state["optimizer"])
    if is_first:
        comm.broadcast_params(params_to_vector(agent.parameters()))
    info = comm.broadcast_object_world(None)
    update, last_log, last_checkpoint, num_updates = (info["update"], info["last_log"], info["last_checkpoint"],
                                                       info["num_updates"])
    scheduler = None
    if cfg.algo.anneal_lr:
        scheduler = PolynomialLR(optimizer, total_iters=num_updates, power=1.0)
        if state and state.get("scheduler"):
            scheduler.load_state_dict(state["scheduler"])
    aggregator = MetricAggregator({k: MeanMetric(sync_on_compute=cfg.metric.sync_on_compute)
                                   for k in ("Loss/value_loss", "Loss/policy_loss", "Loss/entropy_loss")})
    n_tr = comm.world_size - 1
    train_step, last_train = 0, 0
    policy_steps_per_update = cfg.env.num_envs * cfg.algo.rollout_steps
    policy_step = update * policy_steps_per_update
    initial_ent_coef = copy.deepcopy(cfg.algo.ent_coef)
    initial_clip_coef = copy.deepcopy(cfg.algo.clip_coef)
    obs_keys = list(cfg.cnn_keys.encoder) + list(cfg.mlp_keys.encoder)

    def ckpt_state():
        return {"agent": agent.state_dict(), "optimizer": optimizer.state_dict(),
                "scheduler": scheduler.state_dict() if scheduler is not None else None, "update": update,
                "batch_size": cfg.per_rank_batch_size * n_tr, "last_log": last_log, "last_checkpoint": last_checkpoint}

    while True:
        data = comm.recv_chunk()
        if data is None:
            if is_first:
                runner.call("on_checkpoint_trainer", comm=comm, state=ckpt_state())
            return
        train_step += n_tr
        n = data["rewards"].shape[0]
        with timer("Time/train_time"):
            dev = data["rewards"].device
            batches = [perm[s : s + cfg.per_rank_batch_size]
                       for perm in (torch.randperm(n, device=dev) for _ in range(cfg.algo.update_epochs))
                       for s in range(0, n, cfg.per_rank_batch_size)]
            # trainers can hold uneven chunks: agree on the step count, shadow the missing steps
            n_max = tr.max_steps(len(batches))
            for i in range(n_max):
                if i >= len(batches):
                    tr.shadow_step(optimizer)
                    continue
                batch = {k: v[batches[i]] for k, v in data.items()}
                obs = _norm(batch, cfg.cnn_keys.encoder, obs_keys)
                _, logprobs, entropy, new_values = agent(obs, torch.split(batch["actions"], agent.actions_dim, -1))
                adv = normalize_tensor(batch["advantages"]) if cfg.algo.normalize_advantages else batch["advantages"]
                pg = policy_loss(logprobs, batch["logprobs"], adv, cfg.algo.clip_coef, cfg.algo.loss_reduction)
                vl = value_loss(new_values, batch["values"], batch["returns"], cfg.algo.clip_coef,
                                cfg.algo.clip_vloss, cfg.algo.loss_reduction)
                el = entropy_loss(entropy, cfg.algo.loss_reduction)
                loss = pg + cfg.algo.vf_coef * vl + cfg.algo.ent_coef * el
                optimizer.zero_grad()
                tr.backward(loss, optimizer)
                if cfg.algo.max_grad_norm > 0.0:
                    tr.clip_gradients(agent, optimizer, max_norm=cfg.algo.max_grad_norm)
                optimizer.step()
                aggregator.update("Loss/policy_loss", pg.detach())
                aggregator.update("Loss/value_loss", vl.detach())
                aggregator.update("Loss/entropy_loss", el.detach())
            # every rank takes part in the min-steps collective (no short-circuit), then re-syncs if uneven
            if tr.max_steps(-len(batches)) != -n_max:
                tr.sync_from_last_joiner(agent, len(batches), n_max)
        if is_first:
            comm.broadcast_params(params_to_vector(agent.parameters()))
        if policy_step - last_log >= cfg.metric.log_every or cfg.dry_run:
            metrics = aggregator.compute()
            aggregator.reset()
            tm = timer.compute()
            if tm.get("Time/train_time", 0) > 0:
                metrics["Time/sps_train"] = (train_step - last_train) / tm["Time/train_time"]
            timer.reset()
            if is_first:
                metrics["Info/learning_rate"] = scheduler.get_last_lr()[0] if scheduler else cfg.algo.optimizer.lr
                metrics["Info/clip_coef"] = cfg.algo.clip_coef
                metrics["Info/ent_coef"] = cfg.algo.ent_coef
                comm.player_trainer_object(metrics)
            last_log = policy_step
            last_train = train_step
        if scheduler is not None:
            scheduler.step()
        if cfg.algo.anneal_clip_coef:
            cfg.algo.clip_coef = polynomial_decay(update, initial=initial_clip_coef, final=0.0,
                                                  max_decay_steps=num_updates, power=1.0)
        if cfg.algo.anneal_ent_coef:
            cfg.algo.ent_coef = polynomial_decay(update, initial=initial_ent_coef, final=0.0,
                                                 max_decay_steps=num_updates, power=1.0)
        if (cfg.checkpoint.every > 0 and policy_step - last_checkpoint >= cfg.checkpoint.every) or cfg.dry_run:
            last_checkpoint = policy_step
            if is_first:
                runner.call("on_checkpoint_trainer", comm=comm, state=ckpt_state())
        update += 1
        policy_step += policy_steps_per_update


@register_algorithm(decoupled=True)
def main(runner, cfg: Dict[str, Any]):
    if str(cfg.algo.get("topology", "player_trainers")) == "actor_fleet":
        # N-1 actor ranks -> 1 learner (ppo_actor_fleet.py); the default is the reference's 1 player +
        # N-1 trainers split
        from sheeprl_prey_amd.algos.ppo.ppo_actor_fleet import actor_fleet

        cfg, _ = load_resume(runner, cfg)
        runner.seed_everything(cfg.seed)
        _, log_dir = setup_logger(runner, cfg)
        return actor_fleet(runner, cfg, log_dir)
    comm = DecoupledComm(runner)
    if "minedojo" in str(cfg.env.wrapper.get("_target_", "")).lower():
        raise ValueError("MineDojo is not currently supported by PPO agent, since it does not take into consideration "
                         "the action masks provided by the environment, but needed in order to play correctly the game. "
                         "As an alternative you can use one of the Dreamers' agents.")
    if cfg.buffer.share_data:
        warnings.warn("You have called the script with `buffer.share_data=True`: decoupled scripts splits collected "
                      "data in an almost-even way between the number of trainers")
    cfg, state = load_resume(runner, cfg)
    runner.seed_everything(cfg.seed)
    cfg = comm.broadcast_object_world(cfg if comm.is_player else None)
    logger, log_dir = setup_logger(runner, cfg)
    if state is not None:
        cfg["_resume_state"] = state
    if comm.is_player:
        player(runner, cfg, comm, log_dir)
    else:
        trainer(runner, cfg, comm)
