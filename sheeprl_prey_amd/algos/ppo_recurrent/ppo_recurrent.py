"""Recurrent PPO (reference: ``sheeprl/algos/ppo_recurrent/ppo_recurrent.py:33-474``).

Rollouts keep the LSTM state and previous action per env; after GAE every env's rollout is cut
at episode ends, the episodes split into ``per_rank_sequence_length`` chunks and padded into
``[L, N]`` sequences with a mask.  Training runs ``update_epochs`` over random sequence minibatches.
Masked reductions are computed as ``sum(x*m)/sum(m)`` on device (the reference indexes with the
boolean mask, a data-dependent shape that forces a host sync per minibatch) - same values.
"""
from __future__ import annotations

import copy
import os
import warnings
from typing import Any, Dict, List

import numpy as np
import torch
from torch import Tensor

from sheeprl_prey_amd.algos.common import (
    PolynomialLR,
    action_info,
    build_envs,
    check_obs_keys,
    episode_stats,
    load_resume,
    log_throughput,
    setup_logger,
    warn_log_ckpt_every,
)
from sheeprl_prey_amd.algos.ppo_recurrent.agent import RecurrentPPOAgent
from sheeprl_prey_amd.algos.ppo_recurrent.utils import test
from sheeprl_prey_amd.data.buffers import ReplayBuffer
from sheeprl_prey_amd.data.tensordict import TensorDict, pad_sequence
from sheeprl_prey_amd.parallel.flat_optim import build_optimizer
from sheeprl_prey_amd.utils.metric import MeanMetric, MetricAggregator
from sheeprl_prey_amd.utils.registry import register_algorithm
from sheeprl_prey_amd.utils.timer import timer
from sheeprl_prey_amd.utils.utils import gae, polynomial_decay


def _mmean(x: Tensor, m: Tensor) -> Tensor:
    return (x * m).sum() / m.sum().clamp(min=1)


def masked_losses(logprobs, old_logprobs, advantages, values, old_values, returns, entropies, m, cfg):
    """PPO losses restricted to the valid (mask=1) steps, reference ``ppo_recurrent.py:66-93``."""
    n = m.sum()
    if cfg.algo.normalize_advantages:
        mean = _mmean(advantages, m)
        var = ((advantages - mean).pow(2) * m).sum() / (n - 1).clamp(min=1)
        normed = (advantages - mean) / (var.sqrt() + 1e-8)
        advantages = torch.where(n > 1, normed, advantages)
    ratio = (logprobs - old_logprobs).exp()
    clip = cfg.algo.clip_coef
    pg = -torch.min(advantages * ratio, advantages * ratio.clamp(1 - clip, 1 + clip))
    pg_loss = _mmean(pg, m)
    if cfg.algo.clip_vloss:
        pred = old_values + (values - old_values).clamp(-clip, clip)
    else:
        pred = values
    v_loss = _mmean((pred - returns).pow(2), m)
    if str(cfg.algo.loss_reduction).lower() == "sum":
        ent_loss = -(entropies * m).sum()
    else:
        ent_loss = -_mmean(entropies, m)
    return pg_loss, v_loss, ent_loss


def train(runner, agent: RecurrentPPOAgent, optimizer, data: TensorDict, aggregator, cfg) -> None:
    num_sequences = data.shape[1]
    if cfg.per_rank_num_batches > 0:
        batch_size = num_sequences // cfg.per_rank_num_batches
        batch_size = batch_size if batch_size > 0 else num_sequences
    else:
        batch_size = 1
    obs_keys = list(dict.fromkeys(list(cfg.cnn_keys.encoder) + list(cfg.mlp_keys.encoder)))
    batches = []
    for _ in range(cfg.algo.update_epochs):
        perm = torch.randperm(num_sequences)
        batches += [perm[s : s + batch_size] for s in range(0, num_sequences, batch_size)]
    # ranks can hold different numbers of sequences: agree on the step count (DDP Join semantics)
    n_max = runner.max_steps(len(batches))
    for i in range(n_max):
        if i >= len(batches):
            runner.shadow_step(optimizer)
            continue
        idx = batches[i].to(data.device)
        batch = data[:, idx]
        m = batch["mask"].unsqueeze(-1).float()
        obs = {k: batch[k] / 255.0 - 0.5 if k in cfg.cnn_keys.encoder else batch[k] for k in obs_keys}
        _, logprobs, entropies, values, _ = agent(
            obs, prev_actions=batch["prev_actions"], prev_states=(batch["prev_hx"][:1], batch["prev_cx"][:1]),
            actions=torch.split(batch["actions"], agent.actions_dim, dim=-1))
        pg, vl, el = masked_losses(logprobs, batch["logprobs"], batch["advantages"], values, batch["values"],
                                   batch["returns"], entropies, m, cfg)
        loss = pg + cfg.algo.vf_coef * vl + cfg.algo.ent_coef * el
        optimizer.zero_grad()
        runner.backward(loss, optimizer)
        if cfg.algo.max_grad_norm > 0.0:
            runner.clip_gradients(agent, optimizer, max_norm=cfg.algo.max_grad_norm)
        optimizer.step()
        aggregator.update("Loss/policy_loss", pg.detach())
        aggregator.update("Loss/value_loss", vl.detach())
        aggregator.update("Loss/entropy_loss", el.detach())
    # every rank takes part in the min-steps collective (no short-circuit), then re-syncs if uneven
    if runner.world_size > 1 and runner.max_steps(-len(batches)) != -n_max:
        runner.sync_from_last_joiner(agent, len(batches), n_max)


def split_sequences(local: TensorDict, num_envs: int, rollout_steps: int, seq_len: int) -> List[TensorDict]:
    """Cut each env's rollout at its episode ends, then into ``seq_len`` chunks
    (reference ``ppo_recurrent.py:386-404``)."""
    out: List[TensorDict] = []
    dones = local["dones"].detach().cpu().numpy().reshape(rollout_steps, num_envs)
    for e in range(num_envs):
        env_data = local[:, e]
        ends = np.nonzero(dones[:, e])[0].tolist() + [rollout_steps]
        start = 0
        for end in ends:
            ep = env_data[start : end + 1]
            if ep.shape[0] > 0:
                if seq_len and seq_len > 0:
                    for s in range(0, ep.shape[0], seq_len):
                        out.append(ep[s : s + seq_len])
                else:
                    out.append(ep)
            start = end + 1
    return out


@register_algorithm()
def main(runner, cfg: Dict[str, Any]):
    initial_ent_coef = copy.deepcopy(cfg.algo.ent_coef)
    initial_clip_coef = copy.deepcopy(cfg.algo.clip_coef)
    if "minedojo" in str(cfg.env.wrapper.get("_target_", "")).lower():
        raise ValueError("MineDojo is not currently supported by PPO Recurrent agent, since it does not take into "
                         "consideration the action masks provided by the environment, but needed in order to play "
                         "correctly the game. As an alternative you can use one of the Dreamers' agents.")
    if cfg.buffer.share_data:
        warnings.warn("The script has been called with `buffer.share_data=True`: with recurrent PPO only gradients "
                      "are shared")
    cfg, state = load_resume(runner, cfg)
    device = runner.device
    rank, world_size = runner.global_rank, runner.world_size
    runner.seed_everything(cfg.seed + rank)

    logger, log_dir = setup_logger(runner, cfg)
    envs = build_envs(runner, cfg, log_dir)
    obs_space = envs.single_observation_space
    check_obs_keys(cfg, obs_space)
    runner.print("Encoder CNN keys:", cfg.cnn_keys.encoder)
    runner.print("Encoder MLP keys:", cfg.mlp_keys.encoder)
    obs_keys = list(cfg.cnn_keys.encoder) + list(cfg.mlp_keys.encoder)
    is_continuous, _, actions_dim = action_info(envs.single_action_space)
    agent = RecurrentPPOAgent(actions_dim, obs_space, cfg.algo.encoder, cfg.algo.rnn, cfg.algo.actor, cfg.algo.critic,
                              cfg.cnn_keys.encoder, cfg.mlp_keys.encoder, is_continuous, cfg.distribution,
                              cfg.env.num_envs, cfg.env.screen_size, device)
    if state:
        agent.load_state_dict(state["agent"])
    agent = runner.setup_module(agent)
    optimizer = build_optimizer(cfg.algo.optimizer, agent.parameters())
    if state:
        optimizer.load_state_dict(state["optimizer"])

    aggregator = MetricAggregator({k: MeanMetric(sync_on_compute=cfg.metric.sync_on_compute) for k in (
        "Rewards/rew_avg", "Game/ep_len_avg", "Loss/value_loss", "Loss/policy_loss", "Loss/entropy_loss")})
    rb = ReplayBuffer(cfg.algo.rollout_steps, cfg.env.num_envs, device=device,
                      memmap=cfg.buffer.memmap and device.type == "cpu",
                      memmap_dir=os.path.join(log_dir, "memmap_buffer", f"rank_{rank}"))
    step_data = TensorDict({}, batch_size=[1, cfg.env.num_envs], device=device)

    last_train = 0
    train_step = 0
    start_step = state["update"] // world_size if state else 1
    policy_step = state["update"] * cfg.env.num_envs * cfg.algo.rollout_steps if state else 0
    last_log = state["last_log"] if state else 0
    last_checkpoint = state["last_checkpoint"] if state else 0
    policy_steps_per_update = int(cfg.env.num_envs * cfg.algo.rollout_steps * world_size)
    num_updates = cfg.total_steps // policy_steps_per_update if not cfg.dry_run else 1
    warn_log_ckpt_every(cfg, policy_steps_per_update)
    scheduler = None
    if cfg.algo.anneal_lr:
        scheduler = PolynomialLR(optimizer, total_iters=num_updates, power=1.0)
        if state and state.get("scheduler"):
            scheduler.load_state_dict(state["scheduler"])

    def to_obs(o):
        out = {}
        for k in obs_keys:
            t = torch.as_tensor(np.asarray(o[k]), device=device)
            out[k] = t.view(cfg.env.num_envs, -1, *t.shape[-2:]) if k in cfg.cnn_keys.encoder else t.float()
        return out

    def norm(obs):
        return {k: obs[k][None] / 255.0 - 0.5 if k in cfg.cnn_keys.encoder else obs[k][None] for k in obs_keys}

    obs = to_obs(envs.reset(seed=cfg.seed)[0])
    for k in obs_keys:
        step_data[k] = obs[k][None]
    prev_states = agent.initial_states
    prev_actions = torch.zeros(1, cfg.env.num_envs, sum(actions_dim), device=device)
    for update in range(start_step, num_updates + 1):
        for _ in range(cfg.algo.rollout_steps):
            policy_step += cfg.env.num_envs * world_size
            with timer("Time/env_interaction_time"):
                with torch.no_grad():
                    actions, logprobs, _, values, states = agent(norm(obs), prev_actions=prev_actions,
                                                                 prev_states=prev_states)
                    if is_continuous:
                        real_actions = torch.cat(actions, -1).cpu().numpy()
                    else:
                        real_actions = np.concatenate([a.argmax(-1).cpu().numpy() for a in actions], axis=-1)
                    actions = torch.cat(actions, -1)
                o, rewards, dones, truncated, info = envs.step(real_actions.reshape(envs.action_space.shape))
                trunc = np.nonzero(truncated)[0]
                if len(trunc) > 0:
                    final = {}
                    for k in obs_keys:
                        v = torch.as_tensor(np.stack([np.asarray(info["final_observation"][e][k]) for e in trunc]),
                                            dtype=torch.float32, device=device)[None]
                        if k in cfg.cnn_keys.encoder:
                            v = v.view(1, len(trunc), -1, *v.shape[-2:]) / 255.0 - 0.5
                        final[k] = v
                    with torch.no_grad():
                        feat = agent.feature_extractor(final)
                        tix = torch.as_tensor(trunc, device=device)
                        rnn_out, _ = agent.rnn(torch.cat((feat, actions[:, tix]), -1), tuple(s[:, tix] for s in states))
                        vals = agent.get_values(rnn_out).cpu().numpy()
                    rewards[trunc] += vals.reshape(rewards[trunc].shape)
                dones = torch.as_tensor(np.logical_or(dones, truncated), dtype=torch.float32,
                                        device=device).view(1, cfg.env.num_envs, -1)
                rewards = torch.as_tensor(rewards, dtype=torch.float32, device=device).view(1, cfg.env.num_envs, -1)
            step_data["dones"] = dones
            step_data["values"] = values
            step_data["actions"] = actions
            step_data["rewards"] = rewards
            step_data["logprobs"] = logprobs
            step_data["prev_hx"] = prev_states[0]
            step_data["prev_cx"] = prev_states[1]
            step_data["prev_actions"] = prev_actions
            step_data["returns"] = torch.zeros_like(rewards)
            step_data["advantages"] = torch.zeros_like(rewards)
            rb.add(step_data)
            prev_actions = (1 - dones) * actions
            obs = to_obs(o)
            for k in obs_keys:
                step_data[k] = obs[k][None]
            prev_states = tuple((1 - dones) * s for s in states) if cfg.algo.reset_recurrent_state_on_done else states
            for i, ep_rew, ep_len in episode_stats(info):
                aggregator.update("Rewards/rew_avg", ep_rew)
                aggregator.update("Game/ep_len_avg", ep_len)
                runner.print(f"Rank-0: policy_step={policy_step}, reward_env_{i}={ep_rew[-1]}")

        with torch.no_grad():
            feat = agent.feature_extractor(norm(obs))
            rnn_out, _ = agent.rnn(torch.cat((feat, actions), -1), states)
            next_values = agent.get_values(rnn_out)
            returns, advantages = gae(rb["rewards"], rb["values"], rb["dones"], next_values, cfg.algo.rollout_steps,
                                      cfg.algo.gamma, cfg.algo.gae_lambda)
            rb["returns"] = returns.float()
            rb["advantages"] = advantages.float()
        seqs = split_sequences(rb.buffer, cfg.env.num_envs, cfg.algo.rollout_steps, cfg.per_rank_sequence_length)
        padded = pad_sequence(seqs, return_mask=True)
        with timer("Time/train_time"):
            train(runner, agent, optimizer, padded, aggregator, cfg)
        train_step += world_size

        if cfg.algo.anneal_lr:
            runner.log("Info/learning_rate", scheduler.get_last_lr()[0], policy_step)
            scheduler.step()
        else:
            runner.log("Info/learning_rate", cfg.algo.optimizer.lr, policy_step)
        runner.log("Info/clip_coef", cfg.algo.clip_coef, policy_step)
        if cfg.algo.anneal_clip_coef:
            cfg.algo.clip_coef = polynomial_decay(update, initial=initial_clip_coef, final=0.0,
                                                  max_decay_steps=num_updates, power=1.0)
        runner.log("Info/ent_coef", cfg.algo.ent_coef, policy_step)
        if cfg.algo.anneal_ent_coef:
            cfg.algo.ent_coef = polynomial_decay(update, initial=initial_ent_coef, final=0.0,
                                                 max_decay_steps=num_updates, power=1.0)

        if policy_step - last_log >= cfg.metric.log_every or update == num_updates or cfg.dry_run:
            runner.log_dict(aggregator.compute(), policy_step)
            aggregator.reset()
            log_throughput(runner, timer.compute(), policy_step, last_log, train_step, last_train,
                           cfg.env.action_repeat)
            timer.reset()
            last_log = policy_step
            last_train = train_step

        if (cfg.checkpoint.every > 0 and policy_step - last_checkpoint >= cfg.checkpoint.every) or cfg.dry_run or \
                update == num_updates:
            last_checkpoint = policy_step
            ckpt_state = {
                "agent": agent.state_dict(),
                "optimizer": optimizer.state_dict(),
                "scheduler": scheduler.state_dict() if scheduler is not None else None,
                "update": update * world_size,
                "batch_size": cfg.per_rank_batch_size * world_size,
                "last_log": last_log,
                "last_checkpoint": last_checkpoint,
            }
            runner.call("on_checkpoint_coupled", ckpt_path=os.path.join(log_dir, f"checkpoint/ckpt_{policy_step}_{rank}.ckpt"),
                        state=ckpt_state)

    envs.close()
    if runner.is_global_zero:
        test(agent, runner, cfg, log_dir)
