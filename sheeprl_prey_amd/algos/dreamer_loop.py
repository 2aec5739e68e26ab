"""Env-interaction / replay / training loop shared by DreamerV1, DreamerV2 and Plan2Explore
(reference: ``dreamer_v1/dreamer_v1.py:350-520``, ``dreamer_v2/dreamer_v2.py:420-882``,
``p2e_dv1/p2e_dv1.py``, ``p2e_dv2/p2e_dv2.py`` - the same ~400-line loop, written once here).

The algorithm supplies a ``DreamerSpec``: its player, a ``train_step(batch) -> metrics`` callable
(a captured phased step), the target-network hook, the checkpoint state and the test routine.
Variants:
  * ``dv1``: no ``is_first``; trains when ``update > learning_starts`` with ``per_rank_gradient_steps``
  * ``dv2``: ``is_first`` flags, sequential or episode replay, pre-training steps at
    ``learning_starts``, hard target-critic copies every ``target_network_update_freq`` steps.
"""
from __future__ import annotations

import copy
import os
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Sequence

import numpy as np
import torch
from torch import Tensor

from sheeprl_prey_amd.algos.common import episode_stats, log_throughput, warn_log_ckpt_every
from sheeprl_prey_amd.data.buffers import AsyncReplayBuffer, EpisodeBuffer
from sheeprl_prey_amd.data.tensordict import TensorDict, cat
from sheeprl_prey_amd.utils.timer import timer
from sheeprl_prey_amd.utils.utils import polynomial_decay


@dataclass
class DreamerSpec:
    variant: str  # "dv1" | "dv2"
    player: Any
    train_step: Callable[[Dict[str, Tensor]], Dict[str, Tensor]]
    checkpoint_state: Callable[[], Dict[str, Any]]
    test: Callable[[], Any]
    update_target: Optional[Callable[[], None]] = None
    target_every: int = 0
    extra_after_train: Optional[Callable[[], None]] = None
    obs_offset: float = -0.5
    actor_cls_name: str = ""
    before_update: Optional[Callable[[int], None]] = None


def build_replay(cfg, runner, log_dir: str, buffer_size: int):
    rank = runner.global_rank
    btype = str(cfg.buffer.get("type", "sequential")).lower()
    memmap_dir = os.path.join(log_dir, "memmap_buffer", f"rank_{rank}")
    if btype == "sequential":
        return AsyncReplayBuffer(buffer_size, cfg.env.num_envs, device="cpu", memmap=cfg.buffer.memmap,
                                 memmap_dir=memmap_dir, sequential=True), btype
    if btype == "episode":
        return EpisodeBuffer(buffer_size, sequence_length=cfg.per_rank_sequence_length, device="cpu",
                             memmap=cfg.buffer.memmap, memmap_dir=memmap_dir), btype
    raise ValueError(f"Unrecognized buffer type: must be one of `sequential` or `episode`, received: {btype}")


def restore_rb(rb, state, runner) -> None:
    saved = state.get("rb") if state else None
    if saved is None:
        return
    if isinstance(saved, list):
        if len(saved) != runner.world_size:
            raise RuntimeError(f"Given {len(saved)}, but {runner.world_size} processes are instantiated")
        saved = saved[runner.global_rank]
    rb.load_state_dict(saved)


def run_dreamer_loop(runner, cfg, state, envs, spec: DreamerSpec, aggregator, rb, buffer_type: str,
                     actions_dim: Sequence[int], is_continuous: bool, log_dir: str, expl_decay_steps: int = 0,
                     per_rank_gradient_steps: int = 0) -> None:
    device = runner.device
    rank, world_size = runner.global_rank, runner.world_size
    dv2 = spec.variant != "dv1"
    player = spec.player
    obs_keys = list(cfg.cnn_keys.encoder) + list(cfg.mlp_keys.encoder)
    clip_rewards_fn = (lambda r: torch.tanh(r)) if cfg.env.clip_rewards else (lambda r: r)
    step_data = TensorDict({}, batch_size=[cfg.env.num_envs], device="cpu")

    train_step = 0
    last_train = 0
    start_step = state["update"] // world_size if state else 1
    policy_step = state["update"] * cfg.env.num_envs if state else 0
    last_log = state["last_log"] if state else 0
    last_checkpoint = state["last_checkpoint"] if state else 0
    policy_steps_per_update = int(cfg.env.num_envs * world_size)
    updates_before_training = cfg.algo.train_every // policy_steps_per_update if not cfg.dry_run else 0
    num_updates = cfg.total_steps // policy_steps_per_update if not cfg.dry_run else 1
    learning_starts = cfg.algo.learning_starts // policy_steps_per_update if not cfg.dry_run else 0
    if state and not cfg.buffer.checkpoint:
        learning_starts += start_step
    max_step_expl_decay = cfg.algo.player.max_step_expl_decay // (cfg.algo.per_rank_gradient_steps * world_size)
    if state:
        player.expl_amount = polynomial_decay(expl_decay_steps, initial=cfg.algo.player.expl_amount,
                                              final=cfg.algo.player.expl_min, max_decay_steps=max_step_expl_decay)
    warn_log_ckpt_every(cfg, policy_steps_per_update)

    episode_steps: List[List[TensorDict]] = [[] for _ in range(cfg.env.num_envs)]

    def add_rows(td: TensorDict, idx: Optional[List[int]] = None) -> None:
        if buffer_type == "sequential":
            rb.add(td[None, ...], idx)
        else:
            rows = range(cfg.env.num_envs) if idx is None else idx
            for j, e in enumerate(rows):
                episode_steps[e].append(td[j : j + 1][None, ...])

    def to_obs(o) -> Dict[str, Tensor]:
        out = {}
        for k in obs_keys:
            t = torch.from_numpy(np.asarray(o[k])).view(cfg.env.num_envs, *np.asarray(o[k]).shape[1:])
            out[k] = t.float() if k in cfg.mlp_keys.encoder else t
        return out

    o = envs.reset(seed=cfg.seed)[0]
    obs = to_obs(o)
    for k in obs_keys:
        step_data[k] = obs[k]
    step_data["dones"] = torch.zeros(cfg.env.num_envs, 1)
    step_data["actions"] = torch.zeros(cfg.env.num_envs, int(sum(actions_dim)))
    step_data["rewards"] = torch.zeros(cfg.env.num_envs, 1)
    if dv2:
        step_data["is_first"] = torch.ones_like(step_data["dones"])
    add_rows(step_data)
    player.init_states()

    for update in range(start_step, num_updates + 1):
        policy_step += cfg.env.num_envs * world_size
        if spec.before_update is not None:
            spec.before_update(update)
        with timer("Time/env_interaction_time"):
            random_phase = update <= learning_starts and state is None and "minedojo" not in spec.actor_cls_name.lower()
            if random_phase:
                real_actions = actions = np.array(envs.action_space.sample())
                if not is_continuous:
                    actions = np.concatenate(
                        [np.eye(d, dtype=np.float32)[a] for a, d in
                         zip(actions.reshape(len(actions_dim), -1), actions_dim)], axis=-1)
            else:
                with torch.no_grad():
                    pre = {}
                    for k, v in obs.items():
                        v = v[None].to(device, non_blocking=v.is_pinned())
                        pre[k] = v / 255.0 + spec.obs_offset if k in cfg.cnn_keys.encoder else v
                    mask = {k: v for k, v in pre.items() if k.startswith("mask")} or None
                    real_actions = actions = player.get_exploration_action(pre, is_continuous, mask)
                    actions = torch.cat(actions, -1).cpu().numpy()
                    if is_continuous:
                        real_actions = torch.cat(real_actions, -1).cpu().numpy()
                    else:
                        real_actions = np.array([a.cpu().argmax(dim=-1).numpy() for a in real_actions])
            if dv2:
                step_data["is_first"] = copy.deepcopy(step_data["dones"])
            o, rewards, dones, truncated, infos = envs.step(np.asarray(real_actions).reshape(envs.action_space.shape))
            dones = np.logical_or(dones, truncated)
            if cfg.dry_run and buffer_type == "episode":
                dones = np.ones_like(dones)

        for i, ep_rew, ep_len in episode_stats(infos):
            aggregator.update("Rewards/rew_avg", ep_rew)
            aggregator.update("Game/ep_len_avg", ep_len)
            runner.print(f"Rank-0: policy_step={policy_step}, reward_env_{i}={ep_rew[-1]}")

        real_next = {k: np.array(v, copy=True) for k, v in o.items()}
        if "final_observation" in infos:
            for idx, final in enumerate(infos["final_observation"]):
                if final is not None:
                    for k, v in final.items():
                        if k in real_next:
                            real_next[k][idx] = v
        next_obs = to_obs(o)
        for k, v in to_obs(real_next).items():
            step_data[k] = v
        obs = next_obs
        dones_t = torch.from_numpy(np.asarray(dones)).view(cfg.env.num_envs, -1).float()
        step_data["dones"] = dones_t
        step_data["actions"] = torch.from_numpy(np.asarray(actions)).view(cfg.env.num_envs, -1).float()
        step_data["rewards"] = clip_rewards_fn(torch.from_numpy(np.asarray(rewards)).view(cfg.env.num_envs, -1).float())
        add_rows(step_data)

        dones_idxes = dones_t.nonzero(as_tuple=True)[0].tolist()
        if dones_idxes:
            n = len(dones_idxes)
            reset_data = TensorDict({}, batch_size=[n], device="cpu")
            for k in obs_keys:
                reset_data[k] = next_obs[k][dones_idxes]
            reset_data["dones"] = torch.zeros(n, 1)
            reset_data["actions"] = torch.zeros(n, int(np.sum(actions_dim)))
            reset_data["rewards"] = torch.zeros(n, 1)
            if dv2:
                reset_data["is_first"] = torch.ones_like(reset_data["dones"])
            if buffer_type == "episode":
                for j, d in enumerate(dones_idxes):
                    if len(episode_steps[d]) >= cfg.per_rank_sequence_length:
                        rb.add(cat(episode_steps[d], 0).view(-1))
                    episode_steps[d] = [reset_data[j : j + 1][None, ...]]
            else:
                rb.add(reset_data[None, ...], dones_idxes)
            for d in dones_idxes:
                step_data["dones"][d] = torch.zeros_like(step_data["dones"][d])
            player.init_states(dones_idxes)

        updates_before_training -= 1
        ready = (update >= learning_starts) if dv2 else (update > learning_starts)
        if ready and updates_before_training <= 0 and (buffer_type != "episode" or len(rb) > 0):
            runner.barrier()
            if dv2 and update == learning_starts:
                n_samples = cfg.algo.per_rank_pretrain_steps
            else:
                n_samples = cfg.algo.per_rank_gradient_steps
            if buffer_type == "sequential":
                local = rb.sample(cfg.per_rank_batch_size, sequence_length=cfg.per_rank_sequence_length,
                                  n_samples=n_samples)
            else:
                local = rb.sample(cfg.per_rank_batch_size, n_samples=n_samples,
                                  prioritize_ends=cfg.buffer.get("prioritize_ends", False))
            local = local.to(device)
            with timer("Time/train_time"):
                for i in range(n_samples):
                    if spec.update_target is not None and spec.target_every > 0 and \
                            per_rank_gradient_steps % spec.target_every == 0:
                        spec.update_target()
                    batch = {k: v[i].float() if v.dtype != torch.uint8 else v[i] for k, v in local.items()}
                    metrics = spec.train_step(batch)
                    for k, v in metrics.items():
                        if k in aggregator:
                            aggregator.update(k, v)
                    per_rank_gradient_steps += 1
                train_step += world_size
            updates_before_training = cfg.algo.train_every // policy_steps_per_update
            if cfg.algo.player.expl_decay:
                expl_decay_steps += 1
                player.expl_amount = polynomial_decay(expl_decay_steps, initial=cfg.algo.player.expl_amount,
                                                      final=cfg.algo.player.expl_min,
                                                      max_decay_steps=max_step_expl_decay)
            if "Params/exploration_amout" in aggregator:
                aggregator.update("Params/exploration_amout", player.expl_amount)
            if spec.extra_after_train is not None:
                spec.extra_after_train()

        if policy_step - last_log >= cfg.metric.log_every or update == num_updates or cfg.dry_run:
            runner.log_dict(aggregator.compute(), policy_step)
            aggregator.reset()
            log_throughput(runner, timer.compute(), policy_step, last_log, train_step, last_train, cfg.env.action_repeat)
            timer.reset()
            last_log = policy_step
            last_train = train_step

        if (cfg.checkpoint.every > 0 and policy_step - last_checkpoint >= cfg.checkpoint.every) or cfg.dry_run or \
                update == num_updates:
            last_checkpoint = policy_step
            ckpt_state = spec.checkpoint_state()
            ckpt_state.update({
                "expl_decay_steps": expl_decay_steps,
                "update": update * world_size,
                "batch_size": cfg.per_rank_batch_size * world_size,
                "last_log": last_log,
                "last_checkpoint": last_checkpoint,
            })
            runner.call("on_checkpoint_coupled", ckpt_path=os.path.join(log_dir, f"checkpoint/ckpt_{policy_step}_{rank}.ckpt"),
                        state=ckpt_state, replay_buffer=rb if cfg.buffer.checkpoint else None)

    envs.close()
    if runner.is_global_zero:
        spec.test()
