"""PPO actor-fleet topology: N-1 actor ranks feed ONE learner (``algo.topology=actor_fleet`` of
``exp=ppo_decoupled``).  The reference's generalised multi-role template
(``examples/architecture_template.py:35-195``: players -> buffer -> trainers, parameters broadcast
back) specialised to the shape BASELINE config #2 names (1 learner + 7 actor ranks on one node).

rank 0 - learner: gathers every actor's rollout, runs the whole PPO update (``PPOTrainer``: the
         one-graph / fused single-rank update, no gradient collective at all), logs, checkpoints,
         broadcasts the flat weights.
rank 1..N-1 - actors: own ``env.num_envs`` envs each and a full agent copy (the critic too: GAE runs
         on the actor with the HIP reverse scan), collect ``rollout_steps`` x ``num_envs``
         transitions with the current weights, then wait for the next weights (on-policy).

Transport: a rollout is TWO fixed-shape slabs per actor - uint8 (pixel observations, never widened
to fp32 on the wire) and fp32 (vector observations, actions, log-probs, values, returns,
advantages, and three episode statistics) - gathered with ONE ``dist.gather`` each (RCCL over
xGMI on GPUs); the weights come back as ONE flat fp32 ``dist.broadcast``.  Shapes never change, so
no per-update header travels.
"""
from __future__ import annotations

import copy
import os
from typing import Any, Dict, List, Tuple

import numpy as np
import torch
import torch.distributed as dist
from torch import Tensor

from sheeprl_prey_amd.algos.common import PolynomialLR, action_info, build_envs, check_obs_keys, episode_stats
from sheeprl_prey_amd.algos.ppo.utils import test
from sheeprl_prey_amd.data.tensordict import TensorDict
from sheeprl_prey_amd.parallel.decoupled import params_to_vector, vector_to_params
from sheeprl_prey_amd.parallel.flat_optim import build_optimizer
from sheeprl_prey_amd.utils.metric import MeanMetric, MetricAggregator
from sheeprl_prey_amd.utils.timer import timer
from sheeprl_prey_amd.utils.utils import gae, polynomial_decay

LEARNER = 0
N_STATS = 3  # per actor and update: sum of finished-episode returns, their count, sum of their lengths


class _LocalRunner:
    """The learner's view of the runner: a single-rank job (no gradient collectives)."""

    def __init__(self, runner):
        self._r = runner

    def __getattr__(self, name):
        return getattr(self._r, name)

    world_size = 1
    global_rank = 0
    is_global_zero = True

    def sync_gradients(self, optimizer) -> None:
        return None

    def backward(self, loss, optimizer=None, **kwargs) -> None:
        loss.backward(**kwargs)

    def barrier(self, *args, **kwargs) -> None:
        return None  # the actors never take part in the learner's checkpointing

    def save(self, path: str, state) -> None:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        torch.save(state, path + ".tmp")
        os.replace(path + ".tmp", path)

    def call(self, hook: str, **kwargs) -> None:
        for cb in self._r.callbacks:
            fn = getattr(cb, hook, None)
            if fn is not None:
                fn(runner=self, **kwargs)


def _layout(cfg, obs_space, actions_width: int, T: int, ne: int) -> Tuple[List[Tuple[str, Tuple[int, ...]]], List[Tuple[str, Tuple[int, ...]]]]:
    """(uint8 fields, fp32 fields) of one actor's rollout slab, as (name, per-sample shape)."""
    u8, f32 = [], []
    for k in cfg.cnn_keys.encoder:
        shp = tuple(obs_space[k].shape)
        u8.append((k, (int(np.prod(shp[:-2])),) + shp[-2:]))  # frames x channels flattened, as ppo.main
    for k in cfg.mlp_keys.encoder:
        f32.append((k, tuple(obs_space[k].shape)))
    f32 += [("actions", (actions_width,)), ("logprobs", (1,)), ("values", (1,)), ("returns", (1,)), ("advantages", (1,)),
            ("rewards", (1,)), ("dones", (1,))]
    return u8, f32


def _numel(fields, n: int) -> int:
    return sum(n * int(np.prod(s)) for _, s in fields)


def _split(slab: Tensor, fields, n: int) -> Dict[str, Tensor]:
    out, off = {}, 0
    for k, s in fields:
        m = n * int(np.prod(s))
        out[k] = slab[off:off + m].view(n, *s)
        off += m
    return out


def actor_fleet(runner, cfg: Dict[str, Any], log_dir: str) -> None:
    rank, world = runner.global_rank, runner.world_size
    if world < 2:
        raise RuntimeError("The actor fleet needs at least 2 ranks (1 learner + actors): `fabric.devices>=2`")
    device = runner.device
    wire = device if runner.backend == "nccl" else torch.device("cpu")  # gloo moves host tensors
    n_actors = world - 1
    T, ne = int(cfg.algo.rollout_steps), int(cfg.env.num_envs)
    n = T * ne
    envs = build_envs(runner, cfg, log_dir if rank != LEARNER else None)
    obs_space = envs.single_observation_space
    check_obs_keys(cfg, obs_space)
    is_continuous, _, actions_dim = action_info(envs.single_action_space)
    from sheeprl_prey_amd.algos.ppo.ppo_decoupled import _agent, _norm

    torch.manual_seed(cfg.seed)  # identical initial weights on every rank (broadcast anyway below)
    agent = _agent(cfg, envs).to(device)
    params = list(agent.parameters())
    flat = params_to_vector(params).to(wire)
    dist.broadcast(flat, src=LEARNER)
    vector_to_params(flat.to(device), params)
    obs_keys = list(cfg.cnn_keys.encoder) + list(cfg.mlp_keys.encoder)
    u8_fields, f32_fields = _layout(cfg, obs_space, int(sum(actions_dim)), T, ne)
    n_u8, n_f32 = _numel(u8_fields, n), _numel(f32_fields, n) + N_STATS
    num_updates = max(1, int(cfg.total_steps // (n * n_actors))) if not cfg.dry_run else 1

    if rank == LEARNER:
        envs.close()
        _learner(runner, cfg, agent, flat, wire, u8_fields, f32_fields, n_u8, n_f32, num_updates, log_dir)
        return

    # ------------------------------------------------------------------ actor
    def to_obs(o):
        out = {}
        for k in obs_keys:
            t = torch.as_tensor(np.asarray(o[k]), device=device)
            out[k] = t.view(ne, -1, *t.shape[-2:]) if k in cfg.cnn_keys.encoder else t.float()
        return out

    next_obs = to_obs(envs.reset(seed=cfg.seed + rank)[0])
    u8 = torch.zeros(max(1, n_u8), dtype=torch.uint8, device=wire)
    f32 = torch.zeros(n_f32, dtype=torch.float32, device=wire)
    for update in range(1, num_updates + 1):
        buf: Dict[str, List[Tensor]] = {k: [] for k in obs_keys + ["actions", "logprobs", "values", "rewards", "dones"]}
        ep = [0.0, 0.0, 0.0]
        with timer("Time/env_interaction_time"):
            for _ in range(T):
                with torch.no_grad():
                    actions, logprobs, _, values = agent(_norm(next_obs, cfg.cnn_keys.encoder, obs_keys))
                real = (torch.cat(actions, -1).cpu().numpy() if is_continuous
                        else np.stack([a.argmax(-1).cpu().numpy() for a in actions], -1))
                o, rewards, dones, truncated, info = envs.step(real.reshape(envs.action_space.shape))
                trunc = np.nonzero(truncated)[0]
                if len(trunc) > 0:  # truncation bootstrap r += gamma-free V(final obs), as the reference
                    final = {k: torch.as_tensor(np.stack([np.asarray(info["final_observation"][e][k]) for e in trunc]),
                                                dtype=torch.float32, device=device) for k in obs_keys}
                    for k in cfg.cnn_keys.encoder:
                        final[k] = final[k].view(len(trunc), -1, *final[k].shape[-2:]) / 255.0 - 0.5
                    with torch.no_grad():
                        v = agent.get_value(final).cpu().numpy()
                    rewards[trunc] += v.reshape(rewards[trunc].shape)
                for k in obs_keys:
                    buf[k].append(next_obs[k])
                buf["actions"].append(torch.cat(actions, -1))
                buf["logprobs"].append(logprobs)
                buf["values"].append(values)
                buf["rewards"].append(torch.as_tensor(rewards, dtype=torch.float32, device=device).view(ne, 1))
                buf["dones"].append(torch.as_tensor(np.logical_or(dones, truncated), dtype=torch.float32,
                                                    device=device).view(ne, 1))
                next_obs = to_obs(o)
                for _, ep_rew, ep_len in episode_stats(info):
                    ep[0] += float(np.sum(ep_rew))
                    ep[1] += float(np.size(ep_rew))
                    ep[2] += float(np.sum(ep_len))
        roll = {k: torch.stack(v) for k, v in buf.items()}
        with torch.no_grad():
            nv = agent.get_value(_norm(next_obs, cfg.cnn_keys.encoder, obs_keys))
            ret, adv = gae(roll["rewards"], roll["values"], roll["dones"], nv, T, cfg.algo.gamma, cfg.algo.gae_lambda)
        roll["returns"], roll["advantages"] = ret.float(), adv.float()
        # pack the two fixed-shape slabs
        off = 0
        for k, s in u8_fields:
            m = n * int(np.prod(s))
            u8[off:off + m].copy_(roll[k].reshape(-1).to(torch.uint8))
            off += m
        off = 0
        for k, s in f32_fields:
            m = n * int(np.prod(s))
            f32[off:off + m].copy_(roll[k].reshape(-1).float())
            off += m
        f32[off:off + N_STATS].copy_(torch.tensor(ep, dtype=torch.float32))
        if n_u8:
            dist.gather(u8, None, dst=LEARNER)
        dist.gather(f32, None, dst=LEARNER)
        dist.broadcast(flat, src=LEARNER)
        vector_to_params(flat.to(device), params)
    envs.close()


def _learner(runner, cfg, agent, flat, wire, u8_fields, f32_fields, n_u8, n_f32, num_updates, log_dir) -> None:
    from sheeprl_prey_amd.algos.ppo.ppo import PPOTrainer

    world = runner.world_size
    n_actors = world - 1
    T, ne = int(cfg.algo.rollout_steps), int(cfg.env.num_envs)
    n = T * ne
    device = runner.device
    local = _LocalRunner(runner)
    optimizer = build_optimizer(cfg.algo.optimizer, agent.parameters())
    scheduler = PolynomialLR(optimizer, total_iters=num_updates, power=1.0) if cfg.algo.anneal_lr else None
    trainer = PPOTrainer(local, agent, optimizer, cfg, n * n_actors)
    aggregator = MetricAggregator({k: MeanMetric() for k in ("Rewards/rew_avg", "Game/ep_len_avg", "Loss/value_loss",
                                                            "Loss/policy_loss", "Loss/entropy_loss")})
    u8_all = [torch.empty(max(1, n_u8), dtype=torch.uint8, device=wire) for _ in range(world)]
    f32_all = [torch.empty(n_f32, dtype=torch.float32, device=wire) for _ in range(world)]
    initial_ent, initial_clip = copy.deepcopy(cfg.algo.ent_coef), copy.deepcopy(cfg.algo.clip_coef)
    policy_step = last_log = last_checkpoint = train_step = last_train = 0
    for update in range(1, num_updates + 1):
        if n_u8:
            dist.gather(u8_all[LEARNER], u8_all, dst=LEARNER)
        dist.gather(f32_all[LEARNER], f32_all, dst=LEARNER)
        policy_step += n * n_actors
        parts: Dict[str, List[Tensor]] = {}
        for a in range(1, world):
            fields = _split(u8_all[a], u8_fields, n) if n_u8 else {}
            fields.update(_split(f32_all[a][: n_f32 - N_STATS], f32_fields, n))
            for k, v in fields.items():
                parts.setdefault(k, []).append(v.to(device, non_blocking=True))
            st = f32_all[a][n_f32 - N_STATS:].tolist()
            if st[1] > 0:
                aggregator.update("Rewards/rew_avg", st[0] / st[1])
                aggregator.update("Game/ep_len_avg", st[2] / st[1])
        data = TensorDict({k: (torch.cat(v).float() if k in cfg.cnn_keys.encoder else torch.cat(v))
                           for k, v in parts.items()}, batch_size=[n * n_actors])
        with timer("Time/train_time"):
            trainer(data, aggregator)
        train_step += 1
        flat.copy_(params_to_vector(agent.parameters()).to(wire))
        dist.broadcast(flat, src=LEARNER)
        if scheduler is not None:
            scheduler.step()
        if cfg.algo.anneal_clip_coef:
            cfg.algo.clip_coef = polynomial_decay(update, initial=initial_clip, final=0.0, max_decay_steps=num_updates,
                                                  power=1.0)
        if cfg.algo.anneal_ent_coef:
            cfg.algo.ent_coef = polynomial_decay(update, initial=initial_ent, final=0.0, max_decay_steps=num_updates,
                                                 power=1.0)
        if policy_step - last_log >= cfg.metric.log_every or update == num_updates or cfg.dry_run:
            metrics = aggregator.compute()
            aggregator.reset()
            tm = timer.compute()
            if tm.get("Time/train_time", 0) > 0:
                metrics["Time/sps_train"] = (train_step - last_train) / tm["Time/train_time"]
            timer.reset()
            runner.log_dict(metrics, policy_step)
            last_log, last_train = policy_step, train_step
        if (cfg.checkpoint.every > 0 and policy_step - last_checkpoint >= cfg.checkpoint.every) or cfg.dry_run \
                or update == num_updates:
            last_checkpoint = policy_step
            state = {"agent": agent.state_dict(), "optimizer": optimizer.state_dict(),
                     "scheduler": scheduler.state_dict() if scheduler is not None else None, "update": update,
                     "batch_size": cfg.per_rank_batch_size, "last_log": last_log, "last_checkpoint": last_checkpoint}
            local.call("on_checkpoint_coupled", ckpt_path=os.path.join(log_dir, f"checkpoint/ckpt_{policy_step}_0.ckpt"),
                       state=state)
    test(agent, runner, cfg, log_dir)
