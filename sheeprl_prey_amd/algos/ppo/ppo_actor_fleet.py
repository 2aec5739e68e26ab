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

``algo.weight_lag`` (default 0 = the reference's on-policy order, ``ppo_decoupled.py:36-349``): with
lag L >= 1 an actor does not wait for the weights of the update its rollout feeds - it posts the
broadcast receive asynchronously into a second weight buffer and starts the next rollout at once with
the weights it has (at most L updates old); the learner's update and the broadcast then overlap the
actors' next rollout instead of idling them.

Transport: a rollout is TWO fixed-shape slabs per actor - uint8 (pixel observations, never widened
to fp32 on the wire) and fp32 (vector observations, actions, log-probs, values, returns,
advantages, and three episode statistics) - gathered with ONE ``dist.gather`` each (RCCL over
xGMI on GPUs); the weights come back as ONE flat fp32 ``dist.broadcast``.  Shapes never change, so
no per-update header travels.
"""
from __future__ import annotations

import copy
import os
import time
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
N_STATS = 6  # per actor and update: finished-episode return sum, count, length sum; rollout, gather-wait, broadcast-wait s


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
    # rollout engine: device-resident envs -> the whole rollout as one launch / one graph replay; host envs ->
    # graphed policy step with pinned staging into device [T, ne] buffers (ppo.HostRollout)
    from sheeprl_prey_amd.algos.ppo.ppo import DeviceRollout, FusedCartPoleRollout, HostRollout, PPOPlayer

    graphs = device.type == "cuda" and bool(getattr(runner, "cuda_graphs", False))
    denv = None
    if cfg.env.get("device", False):
        from sheeprl_prey_amd.envs.device import make_device_env

        if device.type != "cuda" or obs_keys != ["state"]:
            raise ValueError("env.device=True needs a GPU run with mlp_keys.encoder=[state] and no cnn keys")
        envs.close()
        denv = make_device_env(cfg.env.id, ne, device, seed=cfg.seed + rank * ne, max_episode_steps=cfg.env.max_episode_steps)
        denv.reset()
        roll_fn = (FusedCartPoleRollout(agent, denv, cfg, seed=cfg.seed + rank) if FusedCartPoleRollout.supported(agent, denv)
                   else DeviceRollout(agent, denv, cfg, enabled=graphs))
    else:
        player = PPOPlayer(agent, cfg, is_continuous, enabled=graphs)
        roll_fn = HostRollout(agent, envs, cfg, player, device, obs_keys, envs.reset(seed=cfg.seed + rank)[0])
    u8 = torch.zeros(max(1, n_u8), dtype=torch.uint8, device=wire)
    f32 = torch.zeros(n_f32, dtype=torch.float32, device=wire)
    # the slabs are packed on the compute device, then moved to the wire device in one copy each
    u8_dev = u8 if wire == device else torch.zeros_like(u8, device=device)
    f32_dev = f32 if wire == device else torch.zeros_like(f32, device=device)
    t_gather = t_bcast = 0.0
    lag = int(cfg.algo.get("weight_lag", 0) or 0)
    # lag >= 1: in-flight weight receives (oldest first), each into its own buffer
    inflight: List[Tuple[Any, Tensor]] = []
    for update in range(1, num_updates + 1):
        t0 = time.perf_counter()
        roll = dict(roll_fn())
        if denv is not None:
            next_obs = {"state": denv.obs}
            rets, lens = roll_fn.finished_episodes()
            ep = [float(sum(rets)), float(len(rets)), float(sum(lens))]
        else:
            next_obs = roll_fn.obs
            ep = [float(sum(r for r, _ in roll_fn.episodes)), float(len(roll_fn.episodes)),
                  float(sum(n_ for _, n_ in roll_fn.episodes))]
        with torch.no_grad():
            nv = agent.get_value(_norm(next_obs, cfg.cnn_keys.encoder, obs_keys))
            ret, adv = gae(roll["rewards"], roll["values"], roll["dones"], nv, T, cfg.algo.gamma, cfg.algo.gae_lambda)
        roll["returns"], roll["advantages"] = ret.float(), adv.float()
        # pack the two fixed-shape slabs (on the device: one copy per field, no host round trip)
        off = 0
        for k, sh in u8_fields:
            m = n * int(np.prod(sh))
            u8_dev[off:off + m].copy_(roll[k].reshape(-1))
            off += m
        off = 0
        for k, sh in f32_fields:
            m = n * int(np.prod(sh))
            f32_dev[off:off + m].copy_(roll[k].reshape(-1))
            off += m
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        t_roll = time.perf_counter() - t0
        # per-actor stats travel with the rollout: episode sums + this actor's rollout / wait seconds
        f32_dev[off:off + N_STATS].copy_(torch.tensor(ep + [t_roll, t_gather, t_bcast], dtype=torch.float32))
        if u8_dev is not u8:
            u8.copy_(u8_dev)
        if f32_dev is not f32:
            f32.copy_(f32_dev)
        t1 = time.perf_counter()
        if n_u8:
            dist.gather(u8, None, dst=LEARNER)
        dist.gather(f32, None, dst=LEARNER)
        t2 = time.perf_counter()
        if lag <= 0:
            dist.broadcast(flat, src=LEARNER)
            vector_to_params(flat.to(device), params)
        else:
            buf = torch.empty_like(flat)
            inflight.append((dist.broadcast(buf, src=LEARNER, async_op=True), buf))
            # keep at most ``lag`` updates in flight: the oldest weights are applied before the next rollout
            while len(inflight) > lag or (update == num_updates and inflight):
                work, got = inflight.pop(0)
                work.wait()
                vector_to_params(got.to(device), params)
        t_gather, t_bcast = t2 - t1, time.perf_counter() - t2
    if denv is None:
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
    # per-update breakdown (seconds, summed between logs): learner gather wait / unpack / update / broadcast,
    # and the actors' own rollout, gather-wait and broadcast-wait times (their means over actors)
    brk = {k: 0.0 for k in ("gather", "unpack", "update", "broadcast", "actor_rollout", "actor_gather_wait",
                            "actor_broadcast_wait")}
    n_brk = 0
    for update in range(1, num_updates + 1):
        t0 = time.perf_counter()
        if n_u8:
            dist.gather(u8_all[LEARNER], u8_all, dst=LEARNER)
        dist.gather(f32_all[LEARNER], f32_all, dst=LEARNER)
        t1 = time.perf_counter()
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
            brk["actor_rollout"] += st[3] / n_actors
            brk["actor_gather_wait"] += st[4] / n_actors
            brk["actor_broadcast_wait"] += st[5] / n_actors
        data = TensorDict({k: (torch.cat(v).float() if k in cfg.cnn_keys.encoder else torch.cat(v))
                           for k, v in parts.items()}, batch_size=[n * n_actors])
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        t2 = time.perf_counter()
        with timer("Time/train_time"):
            trainer(data, aggregator)
        train_step += 1
        flat.copy_(params_to_vector(agent.parameters()).to(wire))
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        t3 = time.perf_counter()
        dist.broadcast(flat, src=LEARNER)
        t4 = time.perf_counter()
        brk["gather"] += t1 - t0
        brk["unpack"] += t2 - t1
        brk["update"] += t3 - t2
        brk["broadcast"] += t4 - t3
        n_brk += 1
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
            if n_brk:
                metrics.update({f"Time/fleet_{k}_ms": 1e3 * v / n_brk for k, v in brk.items()})
                runner.print("actor fleet per update (ms): " + ", ".join(f"{k} {1e3 * v / n_brk:.2f}" for k, v in brk.items()))
                brk = dict.fromkeys(brk, 0.0)
                n_brk = 0
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
