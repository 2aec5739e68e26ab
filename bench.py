"""Headline benchmark: DreamerV3 Atari-100k env-steps/sec on MI355X (BASELINE.json).

Workload = ``exp=dreamer_v3_100k_ms_pacman`` (dense 512, mlp_layers 2, cnn mult 32, deter 512,
hidden 512, stoch 32x32, per-rank batch 16 x seq 64, horizon 15, train_every 1, 1 env per rank),
on the synthetic Atari-shaped env (64x64x3 uint8 frames, MsPacman's 9 actions, frame-skip 4),
random-init weights, fp32 compute (the reference runs ``precision: 32-true``).

One bench step = one policy step of every rank's env (player forward, env step, replay add) +
one full gradient step (world model + actor + critic, Adam updates) - the Atari-100k recipe
(``train_every: 1``, ``per_rank_gradient_steps: 1``).  ``value`` = whole-job env steps/s counted
as BASELINE.md defines it: total policy steps across ranks x action_repeat / wall-clock.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=40)
    p.add_argument("--warmup", type=int, default=8)
    p.add_argument("--prefill", type=int, default=1024, help="random-action steps before training (learning_starts)")
    p.add_argument("--no-graphs", action="store_true")
    p.add_argument("--eager-ops", action="store_true", help="route GPU ops through the eager reference (A/B only)")
    p.add_argument("--profile-steps", type=int, default=0)
    p.add_argument("--phase-times", action="store_true",
                   help="per-phase hipGraphs with event timing (diagnostic; adds syncs, not a bench number)")
    p.add_argument("overrides", nargs="*")
    return p.parse_args()


def main():
    args = parse()
    ws_env = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and ws_env == 1:
        # self-launch one process per GPU
        import subprocess

        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr=127.0.0.1", "--master-port=29517", __file__] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))

    from sheeprl_prey_amd import ops
    from sheeprl_prey_amd.algos.common import action_info
    from sheeprl_prey_amd.algos.dreamer_v3.agent import PlayerDV3, build_models
    from sheeprl_prey_amd.algos.dreamer_v3.dreamer_v3 import DreamerV3Trainer
    from sheeprl_prey_amd.algos.dreamer_v3.utils import Moments
    from sheeprl_prey_amd.config.compose import compose
    from sheeprl_prey_amd.data.buffers import AsyncReplayBuffer
    from sheeprl_prey_amd.data.tensordict import TensorDict
    from sheeprl_prey_amd.parallel.flat_optim import build_optimizer
    from sheeprl_prey_amd.parallel.runner import Runner
    from sheeprl_prey_amd.utils.env import make_env, make_vector_env
    from sheeprl_prey_amd.utils.utils import dotdict

    if args.eager_ops:
        ops.set_fused(False)
    overrides = [
        "exp=dreamer_v3_100k_ms_pacman", "env=synthetic_atari", "env.sync_env=True",
        "cnn_keys.encoder=[rgb]", "cnn_keys.decoder=[rgb]", "fabric.accelerator=cuda",
        f"fabric.cuda_graphs={not args.no_graphs}", "metric.log_every=1000000000",
    ] + list(args.overrides)
    cfg = dotdict(compose(overrides))
    cfg.pop("hydra", None)
    runner = Runner(**{k: v for k, v in cfg.fabric.items()})
    runner._init_distributed()
    rank, world = runner.global_rank, runner.world_size
    device = runner.device
    runner.seed_everything(cfg.seed + rank)

    envs = make_vector_env(cfg, [make_env(cfg, cfg.seed + rank * cfg.env.num_envs + i, rank * cfg.env.num_envs, None,
                                          "train", i) for i in range(cfg.env.num_envs)])
    obs_space, act_space = envs.single_observation_space, envs.single_action_space
    is_continuous, _, actions_dim = action_info(act_space)
    world_model, actor, critic, target_critic = build_models(runner, actions_dim, is_continuous, cfg, obs_space)
    player = PlayerDV3(world_model.encoder, world_model.rssm, actor, actions_dim, cfg.algo.player.expl_amount,
                       cfg.env.num_envs, cfg.algo.world_model.stochastic_size,
                       cfg.algo.world_model.recurrent_model.recurrent_state_size, device,
                       discrete_size=cfg.algo.world_model.discrete_size)
    wopt = build_optimizer(cfg.algo.world_model.optimizer, world_model.parameters())
    aopt = build_optimizer(cfg.algo.actor.optimizer, actor.parameters())
    copt = build_optimizer(cfg.algo.critic.optimizer, critic.parameters())
    moments = Moments(runner, cfg.algo.actor.moments.decay, cfg.algo.actor.moments.max,
                      cfg.algo.actor.moments.percentile.low, cfg.algo.actor.moments.percentile.high).to(device)
    trainer = DreamerV3Trainer(runner, cfg, world_model, actor, critic, target_critic, wopt, aopt, copt, moments,
                               is_continuous, actions_dim, force_segmented=args.phase_times)
    n_params = sum(p.numel() for m in (world_model, actor, critic) for p in m.parameters())
    rb = AsyncReplayBuffer(cfg.buffer.size // (cfg.env.num_envs * world), cfg.env.num_envs, device=device, sequential=True)
    obs_keys = list(cfg.cnn_keys.encoder)
    o = envs.reset(seed=cfg.seed + rank)[0]
    step_data = TensorDict({}, batch_size=[cfg.env.num_envs], device="cpu")
    for k in obs_keys:
        step_data[k] = torch.from_numpy(np.asarray(o[k]))
    step_data["dones"] = torch.zeros(cfg.env.num_envs, 1)
    step_data["rewards"] = torch.zeros(cfg.env.num_envs, 1)
    step_data["is_first"] = torch.ones(cfg.env.num_envs, 1)
    player.init_states()
    obs = {k: step_data[k] for k in obs_keys}

    def env_step(random_actions: bool):
        nonlocal obs
        if random_actions:
            real = np.array(envs.action_space.sample())
            acts = np.concatenate([np.eye(d, dtype=np.float32)[a] for a, d in zip(real.reshape(len(actions_dim), -1), actions_dim)], -1)
        else:
            with torch.no_grad():
                pre = {k: v[None].to(device, non_blocking=True) / 255.0 for k, v in obs.items()}
                a = player.get_exploration_action(pre, is_continuous)
                acts = torch.cat(a, -1).cpu().numpy()
                real = np.array([x.argmax(-1).cpu().numpy() for x in a])
        step_data["actions"] = torch.from_numpy(np.asarray(acts)).view(cfg.env.num_envs, -1).float()
        rb.add(step_data[None, ...])
        o, r, d, tr, infos = envs.step(real.reshape(envs.action_space.shape))
        d = np.logical_or(d, tr)
        step_data["is_first"] = torch.zeros(cfg.env.num_envs, 1)
        for k in obs_keys:
            step_data[k] = torch.from_numpy(np.asarray(o[k]))
        obs = {k: step_data[k] for k in obs_keys}
        step_data["rewards"] = torch.from_numpy(np.asarray(r)).view(-1, 1).float()
        step_data["dones"] = torch.from_numpy(np.asarray(d)).view(-1, 1).float()
        idx = np.nonzero(d)[0].tolist()
        if idx:
            step_data["dones"][idx] = 0.0
            step_data["rewards"][idx] = 0.0
            step_data["is_first"][idx] = 1.0
            player.init_states(idx)

    grad_steps = 0

    def train_once():
        nonlocal grad_steps
        data = rb.sample(cfg.per_rank_batch_size, sequence_length=cfg.per_rank_sequence_length, n_samples=1)
        trainer.update_target(1.0 if grad_steps == 0 else cfg.algo.critic.tau)
        batch = {k: (v[0] if v.dtype == torch.uint8 else v[0].float()) for k, v in data.items()}
        out = trainer.train_step(batch)
        grad_steps += 1
        return out

    for _ in range(max(args.prefill, cfg.per_rank_sequence_length + 1)):
        env_step(True)

    env_ms = [0.0]

    def one_step():
        if args.phase_times:
            torch.cuda.synchronize()
            t = time.perf_counter()
            env_step(False)
            torch.cuda.synchronize()
            env_ms[0] += (time.perf_counter() - t) * 1e3
        else:
            env_step(False)
        return train_once()

    for _ in range(args.warmup):
        out = one_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    if args.phase_times:
        trainer.seg.enable_timing()
    if args.profile_steps:
        torch.cuda._sleep(1000)  # marker kernel: scripts/trace_window.py aggregates the dispatches after it
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = one_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if args.phase_times and rank == 0:
        seg = trainer.seg
        if seg.phase_ms is not None and seg.timed_steps:
            names = DreamerV3Trainer.PHASES
            print(f"player+env ms/step: {env_ms[0] / (args.steps + args.warmup):.3f}; phase ms/step: "
                  + ", ".join(f"{n} {v / seg.timed_steps:.3f}" for n, v in zip(names, seg.phase_ms)),
                  file=sys.stderr, flush=True)
    loss = float(out["Loss/world_model_loss"].item())
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    ms_per_step = elapsed / args.steps * 1e3
    policy_steps = args.steps * cfg.env.num_envs * world
    env_steps_per_s = policy_steps * cfg.env.action_repeat / elapsed
    if rank == 0:
        rec = {
            "metric": "env-steps/sec (whole node) DreamerV3 Atari-100k 64x64",
            "value": round(env_steps_per_s, 3),
            "unit": "env_steps/s (policy steps x action_repeat=4, whole job)",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (Atari-shaped 64x64x3 uint8 env, MsPacman action set; random-init weights)",
            "config": {
                "model": "DreamerV3 Atari-100k (dense 512, mlp 2, cnn mult 32, deter 512, stoch 32x32, bins 255)",
                "global_batch": cfg.per_rank_batch_size * world,
                "seq_len": cfg.per_rank_sequence_length,
                "horizon": cfg.algo.horizon,
                "parallelism": f"dp{world}",
                "params": n_params,
                "hipgraph": bool(trainer.graphed.enabled),
                "fused_ops": ops.fused_enabled(),
            },
            "policy_steps_per_s": round(policy_steps / elapsed, 3),
            "grad_steps_per_s": round(args.steps * world / elapsed, 3),
            "final_wm_loss": round(loss, 4),
        }
        print(json.dumps(rec), flush=True)
    envs.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
