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
    p.add_argument("--algo", default="dreamer_v3", choices=["dreamer_v3", "ppo", "sac"],
                   help="dreamer_v3: the headline DV3 Atari-100k bench; ppo: PPO CartPole-v1 (exp=ppo) steps/sec; "
                        "sac: SAC on a dm_control walker_walk-shaped synthetic env (BASELINE config #3)")
    p.add_argument("--steps", type=int, default=40)
    p.add_argument("--warmup", type=int, default=8)
    p.add_argument("--prefill", type=int, default=1024, help="random-action steps before training (learning_starts)")
    p.add_argument("--no-graphs", action="store_true")
    p.add_argument("--eager-ops", action="store_true", help="route GPU ops through the eager reference (A/B only)")
    p.add_argument("--profile-steps", type=int, default=0)
    p.add_argument("--pixel", action="store_true",
                   help="--algo ppo: 84x84 grayscale 4-frame Atari-shaped pixel PPO (NatureCNN) on a synthetic env")
    p.add_argument("--device-env", action="store_true",
                   help="--algo ppo: step CartPole-v1 on the GPU (envs/device.py) and capture the whole rollout")
    p.add_argument("--no-fused-rollout", action="store_true",
                   help="PPO --device-env: graph-captured per-op rollout instead of the one-launch kernel")
    p.add_argument("--torch-profile", type=int, default=0,
                   help="DV3: run N extra eager steps under torch.profiler and print the aten op table (stderr)")
    p.add_argument("--phase-times", action="store_true",
                   help="per-phase hipGraphs with event timing (diagnostic; adds syncs, not a bench number)")
    p.add_argument("--segmented", action="store_true",
                   help="use the multi-rank graph mode (one hipGraph per phase, collectives between replays) "
                        "on any N, to price it against the single-graph step at N=1")
    p.add_argument("--pg-timeout", type=float, default=300.0,
                   help="process-group timeout and host heartbeat (seconds): a stalled rank exits non-zero")
    p.add_argument("--check-finite", type=int, default=0,
                   help="diagnostic: run N untimed steps, report the first non-finite train output per step")
    p.add_argument("--gemm-tuning", default=None, choices=["use", "tune", "off"],
                   help="library-GEMM TunableOp mode (default: fabric.tunable_gemm = use the committed results)")
    p.add_argument("--xl", action="store_true",
                   help="dreamer_v3: the XL model of exp=dreamer_v3_XL_crafter (dense 1024, mlp 5, cnn mult 96, "
                        "deter 4096, hidden 1024) on the synthetic 64x64 env")
    p.add_argument("--continuous", action="store_true",
                   help="dreamer_v3: exp=dreamer_v3_dmc_walker_walk (continuous 6-dim actions, TruncatedNormal actor, "
                        "64x64 pixels + 24-dim state, train_every 2) on the walker_walk-shaped synthetic env")
    p.add_argument("overrides", nargs="*")
    return p.parse_args()


# model dimensions of the reference's configs/exp/dreamer_v3_XL_crafter.yaml:35-47
XL_OVERRIDES = [
    "algo.dense_units=1024", "algo.mlp_layers=5", "algo.world_model.encoder.cnn_channels_multiplier=96",
    "algo.world_model.recurrent_model.recurrent_state_size=4096", "algo.world_model.transition_model.hidden_size=1024",
    "algo.world_model.representation_model.hidden_size=1024",
]


def main():
    args = parse()
    ws_env = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and ws_env == 1:
        # self-launch one process per GPU
        import subprocess

        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr=127.0.0.1", "--master-port=29517", __file__] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))
    if args.algo == "ppo":
        return bench_ppo(args)
    if args.algo == "sac":
        return bench_sac(args)

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

    if args.continuous:
        # reference configs/exp/dreamer_v3_dmc_walker_walk.yaml on the walker_walk-shaped synthetic env
        base = ["exp=dreamer_v3_dmc_walker_walk", "env=gym", "env.id=walker_walk_synthetic", "env.sync_env=True",
                "cnn_keys.encoder=[rgb]", "cnn_keys.decoder=[rgb]", "mlp_keys.encoder=[state]", "mlp_keys.decoder=[state]",
                "buffer.memmap=False", "checkpoint.every=1000000000"]
    else:
        base = ["exp=dreamer_v3_100k_ms_pacman", "env=synthetic_atari", "env.sync_env=True",
                "cnn_keys.encoder=[rgb]", "cnn_keys.decoder=[rgb]"]
    overrides = base + [
        "fabric.accelerator=cuda", f"fabric.cuda_graphs={not args.no_graphs}", "metric.log_every=1000000000",
        f"fabric.fused_ops={not args.eager_ops}",
        f"fabric.pg_timeout_s={args.pg_timeout}",
    ] + ([f"fabric.tunable_gemm={args.gemm_tuning}"] if args.gemm_tuning else []) + (XL_OVERRIDES if args.xl else []) + list(
        args.overrides)
    cfg = dotdict(compose(overrides))
    cfg.pop("hydra", None)
    runner = Runner(**{k: v for k, v in cfg.fabric.items()})
    runner._init_distributed()
    rank, world = runner.global_rank, runner.world_size
    device = runner.device
    runner.seed_everything(cfg.seed + rank)
    from sheeprl_prey_amd.parallel.collectives import CollectiveLog, Heartbeat

    heart = Heartbeat(args.pg_timeout if world > 1 else 0, "init")
    rccl_ranks = formed_ranks(runner)

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
                               is_continuous, actions_dim, force_segmented=args.phase_times or args.segmented)
    n_params = sum(p.numel() for m in (world_model, actor, critic) for p in m.parameters())
    rb = AsyncReplayBuffer(cfg.buffer.size // (cfg.env.num_envs * world), cfg.env.num_envs, device=device, sequential=True)
    # the env-interaction step of dreamer_v3.main itself (interaction.py): pinned staging ring, H2D on
    # a side stream, the player graph, the replay add and the train-graph launch enqueued back to back,
    # the host waits only for the action readback and steps the env while the GPU trains
    from sheeprl_prey_amd.algos.dreamer_v3.interaction import InteractionLoop

    loop = InteractionLoop(runner, cfg, envs, player, rb, actions_dim, is_continuous)
    player.use_graphs = runner.cuda_graphs and os.environ.get("SRL_PLAYER_GRAPH", "1") != "0"
    loop.reset(cfg.seed + rank)

    grad_steps = 0
    last_batch = [None]
    unsampled = [False]  # profile passes: the eager train step (graphs off) instead of the captured sampled replay

    def train_once():
        nonlocal grad_steps
        trainer.update_target(1.0 if grad_steps == 0 else cfg.algo.critic.tau)
        if not args.eager_ops and not args.check_finite and not unsampled[0]:
            # captured step: the sample is drawn into the graph's inputs by one launch (dreamer_v3.main does the same)
            out = trainer.train_step_sampled(rb, cfg.per_rank_batch_size, cfg.per_rank_sequence_length)
            if out is not None:
                grad_steps += 1
                return out
        data = rb.sample(cfg.per_rank_batch_size, sequence_length=cfg.per_rank_sequence_length, n_samples=1)
        batch = {k: (v[0] if v.dtype == torch.uint8 else v[0].float()) for k, v in data.items()}
        last_batch[0] = batch
        out = trainer.train_step(batch)
        grad_steps += 1
        return out

    for _ in range(max(args.prefill, cfg.per_rank_sequence_length + 1)):
        loop.step(True)

    env_ms = [0.0]

    # one bench step = train_every policy steps of every rank's env + the gradient steps they trigger
    # (the Atari-100k recipe: train_every 1; the DMC walker recipe: train_every 2)
    policy_per_step = max(1, int(cfg.algo.train_every) // (cfg.env.num_envs * world))

    def one_step():
        # act (weights W_t) -> store the row -> launch the gradient step (W_t -> W_t+1) -> env step on
        # the CPU while the GPU trains.  --phase-times times the serial form of the same step.
        for _ in range(policy_per_step - 1):
            loop.step(False, None)
        if args.phase_times:
            loop.pipelined = False
            torch.cuda.synchronize()
            t = time.perf_counter()
            loop.step(False, None)
            torch.cuda.synchronize()
            env_ms[0] += (time.perf_counter() - t) * 1e3
            return train_once()
        loop.step(False, train_once)
        return loop.last_train_out

    # the collectives every phase of one step issues (recorded on the second warm-up step: the first one
    # also enables the hook-launched buckets)
    clog = CollectiveLog()
    if args.check_finite:
        check_finite_steps(args, trainer, rb, cfg, one_step, lambda: trainer.train_step(last_batch[0]), (world_model, actor, critic),
                           (wopt, aopt, copt), moments)
    with clog:
        for i in range(args.warmup):
            out = one_step()
            heart.beat(f"warmup step {i}")
    torch.cuda.synchronize()
    heart.beat("warmup done")
    if args.torch_profile:
        heart.grace("rank-0 torch profile")
    if args.torch_profile and rank == 0:
        # op attribution of the small kernels: the same train step run eagerly (graphs off) under
        # torch.profiler; a graph replay dispatches the very same kernels
        from torch.profiler import ProfilerActivity, profile

        trainer.graphed.enabled = False
        unsampled[0] = True
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True,
                     record_shapes=bool(os.environ.get("SRL_PROFILE_SHAPES"))) as prof:
            for _ in range(args.torch_profile):
                one_step()
            torch.cuda.synchronize()
        if os.environ.get("SRL_PROFILE_SITES"):
            # every ATen op of one eager step with its framework call site (innermost frame in the package)
            import collections
            import traceback

            from torch.utils._python_dispatch import TorchDispatchMode

            skip = {"detach", "view", "_unsafe_view", "reshape", "t", "transpose", "permute", "select", "slice", "unsqueeze",
                    "squeeze", "expand", "as_strided", "alias", "split", "split_with_sizes", "unbind", "lift_fresh", "empty",
                    "empty_like", "empty_strided", "is_same_size", "_local_scalar_dense",
                    "mm", "addmm", "bmm", "baddbmm", "convolution", "miopen_convolution", "record_stream", "set_",
                    "new_empty", "new_empty_strided", "resize_", "_has_compatible_shallow_copy_type", "numpy_T"}

            gemm_mode = os.environ.get("SRL_PROFILE_SITES") == "gemm"

            class _Sites(TorchDispatchMode):
                def __init__(self):
                    super().__init__()
                    self.c = collections.Counter()

                def __torch_dispatch__(self, func, types, args=(), kwargs=None):
                    name = func.overloadpacket.__name__
                    if gemm_mode:  # SRL_PROFILE_SITES=gemm: library GEMM calls by site, operand shapes and strides
                        if name in ("mm", "addmm", "addmm_", "bmm", "baddbmm"):
                            fr = [f for f in traceback.extract_stack()[:-1] if "sheeprl_prey_amd" in f.filename]
                            site = f"{fr[-1].filename.split('sheeprl_prey_amd/')[-1]}:{fr[-1].lineno}" if fr else "<autograd>"
                            ops_ = ";".join(f"{tuple(a.shape)}/{a.stride()}" for a in args if isinstance(a, torch.Tensor))
                            self.c[(name, f"{site} {ops_}")] += 1
                    elif name not in skip:
                        fr = [f for f in traceback.extract_stack()[:-1] if "sheeprl_prey_amd" in f.filename]
                        site = f"{fr[-1].filename.split('sheeprl_prey_amd/')[-1]}:{fr[-1].lineno}" if fr else "<autograd>"
                        self.c[(name, site)] += 1
                    return func(*args, **(kwargs or {}))

            trainer.graphed.enabled = False
            with _Sites() as sm:
                one_step()
            torch.cuda.synchronize()
            for (name, site), n in sm.c.most_common(int(os.environ.get("SRL_PROFILE_TOP", 60))):
                print(f"SITE {n:4d} {name:10s} {site}", file=sys.stderr, flush=True)
        trainer.graphed.enabled = True
        unsampled[0] = False
        small = ("aten::cat", "aten::copy_", "aten::fill_", "aten::zero_", "aten::add", "aten::add_", "aten::sum",
                 "aten::mean", "aten::mul", "aten::sub", "aten::rand", "aten::zeros", "aten::clone", "aten::div",
                 "aten::neg", "aten::exp", "aten::where", "aten::stack", "aten::contiguous", "aten::index_select",
                 "aten::lerp_", "aten::_foreach_copy_", "aten::max", "aten::amax", "aten::sort", "aten::quantile")
        big = ("aten::mm", "aten::addmm", "aten::bmm", "aten::baddbmm", "aten::linear", "aten::matmul", "aten::convolution",
               "aten::_convolution", "aten::miopen_convolution", "aten::conv2d", "aten::conv_transpose2d")
        rows = [e for e in prof.key_averages(group_by_stack_n=5)
                if e.key in small or (os.environ.get("SRL_PROFILE_ALL") and e.key.startswith("aten::") and e.key not in big
                                      and getattr(e, "self_device_time_total", 0) > 0)]
        if os.environ.get("SRL_PROFILE_SHAPES"):  # library GEMMs by operand shapes, device time per call
            for e in sorted((e for e in prof.key_averages(group_by_input_shape=True) if e.key in big),
                            key=lambda e: -getattr(e, "device_time_total", 0))[:40]:
                print(f"GEMM {e.key:12s} n={e.count / args.torch_profile:5.1f}/step "
                      f"{getattr(e, 'device_time_total', 0) / max(e.count, 1):8.1f} us/call  {e.input_shapes}",
                      file=sys.stderr, flush=True)
        rows.sort(key=lambda e: -e.count)
        for e in rows[:int(os.environ.get('SRL_PROFILE_TOP', 60))]:
            stack = " <- ".join(f.split("/")[-1] for f in e.stack[:5])
            print(f"{e.key:24s} n={e.count / args.torch_profile:6.1f}/step  {stack}", file=sys.stderr, flush=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    heart.beat("pre-timed barrier")
    if args.phase_times:
        trainer.seg.enable_timing()
    if args.profile_steps:
        torch.cuda._sleep(1000)  # marker kernel: scripts/trace_window.py aggregates the dispatches after it
        torch.cuda.synchronize()
    if os.environ.get("SRL_HOST_TIMES"):
        loop.host_ms = {}  # host-side breakdown of the interaction step (interaction.py)
    t0 = time.perf_counter()
    for i in range(args.steps):
        out = one_step()
        heart.beat(f"timed step {i}")
    torch.cuda.synchronize()
    if loop.host_ms and rank == 0:
        n = max(1, loop.host_ms.pop("steps", 1))
        print("host ms/step: " + ", ".join(f"{k} {v / n:.3f}" for k, v in loop.host_ms.items()), file=sys.stderr, flush=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # loud failure if any persistent-scan hand-off of the run timed out (outside the timed region)
    from sheeprl_prey_amd.ops.rssm import check_scan_health

    check_scan_health()
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
    # data-parallel consistency: every rank must hold the same weights after the timed steps
    spread = 0.0
    if world > 1:
        cs = torch.stack([o.flat_param.double().sum() for o in (wopt, aopt, copt)])
        lo, hi = cs.clone(), cs.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        spread = float((hi - lo).abs().max().item())
    ms_per_step = elapsed / args.steps * 1e3
    policy_steps = args.steps * policy_per_step * cfg.env.num_envs * world
    env_steps_per_s = policy_steps * cfg.env.action_repeat / elapsed
    if rank == 0:
        rec = {
            "metric": ("env-steps/sec (whole node) DreamerV3-XL 64x64" if args.xl
                       else "env-steps/sec (whole node) DreamerV3 DMC walker_walk 64x64 (continuous)" if args.continuous
                       else "env-steps/sec (whole node) DreamerV3 Atari-100k 64x64"),
            "value": round(env_steps_per_s, 3),
            "unit": f"env_steps/s (policy steps x action_repeat={cfg.env.action_repeat}, whole job)",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": ("synthetic walker_walk-shaped env (64x64x3 uint8 render + 24-dim state, 6-dim continuous action; "
                     "random-init weights)" if args.continuous else
                     "synthetic (Atari-shaped 64x64x3 uint8 env, MsPacman action set; random-init weights)"),
            "config": {
                "model": ("DreamerV3-XL (dense 1024, mlp 5, cnn mult 96, deter 4096, hidden 1024, stoch 32x32, bins 255)"
                          if args.xl else
                          "DreamerV3 DMC walker (dense 512, mlp 2, cnn mult 32, deter 512, stoch 32x32, TruncatedNormal actor, "
                          "train_every 2)" if args.continuous else
                          "DreamerV3 Atari-100k (dense 512, mlp 2, cnn mult 32, deter 512, stoch 32x32, bins 255)"),
                "global_batch": cfg.per_rank_batch_size * world,
                "seq_len": cfg.per_rank_sequence_length,
                "horizon": cfg.algo.horizon,
                "parallelism": f"dp{world}",
                "params": n_params,
                "hipgraph": bool(trainer.uses_graphs), "graph_mode": trainer.graph_mode,
                "fused_ops": ops.fused_enabled(),
            },
            "backend": runner.backend if world > 1 else None,
            "rccl_ranks": rccl_ranks,
            "collectives_per_step": clog.per_phase(min(2, clog.step)) if world > 1 else {},
            "policy_steps_per_s": round(policy_steps / elapsed, 3),
            "grad_steps_per_s": round(args.steps * world / elapsed, 3),
            "final_wm_loss": round(loss, 4),
            "dp_param_spread": spread,
        }
        print(json.dumps(rec), flush=True)
    envs.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    heart.stop()


def formed_ranks(runner) -> int:
    """How many ranks the process group actually formed: an all-reduce of ones right after init."""
    if runner.world_size <= 1:
        return 1
    dev = runner.device if runner.backend == "nccl" else torch.device("cpu")
    t = torch.ones(1, device=dev)
    dist.all_reduce(t)
    return int(t.item())


def check_finite_steps(args, trainer, rb, cfg, one_step, train_once, models, opts, moments):
    """Diagnostic (``--check-finite N``): runs N untimed bench steps; before each one snapshots every
    optimiser slab/state, the target critic and Moments.  At the first step with a non-finite output it
    names the parameters whose gradients are non-finite, then restores the snapshot and re-runs a
    gradient step eagerly (graphs off) to tell a capture bug from a numerics bug."""
    names = {}
    for m in models:
        for n, p in m.named_parameters():
            names[id(p)] = n

    def state():
        t = {}
        for j, o in enumerate(opts):
            for k, v in vars(o).items():
                if torch.is_tensor(v):
                    t[(j, k)] = v
        t[("tgt", "flat")] = trainer.target_flat
        t[("mom", "low")], t[("mom", "high")] = moments.low, moments.high
        return t

    for i in range(args.check_finite):
        snap = {k: v.detach().clone() for k, v in state().items()}
        rng = torch.cuda.get_rng_state()
        out = one_step()
        bad = [k for k, v in out.items() if torch.is_tensor(v) and not bool(torch.isfinite(v).all())]
        vals = {k: round(float(v.float().mean()), 4) for k, v in out.items() if torch.is_tensor(v) and k.startswith("Loss/")}
        print(f"check step {i}: non-finite={bad} {vals}", file=sys.stderr, flush=True)
        if not bad:
            continue
        def report(tag):
            for j, o in enumerate(opts):
                stats = []
                for p, off in zip(o.params, o.offsets):
                    g = o.flat_grad[off:off + p.numel()]
                    stats.append((float(g.abs().max()), float(g.double().pow(2).sum()), names.get(id(p), "?")))
                nf = [n for m, _, n in stats if not m == m or m == float("inf")]
                top = sorted(stats, key=lambda x: -x[0] if x[0] == x[0] else -float("inf"))[:6]
                pad = sum(float(o.flat_grad[off + p.numel():(o.offsets[i + 1] if i + 1 < len(o.offsets) else o.numel)].abs().sum())
                          for i, (p, off) in enumerate(zip(o.params, o.offsets)))
                print(f"  [{tag}] opt{j}: scalars={o.scalars.tolist()} non-finite={nf[:6]} pad_abs_sum={pad:.3g} "
                      f"sumsq={sum(x[1] for x in stats):.4g} top={[(n, f'{m:.3g}') for m, _, n in top]}",
                      file=sys.stderr, flush=True)

        report("graphed")
        for k, v in state().items():
            v.copy_(snap[k])
        torch.cuda.set_rng_state(rng)
        trainer.graphed.enabled = False
        out2 = train_once()
        torch.cuda.synchronize()
        bad2 = [k for k, v in out2.items() if torch.is_tensor(v) and not bool(torch.isfinite(v).all())]
        print(f"  eager re-run from the snapshot (same batch): non-finite={bad2}", file=sys.stderr, flush=True)
        report("eager")
        for k, v in state().items():
            v.copy_(snap[k])
        trainer.graphed.enabled = True
        out3 = train_once()
        torch.cuda.synchronize()
        bad3 = [k for k, v in out3.items() if torch.is_tensor(v) and not bool(torch.isfinite(v).all())]
        print(f"  graphed re-run from the snapshot (same batch): non-finite={bad3}", file=sys.stderr, flush=True)
        report("graphed again")
        raise SystemExit(3)


def bench_ppo(args):
    """PPO coupled on CartPole-v1 (``exp=ppo``: 1 env per rank, rollout 128, 10 epochs, minibatch 64,
    64-unit tanh MLPs).  One bench step = one PPO update: the 128-step rollout (policy forward +
    env step + buffer add, per env step), GAE and the full update_epochs x minibatch optimisation.
    value = whole-job policy steps/s."""
    from sheeprl_prey_amd.algos.common import action_info
    from sheeprl_prey_amd.algos.ppo.agent import PPOAgent
    from sheeprl_prey_amd.algos.ppo.ppo import PPOPlayer, PPOTrainer
    from sheeprl_prey_amd.config.compose import compose
    from sheeprl_prey_amd.data.tensordict import TensorDict
    from sheeprl_prey_amd.parallel.flat_optim import build_optimizer
    from sheeprl_prey_amd.parallel.runner import Runner
    from sheeprl_prey_amd.utils.env import make_env, make_vector_env
    from sheeprl_prey_amd.utils.utils import dotdict, gae

    if args.pixel:
        # Atari-shaped pixel PPO (BASELINE config #2 shape): 84x84 grayscale, 4 stacked frames, Pong action
        # set, NatureCNN encoder; cleanrl-style Atari schedule (8 envs x 128 steps, 4 epochs, minibatch 256)
        obs_over = ["env=synthetic_atari", "env.id=PongNoFrameskip-v4", "env.screen_size=84", "env.grayscale=True",
                    "env.frame_stack=4", "cnn_keys.encoder=[rgb]", "mlp_keys.encoder=[]", "env.num_envs=8",
                    "algo.update_epochs=4", "per_rank_batch_size=256"]
    else:
        obs_over = ["mlp_keys.encoder=[state]"]
    overrides = ["exp=ppo"] + obs_over + ["env.sync_env=True", "fabric.accelerator=cuda",
                                          f"fabric.cuda_graphs={not args.no_graphs}",
                                          "metric.log_every=1000000000"] + list(args.overrides)
    cfg = dotdict(compose(overrides))
    cfg.pop("hydra", None)
    runner = Runner(**{k: v for k, v in cfg.fabric.items()})
    runner._init_distributed()
    rank, world = runner.global_rank, runner.world_size
    device = runner.device
    runner.seed_everything(cfg.seed + rank)
    ne = cfg.env.num_envs
    envs = make_vector_env(cfg, [make_env(cfg, cfg.seed + rank * ne + i, rank * ne, None, "train", i) for i in range(ne)])
    obs_space = envs.single_observation_space
    is_continuous, _, actions_dim = action_info(envs.single_action_space)
    obs_keys = list(cfg.cnn_keys.encoder) + list(cfg.mlp_keys.encoder)
    agent = runner.setup_module(PPOAgent(actions_dim, obs_space, cfg.algo.encoder, cfg.algo.actor, cfg.algo.critic,
                                         cfg.cnn_keys.encoder, cfg.mlp_keys.encoder, cfg.env.screen_size,
                                         cfg.distribution, is_continuous))
    optimizer = build_optimizer(cfg.algo.optimizer, agent.parameters())
    player = PPOPlayer(agent, cfg, is_continuous, enabled=runner.cuda_graphs)
    T = cfg.algo.rollout_steps
    trainer = PPOTrainer(runner, agent, optimizer, cfg, T * ne, force_segmented=args.segmented)
    # the CLI's host-env rollout engine (ppo.HostRollout: graphed policy step, pinned staging, device buffers;
    # image frames stay uint8)
    from sheeprl_prey_amd.algos.ppo.ppo import HostRollout

    cnn_keys = set(cfg.cnn_keys.encoder)
    returns_seen = []
    hroll = None if args.device_env else HostRollout(agent, envs, cfg, player, device, obs_keys,
                                                     envs.reset(seed=cfg.seed + rank)[0])

    def update():
        data = dict(hroll())
        returns_seen.extend(r for r, _ in hroll.episodes)
        with torch.no_grad():
            nv = agent.get_value({k: (hroll.obs[k] / 255 - 0.5 if k in cnn_keys else hroll.obs[k]) for k in obs_keys})
            ret, adv = gae(data["rewards"], data["values"], data["dones"], nv, T, cfg.algo.gamma, cfg.algo.gae_lambda)
        data["returns"], data["advantages"] = ret.float(), adv.float()
        trainer(TensorDict({k: v.reshape(T * ne, *v.shape[2:]) for k, v in data.items()}, batch_size=[T * ne]), None)

    if args.device_env:
        from sheeprl_prey_amd.algos.ppo.ppo import DeviceRollout, FusedCartPoleRollout
        from sheeprl_prey_amd.envs.device import make_device_env

        denv = make_device_env(cfg.env.id, ne, device, seed=cfg.seed + rank)
        denv.reset()
        if FusedCartPoleRollout.supported(agent, denv) and not args.no_fused_rollout:
            drollout = FusedCartPoleRollout(agent, denv, cfg, seed=cfg.seed + rank)
        else:
            drollout = DeviceRollout(agent, denv, cfg, enabled=runner.cuda_graphs)

        def update():  # noqa: F811  (device-env variant of the update above)
            buf = drollout()
            with torch.no_grad():
                nv = agent.get_value({"state": denv.obs})
                ret, adv = gae(buf["rewards"], buf["values"], buf["dones"], nv, T, cfg.algo.gamma, cfg.algo.gae_lambda)
            data = dict(buf)
            data["returns"], data["advantages"] = ret.float(), adv.float()
            trainer(TensorDict({k: v.reshape(T * ne, *v.shape[2:]) for k, v in data.items()}, batch_size=[T * ne]), None)
            rets, _ = drollout.finished_episodes()
            returns_seen.extend(rets)

    for _ in range(args.warmup):
        update()
    torch.cuda.synchronize()
    if args.profile_steps:
        torch.cuda._sleep(1000)  # marker kernel for scripts/trace_window.py
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        update()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    spread = 0.0  # data-parallel consistency: every rank must hold the same weights
    if world > 1:
        cs = optimizer.flat_param.double().sum().reshape(1)
        lo, hi = cs.clone(), cs.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        spread = float((hi - lo).abs().max().item())
    policy_steps = args.steps * cfg.algo.rollout_steps * ne * world
    if rank == 0:
        rec = {
            "metric": ("PPO Atari-shaped 84x84 pixel policy steps/sec (whole node)" if args.pixel
                       else "PPO CartPole-v1 policy steps/sec (whole node)"),
            "value": round(policy_steps / elapsed, 3),
            "unit": "policy_steps/s (whole job)",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": ("synthetic 84x84 grayscale sprites, 4 stacked frames, Pong action set (envs/synthetic.py), random-init weights"
                     if args.pixel else
                     "CartPole-v1 dynamics stepped on the GPU (envs/device.py), random-init weights" if args.device_env
                     else "CartPole-v1 dynamics (native host env), random-init weights"),
            "config": {"model": ("PPO NatureCNN 8s4/4s2/3s1 + fc512 encoder, 2x64 tanh heads" if args.pixel
                                 else "PPO MLP 2x64 tanh (exp=ppo)"), "global_batch": cfg.per_rank_batch_size * world,
                       "rollout_steps": cfg.algo.rollout_steps, "num_envs_per_rank": ne,
                       "update_epochs": cfg.algo.update_epochs, "parallelism": f"dp{world}",
                       "hipgraph": trainer.mode != "eager", "update_mode": trainer.mode, "device_env": bool(args.device_env),
                       "rollout": type(drollout).__name__ if args.device_env else "host"},
            "mean_episode_return": round(float(np.mean(returns_seen[-20:])), 2) if returns_seen else None,
            "dp_param_spread": spread,
        }
        print(json.dumps(rec), flush=True)
    envs.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def bench_sac(args):
    """SAC coupled (``exp=sac``: per-rank batch 256, 2 critics, hidden 256, 1 gradient step per env step,
    target EMA every step) on ``walker_walk_synthetic``: dm_control walker_walk's 24-dim state and 6-dim
    action (BASELINE config #3).  One bench step = one env step of every rank (actor forward, env step,
    replay add) + one full SAC gradient step (replay sample, all-gather + re-shard across ranks, twin-Q
    critic update + target EMA, actor + alpha update) - the loop of ``sac.main`` (``SACInteraction`` +
    ``sac_train_update``).  value = whole-job env steps/s."""
    from sheeprl_prey_amd.algos.sac.agent import build_agent
    from sheeprl_prey_amd.algos.sac.sac import SACInteraction, SACTrainer, make_aggregator, sac_train_update
    from sheeprl_prey_amd.config.compose import compose
    from sheeprl_prey_amd.data.buffers import ReplayBuffer
    from sheeprl_prey_amd.parallel.flat_optim import build_optimizer
    from sheeprl_prey_amd.parallel.runner import Runner
    from sheeprl_prey_amd.utils.env import make_env, make_vector_env
    from sheeprl_prey_amd.utils.utils import dotdict

    overrides = ["exp=sac", "env=gym", "env.id=walker_walk_synthetic", "mlp_keys.encoder=[state]", "env.sync_env=True",
                 "fabric.accelerator=cuda", f"fabric.cuda_graphs={not args.no_graphs}", "metric.log_every=1000000000",
                 "buffer.size=1000000"] + list(args.overrides)
    cfg = dotdict(compose(overrides))
    cfg.pop("hydra", None)
    runner = Runner(**{k: v for k, v in cfg.fabric.items()})
    runner._init_distributed()
    rank, world = runner.global_rank, runner.world_size
    device = runner.device
    runner.seed_everything(cfg.seed + rank)
    ne = cfg.env.num_envs
    envs = make_vector_env(cfg, [make_env(cfg, cfg.seed + rank * ne + i, rank * ne, None, "train", i) for i in range(ne)])
    obs_space = envs.single_observation_space
    obs_dim = int(sum(int(np.prod(obs_space[k].shape)) for k in cfg.mlp_keys.encoder))
    agent = build_agent(runner, cfg, obs_dim, envs.single_action_space)
    qf_opt = build_optimizer(cfg.algo.critic.optimizer, agent.critic.parameters())
    actor_opt = build_optimizer(cfg.algo.actor.optimizer, agent.actor.parameters())
    alpha_opt = build_optimizer(cfg.algo.alpha.optimizer, [agent.log_alpha])
    trainer = SACTrainer(runner, cfg, agent, actor_opt, qf_opt, alpha_opt)
    aggregator = make_aggregator(cfg)
    rb = ReplayBuffer(cfg.buffer.size // (ne * world), ne, device=device)
    loop = SACInteraction(runner, cfg, envs, agent, rb, obs_dim, policy=trainer.policy())
    loop.reset(cfg.seed + rank)
    learning_starts = max(int(cfg.algo.learning_starts) // (ne * world), 1)
    ema_every = cfg.algo.critic.target_network_frequency // (ne * world) + 1
    update = [0]
    sync = torch.cuda.synchronize if device.type == "cuda" else (lambda: None)

    def one_step():
        update[0] += 1
        loop.act_and_step(update[0] <= learning_starts)
        loop.store()
        sac_train_update(trainer, runner, cfg, rb, update[0], learning_starts, ema_every, aggregator)

    for _ in range(max(args.prefill, learning_starts + 1)):
        one_step()
    for _ in range(args.warmup):
        one_step()
    sync()
    if args.profile_steps and device.type == "cuda":
        torch.cuda._sleep(1000)  # marker kernel for scripts/trace_window.py
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    spread = 0.0
    if world > 1:
        cs = torch.stack([o.flat_param.double().sum() for o in (qf_opt, actor_opt, alpha_opt)])
        lo, hi = cs.clone(), cs.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        spread = float((hi - lo).abs().max().item())
    env_steps = args.steps * ne * world * cfg.env.action_repeat
    if rank == 0:
        print(json.dumps({
            "metric": "SAC walker_walk-shaped env-steps/sec (whole node)",
            "value": round(env_steps / elapsed, 3),
            "unit": "env_steps/s (policy steps x action_repeat, whole job)",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
            "data": "synthetic walker_walk-shaped control env (24-dim state, 6-dim action; envs/synthetic.py), random-init weights",
            "config": {"model": "SAC actor 2x256 + 2 critics 2x256 (exp=sac)", "global_batch": cfg.per_rank_batch_size * world,
                       "num_envs_per_rank": ne, "gradient_steps_per_env_step": cfg.algo.per_rank_gradient_steps,
                       "parallelism": f"dp{world}", "update_mode": trainer.critic_step.mode,
                       "fused_update": trainer.fused is not None},
            "dp_param_spread": spread,
        }), flush=True)
    envs.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
    if os.environ.get("SRL_DUMP_MAPS"):  # diagnostic: attribute native frames of a crash at exit
        with open("/proc/self/maps") as f, open(os.environ["SRL_DUMP_MAPS"], "w") as o:
            o.write(f.read())
