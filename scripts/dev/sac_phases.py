"""Host-side phase timing of the SAC bench loop (bench.py --algo sac): per env step, wall time of act (player
replay + D2H), env step, store (row staging + replay add), sample (+ gather/shard) and train (two graph
replays), each bracketed by a device synchronise so the GPU time of a phase is charged to it.  Usage:
python scripts/dev/sac_phases.py [steps] [overrides...]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    overrides = sys.argv[2:]
    from sheeprl_prey_amd.algos.sac.agent import build_agent
    from sheeprl_prey_amd.algos.sac.sac import SACInteraction, SACTrainer, gather_and_shard, make_aggregator
    from sheeprl_prey_amd.config.compose import compose
    from sheeprl_prey_amd.data.buffers import ReplayBuffer
    from sheeprl_prey_amd.parallel.flat_optim import build_optimizer
    from sheeprl_prey_amd.parallel.runner import Runner
    from sheeprl_prey_amd.utils.env import make_env, make_vector_env
    from sheeprl_prey_amd.utils.utils import dotdict

    cfg = dotdict(compose(["exp=sac", "env=gym", "env.id=walker_walk_synthetic", "mlp_keys.encoder=[state]",
                           "env.sync_env=True", "fabric.accelerator=cuda", "fabric.cuda_graphs=True",
                           "metric.log_every=1000000000", "buffer.size=1000000"] + overrides))
    cfg.pop("hydra", None)
    runner = Runner(**{k: v for k, v in cfg.fabric.items()})
    runner._init_distributed()
    device = runner.device
    runner.seed_everything(cfg.seed)
    ne = cfg.env.num_envs
    envs = make_vector_env(cfg, [make_env(cfg, cfg.seed + i, 0, None, "train", i) for i in range(ne)])
    obs_dim = int(sum(int(np.prod(envs.single_observation_space[k].shape)) for k in cfg.mlp_keys.encoder))
    agent = build_agent(runner, cfg, obs_dim, envs.single_action_space)
    qf = build_optimizer(cfg.algo.critic.optimizer, agent.critic.parameters())
    ao = build_optimizer(cfg.algo.actor.optimizer, agent.actor.parameters())
    al = build_optimizer(cfg.algo.alpha.optimizer, [agent.log_alpha])
    tr = SACTrainer(runner, cfg, agent, ao, qf, al)
    agg = make_aggregator(cfg)
    rb = ReplayBuffer(cfg.buffer.size // ne, ne, device=device)
    loop = SACInteraction(runner, cfg, envs, agent, rb, obs_dim, policy=tr.policy())
    loop.reset(cfg.seed)
    print("fused update:", tr.fused is not None, flush=True)
    names = ["act", "env", "store", "sample", "train"]
    tot = {k: 0.0 for k in names}
    sync = torch.cuda.synchronize
    B = cfg.per_rank_batch_size
    for step in range(steps + 220):
        timed = step >= 220
        random_actions = step < 110
        t0 = time.perf_counter()
        if random_actions:
            actions = envs.action_space.sample()
        else:
            with torch.no_grad():
                actions = loop.player({"obs": loop.obs})["a"].cpu().numpy()
        sync()
        t1 = time.perf_counter()
        next_o, rewards, dones, truncated, infos = envs.step(actions.reshape(envs.action_space.shape))
        loop._last = (actions, next_o, rewards, np.logical_or(dones, truncated), infos)
        t2 = time.perf_counter()
        loop.store()
        sync()
        t3 = time.perf_counter()
        if step >= 100:
            sample = rb.sample(B, sample_next_obs=cfg.buffer.sample_next_obs)
            data = gather_and_shard(runner, sample, cfg).to(device)
            bd = {k: data[k] for k in ("observations", "next_observations", "actions", "rewards", "dones")}
            sync()
            t4 = time.perf_counter()
            tr.train(bd, True, agg)
            sync()
            t5 = time.perf_counter()
        else:
            t4 = t5 = t3
        if timed:
            for k, v in zip(names, (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4)):
                tot[k] += v
    total = sum(tot.values())
    print(f"{steps} steps, {total / steps * 1e3:.3f} ms/step (phases synchronised)")
    for k in names:
        print(f"  {k:7s} {tot[k] / steps * 1e6:8.1f} us")


if __name__ == "__main__":
    main()
