"""The DreamerV3 player graph replayed right behind the captured train step (the bench's per-step GPU order) vs alone:
GPU time of the player replay (events around it, median of 30) per variant, to locate the gaps the bench step trace
shows inside the player when it follows the train graph (profiles/r5_interaction_idle.md).

    python scripts/player_after_train.py
variants: alone (device idle before the player), after-train (enqueued right behind the train graph), after-train +
host sync (the train graph drained first), after-train + a 50 us spin kernel between (the train graph's tail retired)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from sheeprl_prey_amd.algos.dreamer_v3.agent import PlayerDV3, build_models
    from sheeprl_prey_amd.algos.dreamer_v3.dreamer_v3 import DreamerV3Trainer
    from sheeprl_prey_amd.algos.dreamer_v3.utils import Moments
    from sheeprl_prey_amd.config.compose import compose
    from sheeprl_prey_amd.envs import spaces
    from sheeprl_prey_amd.parallel.flat_optim import build_optimizer
    from sheeprl_prey_amd.parallel.runner import Runner
    from sheeprl_prey_amd.utils.utils import dotdict

    cfg = dotdict(compose(["exp=dreamer_v3_100k_ms_pacman", "env=synthetic_atari", "cnn_keys.encoder=[rgb]",
                           "cnn_keys.decoder=[rgb]", "fabric.accelerator=cuda", "fabric.cuda_graphs=True"]))
    runner = Runner(**dict(cfg.fabric))
    runner._init_distributed()
    torch.manual_seed(0)
    A = 9
    obs_space = spaces.Dict({"rgb": spaces.Box(0, 255, (3, 64, 64), "uint8")})
    wm, actor, critic, target = build_models(runner, [A], False, cfg, obs_space)
    opts = [build_optimizer(c, m.parameters()) for c, m in
            ((cfg.algo.world_model.optimizer, wm), (cfg.algo.actor.optimizer, actor), (cfg.algo.critic.optimizer, critic))]
    tr = DreamerV3Trainer(runner, cfg, wm, actor, critic, target, *opts, Moments(None).cuda(), False, [A])
    T, B = cfg.per_rank_sequence_length, cfg.per_rank_batch_size
    g = torch.Generator(device="cuda").manual_seed(1)
    data = {
        "rgb": torch.randint(0, 255, (T, B, 3, 64, 64), dtype=torch.uint8, device="cuda", generator=g),
        "actions": torch.nn.functional.one_hot(torch.randint(0, A, (T, B), device="cuda", generator=g), A).float(),
        "rewards": torch.randn(T, B, 1, device="cuda", generator=g),
        "dones": torch.zeros(T, B, 1, device="cuda"),
        "is_first": torch.zeros(T, B, 1, device="cuda"),
    }
    wmc = cfg.algo.world_model
    player = PlayerDV3(wm.encoder, wm.rssm, actor, [A], cfg.algo.player.expl_amount, 1, wmc.stochastic_size,
                       wmc.recurrent_model.recurrent_state_size, runner.device, discrete_size=wmc.discrete_size)
    player.init_states()
    player.use_graphs = True
    pre = {"rgb": torch.randint(0, 255, (1, 1, 3, 64, 64), device="cuda", dtype=torch.uint8) / 255.0}
    for _ in range(4):
        tr.train_step(data)
        with torch.no_grad():
            player.get_exploration_action(pre, False)
    torch.cuda.synchronize()

    def timed(before):
        ts = []
        for _ in range(30):
            before()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            with torch.no_grad():
                player.get_exploration_action(pre, False)
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        return np.median(ts), np.min(ts)

    variants = {
        "alone": lambda: torch.cuda.synchronize(),
        "after-train": lambda: tr.train_step(data),
        "after-train + host sync": lambda: (tr.train_step(data), torch.cuda.synchronize()),
        "after-train + 50us spin": lambda: (tr.train_step(data), torch.cuda._sleep(50000)),
    }
    for name, fn in variants.items():
        med, mn = timed(fn)
        print(f"player {name:26s}: median {med:7.1f} us  min {mn:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
