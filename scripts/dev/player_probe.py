"""DreamerV3 player step (bench config: Atari-100k dims, 1 env) replayed alone: GPU time per graph replay vs eager,
to locate the gaps seen inside the player in the bench step trace.  Prints us per call (events, median of 200)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from sheeprl_prey_amd.algos.dreamer_v3.agent import PlayerDV3, build_models  # noqa: E402
from sheeprl_prey_amd.config.compose import compose  # noqa: E402
from sheeprl_prey_amd.parallel.runner import Runner  # noqa: E402
from sheeprl_prey_amd.utils.env import make_env, make_vector_env  # noqa: E402
from sheeprl_prey_amd.utils.utils import dotdict  # noqa: E402
from sheeprl_prey_amd.algos.common import action_info  # noqa: E402


def main():
    cfg = dotdict(compose(["exp=dreamer_v3_100k_ms_pacman", "env=synthetic_atari", "env.sync_env=True",
                           "cnn_keys.encoder=[rgb]", "cnn_keys.decoder=[rgb]", "fabric.accelerator=cuda"]))
    cfg.pop("hydra", None)
    runner = Runner(**{k: v for k, v in cfg.fabric.items()})
    runner._init_distributed()
    envs = make_vector_env(cfg, [make_env(cfg, 0, 0, None, "train", 0)])
    obs_space = envs.single_observation_space
    is_cont, _, adim = action_info(envs.single_action_space)
    wm, actor, critic, tc = build_models(runner, adim, is_cont, cfg, obs_space)
    dev = runner.device
    player = PlayerDV3(wm.encoder, wm.rssm, actor, adim, cfg.algo.player.expl_amount, 1,
                       cfg.algo.world_model.stochastic_size, cfg.algo.world_model.recurrent_model.recurrent_state_size,
                       dev, discrete_size=cfg.algo.world_model.discrete_size)
    player.init_states()
    obs = {"rgb": torch.randint(0, 255, (1, 1, *obs_space["rgb"].shape), device=dev, dtype=torch.uint8)}
    pre = {"rgb": obs["rgb"] / 255.0}
    for graphs in (False, True):
        player.use_graphs = graphs
        player._graphed = None
        with torch.no_grad():
            for _ in range(5):
                player.get_exploration_action(pre, is_cont)
            torch.cuda.synchronize()
            ts = []
            for _ in range(200):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                player.get_exploration_action(pre, is_cont)
                b.record()
                torch.cuda.synchronize()
                ts.append(a.elapsed_time(b) * 1e3)
        print(f"player {'graph' if graphs else 'eager'}: median {np.median(ts):.1f} us, min {np.min(ts):.1f} us", flush=True)
    torch.cuda._sleep(1000)  # marker for the trace
    torch.cuda.synchronize()
    with torch.no_grad():
        for _ in range(3):
            player.get_exploration_action(pre, is_cont)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
