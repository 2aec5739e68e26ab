"""Print an environment's observation / action space as an agent would see it (reference
``examples/observation_space.py``).

    python examples/observation_space.py agent=dreamer_v3 env=prey
    python examples/observation_space.py agent=ppo env=gym env.id=CartPole-v1
"""
from __future__ import annotations

import sys

from sheeprl_prey_amd.config.compose import compose
from sheeprl_prey_amd.utils.env import make_env
from sheeprl_prey_amd.utils.registry import algorithm_names
from sheeprl_prey_amd.utils.utils import dotdict


def main(argv=None) -> None:
    argv = list(sys.argv[1:] if argv is None else argv)
    agent = next((a.split("=", 1)[1] for a in argv if a.startswith("agent=")), "dreamer_v3")
    rest = [a for a in argv if not a.startswith("agent=")]
    if agent not in algorithm_names():
        raise ValueError(f"Invalid agent `{agent}`: check `python sheeprl.py --sheeprl_help`")
    cfg = dotdict(compose([f"exp={agent}"] + rest))
    cfg.env.capture_video = False
    env = make_env(cfg, cfg.seed, 0, None, "obs")()
    print(f"Observation space of `{cfg.env.id}` for `{agent}`:\n{env.observation_space}")
    print(f"Action space: {env.action_space}")
    env.close()


if __name__ == "__main__":
    main()
