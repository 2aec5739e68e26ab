"""Command line entry point (reference: ``sheeprl/cli.py:19-84``).

``python sheeprl.py exp=<preset> [group=option] [a.b=value] ...`` composes the config tree
(Hydra semantics, see ``config/compose.py``), saves ``<run_dir>/.hydra/config.yaml``, looks the
algorithm up in the registry and launches it through the :class:`Runner` (one process per
device; torchrun-compatible).
"""
from __future__ import annotations

import os
import sys
import warnings
from typing import Any, Dict, List, Optional

from sheeprl_prey_amd.config.compose import check_missing, compose
from sheeprl_prey_amd.utils.callback import CheckpointCallback
from sheeprl_prey_amd.utils.registry import find_algorithm, tasks
from sheeprl_prey_amd.utils.utils import dotdict, print_config, save_configs


def check_configs(cfg: Dict[str, Any]) -> None:
    strategy = str(cfg["fabric"].get("strategy", "auto")).lower()
    if "fsdp" in strategy:
        raise ValueError(
            "FSDP strategy is not supported: RL models here are small and replicated; use `fabric.strategy=ddp`"
        )
    missing = check_missing(cfg, skip=("hydra",))
    if missing:
        raise ValueError(f"Missing mandatory value(s): {missing}")


def run_algorithm(cfg: Dict[str, Any]) -> None:
    import importlib

    from sheeprl_prey_amd.parallel.runner import Runner

    import sheeprl_prey_amd  # noqa: F401  (registers the algorithms)

    algo_name = cfg.algo.name
    module_path, entry = find_algorithm(algo_name)
    if entry is None:
        raise RuntimeError(f"Given the algorithm named `{algo_name}`, no module has been found to be imported.")
    module = importlib.import_module(f"{module_path}.{entry['name']}")
    fn = getattr(module, entry["entrypoint"])
    fabric_cfg = dict(cfg.fabric)
    fabric_cfg.pop("_target_", None)
    runner = Runner(**fabric_cfg, callbacks=[CheckpointCallback()])
    runner.launch(fn, cfg)


def compose_cli(argv: Optional[List[str]] = None, config_name: str = "config") -> dotdict:
    argv = list(sys.argv[1:] if argv is None else argv)
    cfg = compose(argv, config_name=config_name)
    return dotdict(cfg)


def run(argv: Optional[List[str]] = None) -> None:
    cfg = compose_cli(argv)
    check_configs(cfg)
    hydra_cfg = cfg.pop("hydra", None)
    cfg.pop("_choices_", None)
    is_rank_zero = int(os.environ.get("RANK", "0")) == 0
    if is_rank_zero:
        print_config(cfg)
        run_dir = hydra_cfg["run"]["dir"] if hydra_cfg else os.path.join("logs", "runs", cfg.root_dir, cfg.run_name)
        save_configs(cfg, run_dir)
    run_algorithm(cfg)


def evaluation(argv: Optional[List[str]] = None) -> None:
    """``sheeprl-eval checkpoint_path=<ckpt> [env overrides]``: greedy test episode of a DV3 checkpoint
    (the fork's ``eval.py`` / ``visulize.py``)."""
    from sheeprl_prey_amd.evaluate import evaluate_from_cli

    evaluate_from_cli(list(sys.argv[1:] if argv is None else argv))


if __name__ == "__main__":
    run()
