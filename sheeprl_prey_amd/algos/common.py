"""Pieces every algorithm main() shares (the reference re-implements them in each ~500-line
main; e.g. ``ppo/ppo.py:107-459``, ``dreamer_v3/dreamer_v3.py:354-807``): resume handling,
env construction, action-space introspection, obs conversion, throughput logging."""
from __future__ import annotations

import copy
import os
import pathlib
import warnings
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
from torch import Tensor

from sheeprl_prey_amd.envs import spaces
from sheeprl_prey_amd.utils.env import make_env, make_vector_env
from sheeprl_prey_amd.utils.timer import timer
from sheeprl_prey_amd.utils.utils import dotdict


def load_resume(runner, cfg) -> Tuple[Any, Optional[Dict[str, Any]]]:
    """If ``checkpoint.resume_from`` is set: load the state and the run's saved config, keeping
    the new ``root_dir/run_name`` and rescaling ``per_rank_batch_size`` to the new world size
    (reference ``dreamer_v3.py:363-372``)."""
    if not cfg.checkpoint.resume_from:
        return cfg, None
    import yaml

    root_dir, run_name = cfg.root_dir, cfg.run_name
    state = runner.load(cfg.checkpoint.resume_from)
    ckpt_path = pathlib.Path(cfg.checkpoint.resume_from)
    cfg_path = ckpt_path.parent.parent.parent / ".hydra" / "config.yaml"
    if not cfg_path.exists():
        cfg_path = ckpt_path.parent.parent / ".hydra" / "config.yaml"
    with open(cfg_path) as f:
        old = dotdict(yaml.safe_load(f))
    old.checkpoint.resume_from = str(ckpt_path)
    if "batch_size" in state and state["batch_size"] is not None:
        old.per_rank_batch_size = state["batch_size"] // runner.world_size
    old.root_dir = root_dir
    old.run_name = run_name
    old.fabric = cfg.fabric
    return old, state


def build_envs(runner, cfg, log_dir: Optional[str], prefix: str = "train", restart_on_exception: bool = False):
    from functools import partial

    from sheeprl_prey_amd.envs.wrappers import RestartOnException

    rank = runner.global_rank
    fns = []
    for i in range(cfg.env.num_envs):
        thunk = make_env(cfg, cfg.seed + rank * cfg.env.num_envs + i, rank * cfg.env.num_envs,
                         log_dir if rank == 0 else None, prefix, vector_env_idx=i)
        fns.append(partial(RestartOnException, thunk) if restart_on_exception else thunk)
    return make_vector_env(cfg, fns)


def action_info(action_space) -> Tuple[bool, bool, List[int]]:
    is_continuous = isinstance(action_space, spaces.Box)
    is_multidiscrete = isinstance(action_space, spaces.MultiDiscrete)
    if is_continuous:
        actions_dim = list(action_space.shape)
    elif is_multidiscrete:
        actions_dim = action_space.nvec.tolist()
    else:
        actions_dim = [action_space.n]
    return is_continuous, is_multidiscrete, actions_dim


def check_obs_keys(cfg, observation_space) -> None:
    if not isinstance(observation_space, spaces.Dict):
        raise RuntimeError(f"Unexpected observation type, should be of type Dict, got: {observation_space}")
    if (cfg.cnn_keys.encoder or []) + (cfg.mlp_keys.encoder or []) == []:
        raise RuntimeError(
            "You should specify at least one CNN keys or MLP keys from the cli: "
            "`cnn_keys.encoder=[rgb]` or `mlp_keys.encoder=[state]`"
        )


def one_hot_actions(actions: np.ndarray, actions_dim: Sequence[int]) -> np.ndarray:
    """Env-format discrete actions -> concatenated one-hot (reference ``dreamer_v3.py:599-607``)."""
    acts = np.asarray(actions).reshape(len(actions_dim), -1) if len(actions_dim) > 1 else np.asarray(actions).reshape(1, -1)
    out = [np.eye(d, dtype=np.float32)[a.astype(np.int64)] for a, d in zip(acts, actions_dim)]
    return np.concatenate(out, axis=-1)


def log_throughput(runner, timer_metrics: Dict[str, float], policy_step: int, last_log: int, train_step: int,
                   last_train: int, action_repeat: int) -> None:
    """``Time/sps_train`` and ``Time/sps_env_interaction`` (reference ``dreamer_v3.py:754-767``).  Also the
    shared device health check (``ops.check_faults``): a recorded kernel fault raises here at the latest."""
    from sheeprl_prey_amd import ops

    ops.check_faults()
    ws = runner.world_size
    if "Time/train_time" in timer_metrics and timer_metrics["Time/train_time"] > 0:
        runner.log("Time/sps_train", (train_step - last_train) / timer_metrics["Time/train_time"], policy_step)
    if "Time/env_interaction_time" in timer_metrics and timer_metrics["Time/env_interaction_time"] > 0:
        runner.log(
            "Time/sps_env_interaction",
            ((policy_step - last_log) / ws * action_repeat) / timer_metrics["Time/env_interaction_time"],
            policy_step,
        )


def warn_log_ckpt_every(cfg, policy_steps_per_update: int) -> None:
    if cfg.metric.log_every % policy_steps_per_update != 0:
        warnings.warn(
            f"The metric.log_every parameter ({cfg.metric.log_every}) is not a multiple of the "
            f"policy_steps_per_update value ({policy_steps_per_update}), so the metrics will be logged at the "
            "nearest greater multiple of the policy_steps_per_update value."
        )
    if cfg.checkpoint.every % policy_steps_per_update != 0:
        warnings.warn(
            f"The checkpoint.every parameter ({cfg.checkpoint.every}) is not a multiple of the "
            f"policy_steps_per_update value ({policy_steps_per_update}), so the checkpoint will be saved at the "
            "nearest greater multiple of the policy_steps_per_update value."
        )


def episode_stats(infos: Dict[str, Any]):
    """Yield (env_idx, return, length) for finished episodes."""
    if "final_info" not in infos:
        return
    for i, ep in enumerate(infos["final_info"]):
        if ep is not None and "episode" in ep:
            yield i, ep["episode"]["r"], ep["episode"]["l"]


def episode_success(infos: Dict[str, Any]):
    """Yield (env_idx, 1.0 / 0.0) for finished episodes whose final info carries the env's ``is success`` flag (the
    prey env's goal-reached flag, ``prey_env/gymnasium_env_bins.py:195``); nothing for envs without one."""
    if "final_info" not in infos:
        return
    for i, ep in enumerate(infos["final_info"]):
        if ep is not None and "episode" in ep and "is success" in ep:
            yield i, float(bool(np.asarray(ep["is success"]).reshape(-1)[0]))


class PolynomialLR:
    """``torch.optim.lr_scheduler.PolynomialLR`` for the flat optimisers (state-dict compatible)."""

    def __init__(self, optimizer, total_iters: int = 5, power: float = 1.0):
        self.optimizer = optimizer
        self.total_iters = total_iters
        self.power = power
        self.base_lrs = [g["lr"] for g in optimizer.param_groups]
        self.last_epoch = 0
        self._last_lr = list(self.base_lrs)

    def get_last_lr(self):
        return self._last_lr

    def step(self):
        self.last_epoch += 1
        t = min(self.last_epoch, self.total_iters)
        factor = (1.0 - t / self.total_iters) ** self.power if self.total_iters > 0 else 1.0
        for g, base in zip(self.optimizer.param_groups, self.base_lrs):
            g["lr"] = base * factor
        self._last_lr = [g["lr"] for g in self.optimizer.param_groups]

    def state_dict(self):
        return {"last_epoch": self.last_epoch, "base_lrs": self.base_lrs, "total_iters": self.total_iters,
                "power": self.power, "_last_lr": self._last_lr}

    def load_state_dict(self, sd):
        self.last_epoch = sd["last_epoch"]
        self.base_lrs = sd["base_lrs"]
        self._last_lr = sd.get("_last_lr", self.base_lrs)
        for g, lr in zip(self.optimizer.param_groups, self._last_lr):
            g["lr"] = lr


def setup_logger(runner, cfg):
    from sheeprl_prey_amd.utils.logger import create_tensorboard_logger
    from sheeprl_prey_amd.utils.utils import save_configs

    logger, log_dir = create_tensorboard_logger(runner, cfg)
    if runner.is_global_zero:
        runner._loggers = [logger]
        logger.log_hyperparams(cfg)
        save_configs(cfg, os.path.dirname(log_dir))
    return logger, log_dir


def to_torch_obs(obs: Dict[str, np.ndarray], keys: Sequence[str], mlp_keys: Sequence[str], device, num_envs: int,
                 cnn_keys: Sequence[str] = ()) -> Dict[str, Tensor]:
    out = {}
    for k in keys:
        t = torch.as_tensor(np.asarray(obs[k]))
        if k in cnn_keys:
            t = t.view(num_envs, -1, *t.shape[-2:])
        if k in mlp_keys:
            t = t.float()
        out[k] = t.to(device, non_blocking=t.is_pinned())
    return out


def shard_indices(n: int, runner, shuffle: bool, seed: int, epoch: int) -> torch.Tensor:
    """DistributedSampler semantics: a seeded permutation, padded to a multiple of world, strided."""
    g = torch.Generator().manual_seed(seed + epoch)
    idx = torch.randperm(n, generator=g) if shuffle else torch.arange(n)
    ws, rk = runner.world_size, runner.global_rank
    total = ((n + ws - 1) // ws) * ws
    if total > n:
        idx = torch.cat([idx, idx[: total - n]])
    return idx[rk:total:ws]


def restore_replay_buffer(rb, saved, runner) -> None:
    """Resume a replay buffer saved by ``CheckpointCallback``: a per-rank list (gathered on rank 0)
    or a single state (reference ``sac/sac.py:186-193``)."""
    if isinstance(saved, list):
        if len(saved) != runner.world_size:
            raise RuntimeError(f"Given {len(saved)}, but {runner.world_size} processes are instantiated")
        saved = saved[runner.global_rank]
    if not isinstance(saved, dict):
        raise RuntimeError("unrecognised replay buffer checkpoint format")
    rb.load_state_dict(saved)
