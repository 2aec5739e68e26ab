"""Environment factory (reference: ``sheeprl/utils/env.py:25-221``).

``make_env(cfg, seed, rank, run_name, prefix, vector_env_idx)`` returns a thunk that builds the
configured env and normalises it to a ``Dict`` observation space: vector obs under the first
``mlp_keys.encoder`` key (default ``state``), images under the first ``cnn_keys.encoder`` key
(default ``rgb``) as CHW uint8 ``screen_size``^2 (area resize, optional grayscale), then frame
stacking, reward-as-observation, time limit, episode statistics and optional video capture.
"""
from __future__ import annotations

import os
import warnings
from typing import Any, Callable, Dict, Optional

import numpy as np

from sheeprl_prey_amd.config.instantiate import instantiate
from sheeprl_prey_amd.envs import spaces
from sheeprl_prey_amd.envs.atari import area_resize, rgb_to_gray
from sheeprl_prey_amd.envs.core import Env, PixelObservationWrapper, RecordEpisodeStatistics, TimeLimit, TransformObservation
from sheeprl_prey_amd.envs.wrappers import (
    ActionRepeat,
    FrameStack,
    GrayscaleRenderWrapper,
    MaskVelocityWrapper,
    RecordVideo,
    RewardAsObservationWrapper,
)


def _entry_point(env_id: str) -> str:
    try:
        from sheeprl_prey_amd.envs.registry import spec

        return str(spec(env_id).entry_point)
    except Exception:
        return ""


def make_env(
    cfg: Dict[str, Any],
    seed: int,
    rank: int,
    run_name: Optional[str] = None,
    prefix: str = "",
    vector_env_idx: int = 0,
) -> Callable[[], Env]:
    def thunk() -> Env:
        wrapper_cfg = dict(cfg.env.wrapper)
        target = str(wrapper_cfg.get("_target_", ""))
        if "diambra" in target.lower() and not cfg.env.sync_env:
            ds = dict(wrapper_cfg.get("diambra_settings", {}))
            if ds.pop("splash_screen", True):
                warnings.warn("`splash_screen` must be False with async DIAMBRA envs: it is ignored and set to False.")
            ds["splash_screen"] = False
            wrapper_cfg["diambra_settings"] = ds
        kwargs = {}
        if "seed" in wrapper_cfg:
            kwargs["seed"] = seed
        if "rank" in wrapper_cfg:
            kwargs["rank"] = rank + vector_env_idx
        env = instantiate(wrapper_cfg, **kwargs)
        env_spec = _entry_point(cfg.env.id) or str(getattr(getattr(env, "spec", None), "entry_point", ""))
        is_diambra = "diambra" in target.lower()
        # action repeat (Atari-style envs skip frames themselves)
        if cfg.env.action_repeat > 1 and "atari" not in env_spec.lower() and "atari" not in target.lower() and not is_diambra:
            env = ActionRepeat(env, cfg.env.action_repeat)
        if cfg.env.get("mask_velocities", False):
            env = MaskVelocityWrapper(env)

        # -------- Dict observation space
        obs_space = env.observation_space
        if isinstance(obs_space, spaces.Box) and len(obs_space.shape) < 2:
            if cfg.cnn_keys.encoder:
                if len(cfg.cnn_keys.encoder) > 1:
                    warnings.warn(f"Multiple cnn keys given, only one pixel observation exists in {cfg.env.id}: "
                                  f"keeping {cfg.cnn_keys.encoder[0]}")
                state_key = cfg.mlp_keys.encoder[0] if cfg.mlp_keys.encoder else "state"
                env = PixelObservationWrapper(env, pixels_only=not cfg.mlp_keys.encoder,
                                              pixel_keys=(cfg.cnn_keys.encoder[0],), state_key=state_key)
            else:
                if cfg.mlp_keys.encoder:
                    if len(cfg.mlp_keys.encoder) > 1:
                        warnings.warn(f"Multiple mlp keys given, only one vector observation exists in {cfg.env.id}: "
                                      f"keeping {cfg.mlp_keys.encoder[0]}")
                    mlp_key = cfg.mlp_keys.encoder[0]
                else:
                    mlp_key = "state"
                    cfg.mlp_keys.encoder = [mlp_key]
                inner = env.observation_space
                env = TransformObservation(env, lambda obs, _k=mlp_key: {_k: obs})
                env.observation_space = spaces.Dict({mlp_key: inner})
        elif isinstance(obs_space, spaces.Box) and 2 <= len(obs_space.shape) <= 3:
            if cfg.cnn_keys.encoder and len(cfg.cnn_keys.encoder) > 0:
                if len(cfg.cnn_keys.encoder) > 1:
                    warnings.warn(f"Multiple cnn keys given, only one pixel observation exists in {cfg.env.id}: "
                                  f"keeping {cfg.cnn_keys.encoder[0]}")
                cnn_key = cfg.cnn_keys.encoder[0]
            else:
                cnn_key = "rgb"
                cfg.cnn_keys.encoder = [cnn_key]
            inner = env.observation_space
            env = TransformObservation(env, lambda obs, _k=cnn_key: {_k: obs})
            env.observation_space = spaces.Dict({cnn_key: inner})

        env_cnn_keys = {k for k, v in env.observation_space.spaces.items() if len(v.shape) in (2, 3)}
        cnn_keys = env_cnn_keys.intersection(set(cfg.cnn_keys.encoder or []))
        screen, gray = cfg.env.screen_size, cfg.env.grayscale

        def transform_obs(obs: Dict[str, Any]):
            for k in cnn_keys:
                cur = np.asarray(obs[k])
                is_3d = cur.ndim == 3
                is_gray = not is_3d or cur.shape[0] == 1 or cur.shape[-1] == 1
                channel_first = not is_3d or cur.shape[0] in (1, 3)
                if not is_3d:
                    cur = cur[None]
                if channel_first:
                    cur = np.transpose(cur, (1, 2, 0))
                if cur.shape[:-1] != (screen, screen):
                    cur = area_resize(cur, screen)
                if gray and not is_gray:
                    cur = rgb_to_gray(cur)[..., None]
                if cur.ndim == 2:
                    cur = cur[..., None]
                if cur.shape[-1] == 1 and not gray:
                    cur = np.repeat(cur, 3, axis=-1)
                obs[k] = np.ascontiguousarray(cur.transpose(2, 0, 1))
            return obs

        inner_space = env.observation_space
        env = TransformObservation(env, transform_obs)
        env.observation_space = spaces.Dict(dict(inner_space.items()))
        for k in cnn_keys:
            env.observation_space[k] = spaces.Box(0, 255, (1 if gray else 3, screen, screen), np.uint8)

        if cnn_keys and cfg.env.frame_stack > 1:
            if cfg.env.frame_stack_dilation <= 0:
                raise ValueError(f"The frame stack dilation argument must be greater than zero, got: {cfg.env.frame_stack_dilation}")
            env = FrameStack(env, cfg.env.frame_stack, list(cnn_keys), cfg.env.frame_stack_dilation)
        if cfg.env.reward_as_observation:
            env = RewardAsObservationWrapper(env)
        env.action_space.seed(seed)
        env.observation_space.seed(seed)
        if cfg.env.max_episode_steps and cfg.env.max_episode_steps > 0:
            env = TimeLimit(env, max_episode_steps=cfg.env.max_episode_steps)
        env = RecordEpisodeStatistics(env)
        if cfg.env.capture_video and rank == 0 and vector_env_idx == 0 and run_name is not None:
            if cfg.env.grayscale:
                env = GrayscaleRenderWrapper(env)
            env = RecordVideo(env, os.path.join(run_name, prefix + "_videos" if prefix else "videos"))
        return env

    return thunk


def get_dummy_env(id: str, size=None):
    """Test envs (reference ``utils/env.py`` dummy branch).  ``*_vec`` ids (or a 1-D ``size``) give
    vector observations (mapped to the ``state`` key) for the vector-only agents (SAC, DroQ)."""
    from sheeprl_prey_amd.envs.dummy import ContinuousDummyEnv, DiscreteDummyEnv, MultiDiscreteDummyEnv

    kw = {}
    if size is not None:
        kw["size"] = tuple(size)
    elif id.endswith("_vec"):
        kw["size"] = (8,)
    if "continuous" in id:
        return ContinuousDummyEnv(**kw)
    if "multidiscrete" in id:
        return MultiDiscreteDummyEnv(**kw)
    if "discrete" in id:
        return DiscreteDummyEnv(**kw)
    raise ValueError(f"Unrecognized dummy environment: {id}")


def make_vector_env(cfg, env_fns):
    """SyncVectorEnv if ``cfg.env.sync_env`` else AsyncVectorEnv (one worker process per env)."""
    from sheeprl_prey_amd.envs.vector import AsyncVectorEnv, SyncVectorEnv

    return SyncVectorEnv(env_fns) if cfg.env.sync_env else AsyncVectorEnv(env_fns)
