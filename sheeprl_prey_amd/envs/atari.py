"""ALE Atari support: ``make_ale`` (needs ``ale_py`` + ROMs, not in the image) and a native
``AtariPreprocessing`` (noop-reset, frame-skip with 2-frame max-pool, terminal-on-life-loss,
area resize, grayscale) matching gymnasium's wrapper semantics used by ``configs/env/atari.yaml``."""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch
import torch.nn.functional as F

from sheeprl_prey_amd.envs import spaces
from sheeprl_prey_amd.envs.core import Env, Wrapper
from sheeprl_prey_amd.utils.imports import _IS_ATARI_AVAILABLE


def make_ale(id: str, render_mode: Optional[str] = "rgb_array", **kwargs) -> Env:
    if not _IS_ATARI_AVAILABLE:
        raise ModuleNotFoundError(
            f"ALE (ale_py + ROMs) is not installed, cannot create '{id}'. "
            "Use `env=synthetic_atari` for an Atari-shaped synthetic pixel environment."
        )
    import gymnasium  # pragma: no cover - requires ale_py

    return gymnasium.make(id, render_mode=render_mode, **kwargs)  # pragma: no cover


def area_resize(img: np.ndarray, size: int) -> np.ndarray:
    """HWC uint8 -> size x size x C with area interpolation (cv2.INTER_AREA equivalent)."""
    t = torch.from_numpy(np.ascontiguousarray(img)).permute(2, 0, 1)[None].float()
    out = F.adaptive_avg_pool2d(t, (size, size))
    return out[0].permute(1, 2, 0).round().clamp(0, 255).to(torch.uint8).numpy()


def rgb_to_gray(img: np.ndarray) -> np.ndarray:
    g = img[..., 0] * 0.299 + img[..., 1] * 0.587 + img[..., 2] * 0.114
    return np.clip(np.round(g), 0, 255).astype(np.uint8)


class AtariPreprocessing(Wrapper):
    def __init__(self, env: Env, noop_max: int = 30, frame_skip: int = 4, screen_size: int = 84,
                 terminal_on_life_loss: bool = False, grayscale_obs: bool = True, grayscale_newaxis: bool = False,
                 scale_obs: bool = False):
        super().__init__(env)
        self.noop_max = noop_max
        self.frame_skip = frame_skip
        self.screen_size = screen_size
        self.terminal_on_life_loss = terminal_on_life_loss
        self.grayscale_obs = grayscale_obs
        self.grayscale_newaxis = grayscale_newaxis
        self.scale_obs = scale_obs
        self.lives = 0
        self.game_over = False
        shape = (screen_size, screen_size, 1 if grayscale_obs else 3)
        if grayscale_obs and not grayscale_newaxis:
            shape = shape[:-1]
        self.observation_space = spaces.Box(0, 1 if scale_obs else 255, shape, np.float32 if scale_obs else np.uint8)

    def _ale_lives(self) -> int:
        ale = getattr(self.env.unwrapped, "ale", None)
        return ale.lives() if ale is not None else 0

    def _process(self, frames) -> np.ndarray:
        f = np.maximum(frames[0], frames[1]) if len(frames) > 1 else frames[0]
        if f.ndim == 2:
            f = f[..., None]
        if self.grayscale_obs and f.shape[-1] == 3:
            f = rgb_to_gray(f)[..., None]
        f = area_resize(f, self.screen_size)
        if self.grayscale_obs and not self.grayscale_newaxis:
            f = f[..., 0]
        return (f.astype(np.float32) / 255.0) if self.scale_obs else f

    def step(self, action):
        total, terminated, truncated, info = 0.0, False, False, {}
        buf = []
        for t in range(self.frame_skip):
            obs, r, terminated, truncated, info = self.env.step(action)
            total += r
            self.game_over = terminated
            if self.terminal_on_life_loss:
                new_lives = self._ale_lives()
                terminated = terminated or new_lives < self.lives
                self.lives = new_lives
            if terminated or truncated:
                buf.append(obs)
                break
            if t >= self.frame_skip - 2:
                buf.append(obs)
        buf = buf[-2:]
        return self._process(buf), total, terminated, truncated, info

    def reset(self, *, seed=None, options=None):
        obs, info = self.env.reset(seed=seed, options=options)
        noops = int(self.env.unwrapped.np_random.integers(1, self.noop_max + 1)) if self.noop_max > 0 else 0
        for _ in range(noops):
            obs, _, terminated, truncated, info = self.env.step(0)
            if terminated or truncated:
                obs, info = self.env.reset(seed=seed, options=options)
        self.lives = self._ale_lives()
        return self._process([obs]), info
