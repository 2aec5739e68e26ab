"""Synthetic Atari-shaped pixel environment (no emulator / ROMs in the MI355X image).

Same interface as an ``AtariPreprocessing``-wrapped ALE game: ``screen x screen x 3`` (or x1
grayscale) uint8 HWC frames, ``Discrete(n)`` with the minimal action set of ``id``, internal
frame-skip, episodic rewards.  Frames are procedurally rendered moving sprites over a textured
background so that the world model has real structure to fit; the per-step CPU cost is a few
tens of microseconds, so benchmarks measure the learner, not an emulator.
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from sheeprl_prey_amd.envs import spaces
from sheeprl_prey_amd.envs.core import Env, EnvSpec

# minimal action-set sizes of common ALE games
ATARI_ACTIONS = {
    "MsPacman": 9, "Pong": 6, "Boxing": 18, "Breakout": 4, "SpaceInvaders": 6, "Seaquest": 18, "Qbert": 6,
    "Freeway": 3, "Alien": 18, "Amidar": 10, "Assault": 7, "Asterix": 9, "BankHeist": 18, "BattleZone": 18,
    "ChopperCommand": 18, "CrazyClimber": 9, "DemonAttack": 6, "Frostbite": 18, "Gopher": 8, "Hero": 18,
    "Jamesbond": 18, "Kangaroo": 18, "Krull": 18, "KungFuMaster": 14, "PrivateEye": 18, "RoadRunner": 18,
    "UpNDown": 6,
}


def n_actions_for(env_id: str) -> int:
    base = env_id.split("NoFrameskip")[0].split("-v")[0].split("Deterministic")[0]
    return ATARI_ACTIONS.get(base, 18)


class SyntheticAtari(Env):
    metadata = {"render_modes": ["rgb_array"], "render_fps": 15}

    def __init__(self, id: str = "MsPacmanNoFrameskip-v4", screen_size: int = 64, grayscale: bool = False,
                 frame_skip: int = 4, episode_length: int = 2000, render_mode: Optional[str] = "rgb_array",
                 seed: Optional[int] = None, n_sprites: int = 4):
        self.id = id
        self.size = int(screen_size)
        self.grayscale = bool(grayscale)
        self.frame_skip = max(1, int(frame_skip))
        self.episode_length = int(episode_length)
        self.render_mode = render_mode
        self.n_actions = n_actions_for(id)
        self.action_space = spaces.Discrete(self.n_actions)
        c = 1 if self.grayscale else 3
        self.observation_space = spaces.Box(0, 255, (self.size, self.size, c), np.uint8)
        self.spec = EnvSpec(id, entry_point="sheeprl_prey_amd.envs.synthetic:SyntheticAtari")
        self.n_sprites = n_sprites
        self._rng = np.random.default_rng(seed)
        yy, xx = np.mgrid[0 : self.size, 0 : self.size]
        self._bg = (((xx // 8 + yy // 8) % 2) * 40 + 30).astype(np.uint8)
        self._t = 0
        self._frame = None
        # action -> (dx, dy) on a 3x3 stencil, extra actions reuse the stencil
        self._moves = np.array([(dx, dy) for dy in (-1, 0, 1) for dx in (-1, 0, 1)], dtype=np.int64)

    def _render_frame(self) -> np.ndarray:
        s = self.size
        img = np.repeat(self._bg[..., None], 3, axis=-1)
        for i, (p, col) in enumerate(zip(self._pos, self._colors)):
            x, y = int(p[0]), int(p[1])
            r = 3 if i == 0 else 2
            img[max(y - r, 0) : min(y + r, s), max(x - r, 0) : min(x + r, s)] = col
        if self.grayscale:
            g = (img[..., 0] * 0.299 + img[..., 1] * 0.587 + img[..., 2] * 0.114).astype(np.uint8)
            return g[..., None]
        return img

    def reset(self, *, seed: Optional[int] = None, options=None):
        if seed is not None:
            self._rng = np.random.default_rng(seed)
        self._t = 0
        self._pos = self._rng.uniform(4, self.size - 4, size=(self.n_sprites, 2))
        self._vel = self._rng.uniform(-1.5, 1.5, size=(self.n_sprites, 2))
        self._colors = self._rng.integers(60, 255, size=(self.n_sprites, 3)).astype(np.uint8)
        self._frame = self._render_frame()
        return self._frame.copy(), {}

    def step(self, action):
        a = int(np.asarray(action).reshape(-1)[0]) % self.n_actions
        reward = 0.0
        for _ in range(self.frame_skip):
            mv = self._moves[a % len(self._moves)]
            self._pos[0] = np.clip(self._pos[0] + 2 * mv, 3, self.size - 4)
            self._pos[1:] += self._vel[1:]
            bounce = (self._pos[1:] < 3) | (self._pos[1:] > self.size - 4)
            self._vel[1:][bounce] *= -1
            self._pos[1:] = np.clip(self._pos[1:], 3, self.size - 4)
            d = np.abs(self._pos[1:] - self._pos[0]).max(axis=1)
            hit = d < 4
            if hit.any():
                reward += float(hit.sum())
                self._pos[1:][hit] = self._rng.uniform(4, self.size - 4, size=(int(hit.sum()), 2))
        self._t += 1
        self._frame = self._render_frame()
        terminated = False
        truncated = self._t >= self.episode_length
        return self._frame.copy(), reward, terminated, truncated, {}

    def render(self):
        if self._frame is None:
            return None
        f = self._frame
        return np.repeat(f, 3, axis=-1) if f.shape[-1] == 1 else f
