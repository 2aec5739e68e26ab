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


class SyntheticControl(Env):
    """Synthetic continuous-control env with the dm_control ``walker_walk`` interface (no MuJoCo /
    dm_control in the image): a ``Box(obs_dim)`` float32 ``state`` vector, ``Box(-1, 1, act_dim)``
    actions, 1000-step episodes.  The state follows a fixed random stable linear system driven by the
    action through a tanh, and the reward is a smooth function of state and action in [0, 1] (walker's
    upright x speed reward shape), so an agent has something learnable; a step costs a few
    microseconds of host time, so benchmarks measure the learner.  With ``from_pixels`` the
    observation is the dict ``{"rgb": CHW uint8 render, "state": ...}`` of the DMC adapter."""

    metadata = {"render_modes": ["rgb_array"], "render_fps": 30}

    def __init__(self, id: str = "walker_walk", obs_dim: int = 24, act_dim: int = 6, episode_length: int = 1000,
                 render_mode: Optional[str] = "rgb_array", seed: Optional[int] = None, screen_size: int = 64,
                 from_pixels: bool = True, from_vectors: bool = True):
        # from_pixels / from_vectors: accepted for DMC-config compatibility; the env factory adds the rendered
        # pixels (PixelObservationWrapper) when cnn keys are requested
        self.id = id
        self.obs_dim, self.act_dim = int(obs_dim), int(act_dim)
        self.episode_length = int(episode_length)
        self.render_mode = render_mode
        self.size = int(screen_size)
        self.action_space = spaces.Box(-1.0, 1.0, (self.act_dim,), np.float32)
        self.observation_space = spaces.Box(-np.inf, np.inf, (self.obs_dim,), np.float32)
        self.spec = EnvSpec(id, entry_point="sheeprl_prey_amd.envs.synthetic:SyntheticControl")
        g = np.random.default_rng(1234 + self.obs_dim * 31 + self.act_dim)  # the system itself is fixed
        q, _ = np.linalg.qr(g.standard_normal((self.obs_dim, self.obs_dim)))
        self._A = (0.97 * q).astype(np.float32)
        self._B = (0.3 * g.standard_normal((self.obs_dim, self.act_dim))).astype(np.float32)
        self._w = g.standard_normal(self.obs_dim).astype(np.float32) / np.sqrt(self.obs_dim)
        self._rng = np.random.default_rng(seed)
        self._x = np.zeros(self.obs_dim, np.float32)
        self._t = 0

    def reset(self, *, seed: Optional[int] = None, options=None):
        if seed is not None:
            self._rng = np.random.default_rng(seed)
        self._t = 0
        self._x = self._rng.normal(0.0, 0.1, self.obs_dim).astype(np.float32)
        return self._x.copy(), {}

    def step(self, action):
        a = np.clip(np.asarray(action, dtype=np.float32).reshape(self.act_dim), -1.0, 1.0)
        self._x = np.tanh(self._A @ self._x + self._B @ a) + self._rng.normal(0.0, 0.01, self.obs_dim).astype(np.float32)
        speed = float(self._w @ self._x)
        reward = float(0.5 * (1.0 + np.tanh(speed)) * (1.0 - 0.1 * float(np.mean(a * a))))
        self._t += 1
        return self._x.copy(), reward, False, self._t >= self.episode_length, {}

    def render(self):
        """A 'stick figure' of the state: 8 segments whose endpoints follow pairs of state coordinates,
        drawn over a tiled floor (64x64x3 uint8 by default)."""
        s = self.size
        yy, xx = np.mgrid[0:s, 0:s]
        img = np.repeat((((xx // 8 + yy // 8) % 2) * 30 + 40).astype(np.uint8)[..., None], 3, axis=-1)
        pts = np.clip((np.tanh(self._x[:16].reshape(8, 2)) * 0.45 + 0.5) * (s - 1), 0, s - 1).astype(np.int64)
        for i, (x, y) in enumerate(pts):
            img[max(y - 2, 0):y + 2, max(x - 2, 0):x + 2] = (200, 60 + 20 * i, 255 - 25 * i)
        return img
