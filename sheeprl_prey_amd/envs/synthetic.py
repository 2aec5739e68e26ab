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
        # the background (RGB or its grayscale) is cached; sprites are drawn straight into the output format with
        # their precomputed values (grayscale = the luma formula applied to the RGB sprite, as a per-pixel
        # conversion of the RGB frame would give)
        s = self.size
        img = self._bg_out.copy()
        for i, ((x, y), col) in enumerate(zip(self._pos, self._col_out)):
            x, y = int(x), int(y)
            r = 3 if i == 0 else 2
            img[max(y - r, 0) : min(y + r, s), max(x - r, 0) : min(x + r, s)] = col
        return img

    def reset(self, *, seed: Optional[int] = None, options=None):
        if seed is not None:
            self._rng = np.random.default_rng(seed)
        self._t = 0
        # sprite state as Python floats: a handful of scalars per step, where numpy's per-call overhead dominated
        self._pos = self._rng.uniform(4, self.size - 4, size=(self.n_sprites, 2)).tolist()
        self._vel = self._rng.uniform(-1.5, 1.5, size=(self.n_sprites, 2)).tolist()
        colors = self._rng.integers(60, 255, size=(self.n_sprites, 3)).astype(np.uint8)
        if self.grayscale:
            bg = self._bg.astype(np.float64)
            self._bg_out = (bg * 0.299 + bg * 0.587 + bg * 0.114).astype(np.uint8)[..., None]
            self._col_out = [np.uint8(int(float(c[0]) * 0.299 + float(c[1]) * 0.587 + float(c[2]) * 0.114)) for c in colors]
        else:
            self._bg_out = np.repeat(self._bg[..., None], 3, axis=-1)
            self._col_out = [c for c in colors]
        self._frame = self._render_frame()
        return self._frame.copy(), {}

    def step(self, action):
        a = int(np.asarray(action).reshape(-1)[0]) % self.n_actions
        reward = 0.0
        lo, hi = 3.0, float(self.size - 4)
        pos, vel = self._pos, self._vel
        dx, dy = (int(v) for v in self._moves[a % len(self._moves)])
        for _ in range(self.frame_skip):
            p0 = pos[0]
            x0, y0 = p0[0] + 2 * dx, p0[1] + 2 * dy
            x0 = lo if x0 < lo else (hi if x0 > hi else x0)
            y0 = lo if y0 < lo else (hi if y0 > hi else y0)
            p0[0], p0[1] = x0, y0
            hits = []
            for i in range(1, self.n_sprites):
                p, v = pos[i], vel[i]
                x, y = p[0] + v[0], p[1] + v[1]
                if x < lo or x > hi:  # bounce, then clip into the field
                    v[0] = -v[0]
                    x = lo if x < lo else hi
                if y < lo or y > hi:
                    v[1] = -v[1]
                    y = lo if y < lo else hi
                p[0], p[1] = x, y
                ax, ay = x - x0, y - y0
                if (ax if ax >= 0 else -ax) < 4 and (ay if ay >= 0 else -ay) < 4:
                    hits.append(i)
            if hits:
                reward += float(len(hits))
                new = self._rng.uniform(4, self.size - 4, size=(len(hits), 2)).tolist()
                for i, q in zip(hits, new):
                    pos[i] = q
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
        if getattr(self, "_floor", None) is None:  # the tiled floor is the same every frame
            yy, xx = np.mgrid[0:s, 0:s]
            self._floor = np.repeat((((xx // 8 + yy // 8) % 2) * 30 + 40).astype(np.uint8)[..., None], 3, axis=-1)
        img = self._floor.copy()
        pts = np.clip((np.tanh(self._x[:16].reshape(8, 2)) * 0.45 + 0.5) * (s - 1), 0, s - 1).astype(np.int64)
        for i, (x, y) in enumerate(pts):
            img[max(y - 2, 0):y + 2, max(x - 2, 0):x + 2] = (200, 60 + 20 * i, 255 - 25 * i)
        return img
