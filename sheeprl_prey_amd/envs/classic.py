"""Classic-control environments (CartPole, Pendulum, MountainCar, MountainCarContinuous).

Written natively (gymnasium is not in the image) with the standard published dynamics,
constants, termination rules and episode limits of the ``*-v0/v1`` ids, so the PPO/SAC
vector-observation configs of the reference (``configs/exp/ppo.yaml``: CartPole-v1) run as-is.
``render_mode="rgb_array"`` rasterises a small frame with numpy for pixel-observation configs.
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np

from sheeprl_prey_amd.envs import spaces
from sheeprl_prey_amd.envs.core import Env


def _canvas(h: int, w: int) -> np.ndarray:
    return np.full((h, w, 3), 255, dtype=np.uint8)


def _draw_line(img: np.ndarray, x0: float, y0: float, x1: float, y1: float, color, width: int = 3) -> None:
    n = int(max(abs(x1 - x0), abs(y1 - y0))) + 1
    xs = np.linspace(x0, x1, n)
    ys = np.linspace(y0, y1, n)
    h, w = img.shape[:2]
    for dx in range(-(width // 2), width // 2 + 1):
        for dy in range(-(width // 2), width // 2 + 1):
            xi = np.clip((xs + dx).astype(int), 0, w - 1)
            yi = np.clip((ys + dy).astype(int), 0, h - 1)
            img[yi, xi] = color


class CartPoleEnv(Env):
    metadata = {"render_modes": ["rgb_array"], "render_fps": 50}

    def __init__(self, render_mode: Optional[str] = None):
        self.gravity = 9.8
        self.masscart = 1.0
        self.masspole = 0.1
        self.total_mass = self.masspole + self.masscart
        self.length = 0.5
        self.polemass_length = self.masspole * self.length
        self.force_mag = 10.0
        self.tau = 0.02
        self.theta_threshold_radians = 12 * 2 * math.pi / 360
        self.x_threshold = 2.4
        high = np.array([self.x_threshold * 2, np.finfo(np.float32).max, self.theta_threshold_radians * 2,
                         np.finfo(np.float32).max], dtype=np.float32)
        self.action_space = spaces.Discrete(2)
        self.observation_space = spaces.Box(-high, high, dtype=np.float32)
        self.render_mode = render_mode
        self.state = None
        self.steps_beyond_terminated = None

    def step(self, action):
        x, x_dot, theta, theta_dot = self.state
        force = self.force_mag if int(action) == 1 else -self.force_mag
        costheta, sintheta = math.cos(theta), math.sin(theta)
        temp = (force + self.polemass_length * theta_dot**2 * sintheta) / self.total_mass
        thetaacc = (self.gravity * sintheta - costheta * temp) / (
            self.length * (4.0 / 3.0 - self.masspole * costheta**2 / self.total_mass)
        )
        xacc = temp - self.polemass_length * thetaacc * costheta / self.total_mass
        x = x + self.tau * x_dot
        x_dot = x_dot + self.tau * xacc
        theta = theta + self.tau * theta_dot
        theta_dot = theta_dot + self.tau * thetaacc
        self.state = (x, x_dot, theta, theta_dot)
        terminated = bool(
            x < -self.x_threshold or x > self.x_threshold
            or theta < -self.theta_threshold_radians or theta > self.theta_threshold_radians
        )
        if not terminated:
            reward = 1.0
        elif self.steps_beyond_terminated is None:
            self.steps_beyond_terminated = 0
            reward = 1.0
        else:
            self.steps_beyond_terminated += 1
            reward = 0.0
        return np.array(self.state, dtype=np.float32), reward, terminated, False, {}

    def reset(self, *, seed: Optional[int] = None, options=None):
        super().reset(seed=seed)
        self.state = self.np_random.uniform(low=-0.05, high=0.05, size=(4,))
        self.steps_beyond_terminated = None
        return np.array(self.state, dtype=np.float32), {}

    def render(self):
        if self.render_mode != "rgb_array" or self.state is None:
            return None
        H, W = 400, 600
        img = _canvas(H, W)
        scale = W / (self.x_threshold * 2)
        cx = self.state[0] * scale + W / 2.0
        cy = 300
        img[cy - 15 : cy + 15, int(max(cx - 25, 0)) : int(min(cx + 25, W))] = (0, 0, 0)
        plen = scale * 2 * self.length
        _draw_line(img, cx, cy, cx + plen * math.sin(self.state[2]), cy - plen * math.cos(self.state[2]), (202, 152, 101), 9)
        img[cy + 15 :, :] = img[cy + 15 :, :]
        return img


def _angle_normalize(x):
    return ((x + np.pi) % (2 * np.pi)) - np.pi


class PendulumEnv(Env):
    metadata = {"render_modes": ["rgb_array"], "render_fps": 30}

    def __init__(self, render_mode: Optional[str] = None, g: float = 10.0):
        self.max_speed = 8
        self.max_torque = 2.0
        self.dt = 0.05
        self.g = g
        self.m = 1.0
        self.l = 1.0
        self.render_mode = render_mode
        high = np.array([1.0, 1.0, self.max_speed], dtype=np.float32)
        self.action_space = spaces.Box(-self.max_torque, self.max_torque, shape=(1,), dtype=np.float32)
        self.observation_space = spaces.Box(-high, high, dtype=np.float32)
        self.state = None

    def step(self, u):
        th, thdot = self.state
        u = float(np.clip(np.asarray(u).reshape(-1)[0], -self.max_torque, self.max_torque))
        costs = _angle_normalize(th) ** 2 + 0.1 * thdot**2 + 0.001 * (u**2)
        newthdot = thdot + (3 * self.g / (2 * self.l) * np.sin(th) + 3.0 / (self.m * self.l**2) * u) * self.dt
        newthdot = np.clip(newthdot, -self.max_speed, self.max_speed)
        newth = th + newthdot * self.dt
        self.state = np.array([newth, newthdot])
        return self._obs(), -float(costs), False, False, {}

    def reset(self, *, seed=None, options=None):
        super().reset(seed=seed)
        high = np.array([np.pi, 1.0])
        self.state = self.np_random.uniform(low=-high, high=high)
        return self._obs(), {}

    def _obs(self):
        th, thdot = self.state
        return np.array([np.cos(th), np.sin(th), thdot], dtype=np.float32)

    def render(self):
        if self.render_mode != "rgb_array" or self.state is None:
            return None
        S = 500
        img = _canvas(S, S)
        c = S / 2
        th = self.state[0] + np.pi / 2
        _draw_line(img, c, c, c + 0.4 * S * np.cos(th), c - 0.4 * S * np.sin(th), (204, 77, 77), 15)
        return img


class MountainCarContinuousEnv(Env):
    metadata = {"render_modes": ["rgb_array"], "render_fps": 30}

    def __init__(self, render_mode: Optional[str] = None, goal_velocity: float = 0.0):
        self.min_action, self.max_action = -1.0, 1.0
        self.min_position, self.max_position = -1.2, 0.6
        self.max_speed = 0.07
        self.goal_position = 0.45
        self.goal_velocity = goal_velocity
        self.power = 0.0015
        self.render_mode = render_mode
        self.low_state = np.array([self.min_position, -self.max_speed], dtype=np.float32)
        self.high_state = np.array([self.max_position, self.max_speed], dtype=np.float32)
        self.action_space = spaces.Box(self.min_action, self.max_action, shape=(1,), dtype=np.float32)
        self.observation_space = spaces.Box(self.low_state, self.high_state, dtype=np.float32)
        self.state = None

    def step(self, action):
        position, velocity = self.state
        force = min(max(float(np.asarray(action).reshape(-1)[0]), self.min_action), self.max_action)
        velocity += force * self.power - 0.0025 * math.cos(3 * position)
        velocity = min(max(velocity, -self.max_speed), self.max_speed)
        position += velocity
        position = min(max(position, self.min_position), self.max_position)
        if position == self.min_position and velocity < 0:
            velocity = 0
        terminated = bool(position >= self.goal_position and velocity >= self.goal_velocity)
        reward = 100.0 if terminated else 0.0
        reward -= math.pow(force, 2) * 0.1
        self.state = np.array([position, velocity], dtype=np.float32)
        return self.state.copy(), reward, terminated, False, {}

    def reset(self, *, seed=None, options=None):
        super().reset(seed=seed)
        self.state = np.array([self.np_random.uniform(low=-0.6, high=-0.4), 0], dtype=np.float32)
        return self.state.copy(), {}


class MountainCarEnv(Env):
    metadata = {"render_modes": ["rgb_array"], "render_fps": 30}

    def __init__(self, render_mode: Optional[str] = None, goal_velocity: float = 0.0):
        self.min_position, self.max_position = -1.2, 0.6
        self.max_speed = 0.07
        self.goal_position = 0.5
        self.goal_velocity = goal_velocity
        self.force = 0.001
        self.gravity = 0.0025
        self.render_mode = render_mode
        self.low = np.array([self.min_position, -self.max_speed], dtype=np.float32)
        self.high = np.array([self.max_position, self.max_speed], dtype=np.float32)
        self.action_space = spaces.Discrete(3)
        self.observation_space = spaces.Box(self.low, self.high, dtype=np.float32)
        self.state = None

    def step(self, action: int):
        position, velocity = self.state
        velocity += (int(action) - 1) * self.force + math.cos(3 * position) * (-self.gravity)
        velocity = float(np.clip(velocity, -self.max_speed, self.max_speed))
        position += velocity
        position = float(np.clip(position, self.min_position, self.max_position))
        if position == self.min_position and velocity < 0:
            velocity = 0
        terminated = bool(position >= self.goal_position and velocity >= self.goal_velocity)
        self.state = (position, velocity)
        return np.array(self.state, dtype=np.float32), -1.0, terminated, False, {}

    def reset(self, *, seed=None, options=None):
        super().reset(seed=seed)
        self.state = np.array([self.np_random.uniform(low=-0.6, high=-0.4), 0])
        return np.array(self.state, dtype=np.float32), {}
