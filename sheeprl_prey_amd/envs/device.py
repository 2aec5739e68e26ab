"""Device-resident vectorised environments (MI355X-native rollouts).

``CartPoleDevice`` keeps N CartPole-v1 environments in GPU memory and steps them all with one HIP
kernel (``ops/csrc/envs.hip``): same dynamics, termination bounds, reward (+1 per step, including
the terminating one), 500-step time limit (truncation) and autoreset semantics as the host path
(gymnasium ``SyncVectorEnv`` + ``TimeLimit`` + ``RecordEpisodeStatistics``: the returned observation
of a finished env is the reset observation, the pre-reset one is ``final_obs``).  Nothing in
``step`` synchronises with the host, so a whole rollout can be captured in a hipGraph
(``algos/ppo/ppo.py: DeviceRollout``).  CPU tensors step with the same math in torch ops.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch
from torch import Tensor

from sheeprl_prey_amd.envs import spaces

DEVICE_ENVS = ("CartPole-v1", "CartPole-v0")


class CartPoleDevice:
    single_observation_space = spaces.Dict({"state": spaces.Box(-float("inf"), float("inf"), (4,), "float32")})
    single_action_space = spaces.Discrete(2)

    def __init__(self, num_envs: int, device, max_episode_steps: int = 500, seed: Optional[int] = None):
        self.num_envs = int(num_envs)
        self.device = torch.device(device)
        self.max_steps = int(max_episode_steps)
        n, dev = self.num_envs, self.device
        self.gen = torch.Generator(device=dev)
        if seed is not None:
            self.gen.manual_seed(int(seed))
        self.state = torch.zeros(n, 4, device=dev)
        self.steps = torch.zeros(n, dtype=torch.int32, device=dev)
        self.ep_ret = torch.zeros(n, device=dev)
        # step outputs (fixed buffers: a captured rollout reads / writes the same addresses)
        self.obs = torch.zeros(n, 4, device=dev)
        self.reward = torch.zeros(n, device=dev)
        self.terminated = torch.zeros(n, device=dev)
        self.truncated = torch.zeros(n, device=dev)
        self.final_obs = torch.zeros(n, 4, device=dev)
        self.done_ret = torch.zeros(n, device=dev)
        self.done_len = torch.zeros(n, device=dev)

    def reset(self, seed: Optional[int] = None) -> Dict[str, Tensor]:
        if seed is not None:
            self.gen.manual_seed(int(seed))
        u = torch.rand(self.num_envs, 4, device=self.device, generator=self.gen)
        self.state.copy_(u * 0.1 - 0.05)
        self.steps.zero_()
        self.ep_ret.zero_()
        self.obs.copy_(self.state)
        return {"state": self.obs}

    def step(self, action: Tensor) -> Dict[str, Tensor]:
        """``action``: [N] int64 indices.  Updates the env buffers in place and returns them."""
        # capture-safe RNG: the default (graph-aware) generator on device
        u = torch.rand(self.num_envs, 4, device=self.device)
        a = action.reshape(-1).to(torch.int64).contiguous()
        if self.device.type == "cuda":
            from sheeprl_prey_amd import ops

            ops._ext().cartpole_step(self.state, self.steps, self.ep_ret, a, u, self.obs, self.reward, self.terminated,
                                     self.truncated, self.final_obs, self.done_ret, self.done_len, self.max_steps)
        else:
            self._step_torch(a, u)
        return {"obs": self.obs, "reward": self.reward, "terminated": self.terminated, "truncated": self.truncated,
                "final_obs": self.final_obs, "done_ret": self.done_ret, "done_len": self.done_len}

    def _step_torch(self, a: Tensor, u: Tensor) -> None:
        gravity, masscart, masspole, length, force_mag, tau = 9.8, 1.0, 0.1, 0.5, 10.0, 0.02
        total_mass, pml = masspole + masscart, masspole * length
        x, x_dot, th, th_dot = self.state.unbind(-1)
        force = torch.where(a == 1, force_mag, -force_mag).to(x.dtype)
        c, s = torch.cos(th), torch.sin(th)
        temp = (force + pml * th_dot * th_dot * s) / total_mass
        thacc = (gravity * s - c * temp) / (length * (4.0 / 3.0 - masspole * c * c / total_mass))
        xacc = temp - pml * thacc * c / total_mass
        nxt = torch.stack((x + tau * x_dot, x_dot + tau * xacc, th + tau * th_dot, th_dot + tau * thacc), -1)
        thr = 12 * 2 * math.pi / 360
        term = (nxt[:, 0].abs() > 2.4) | (nxt[:, 2].abs() > thr)
        n = self.steps + 1
        trunc = (~term) & (n >= self.max_steps)
        done = term | trunc
        ret = self.ep_ret + 1.0
        self.final_obs.copy_(nxt)
        self.reward.fill_(1.0)
        self.terminated.copy_(term.float())
        self.truncated.copy_(trunc.float())
        self.done_ret.copy_(torch.where(done, ret, torch.zeros_like(ret)))
        self.done_len.copy_(torch.where(done, n.float(), torch.zeros_like(ret)))
        self.state.copy_(torch.where(done[:, None], u * 0.1 - 0.05, nxt))
        self.steps.copy_(torch.where(done, torch.zeros_like(n), n))
        self.ep_ret.copy_(torch.where(done, torch.zeros_like(ret), ret))
        self.obs.copy_(self.state)


def make_device_env(env_id: str, num_envs: int, device, seed: Optional[int] = None, max_episode_steps: Optional[int] = None):
    if env_id not in DEVICE_ENVS:
        raise ValueError(f"no device implementation for {env_id}; available: {DEVICE_ENVS}")
    steps = max_episode_steps or (500 if env_id == "CartPole-v1" else 200)
    return CartPoleDevice(num_envs, device, steps, seed)
