"""The env-interaction step of the DreamerV3 loop (reference ``dreamer_v3.py:587-709``), shared by
``dreamer_v3.main`` and ``bench.py`` so the headline number measures the loop users run.

One step on the GPU, in stream order:

    host: row (obs_t, reward_t, done_t, is_first_t) -> pinned ring slot (two slots, alternating)
    side stream: pinned slot -> device obs buffer (H2D), event
    main stream: wait(H2D event) -> player graph (act with W_t) -> action readback into pinned memory,
                 event -> replay-buffer add of the row (+ action) -> [gradient steps: graph launches]
    host: wait(readback event) only -> env.step on the CPU while the GPU trains -> bookkeeping

Order of effects vs the reference (act / add / env step / add reset rows / train,
``dreamer_v3.py:609-709``): the row a gradient step samples is added before it and the next action
uses the trained weights, as there; the gradient steps are launched BEFORE the env step so the CPU
env step overlaps them.  Divergence: the reset rows (final obs, ``done=1``) of episodes that end at
this env step are added after this step's gradient launch, so they reach training one step later
than in the reference (a sequence sample covers the newest row with probability ~ B*L / buffer
length).  ``algo.interaction_serial_order=True`` (the default since round 5) keeps the reference's order exactly: the
gradient steps run after the env step and the reset rows, and the GPU idles while the CPU steps the env; the
pipelined opt-in measured +1.6 % on the Atari-100k bench in round 6 (three alternating pairs,
``profiles/r6_interaction_drain.md``; round 5: no difference, ``profiles/r5_serial_order.md``).

``last_train_host_s`` is the host time spent inside ``train_fn`` during the last ``step``; callers
timing the env interaction subtract it (the reference times interaction and training separately,
``dreamer_v3.py:592`` vs ``:711``).
"""
from __future__ import annotations

import os
import time
from typing import Any, Callable, Dict, List, Optional, Sequence

import numpy as np
import torch

from sheeprl_prey_amd.data.tensordict import TensorDict

_SPIN = os.environ.get("SRL_SPIN_WAIT", "1") != "0"
# the host polls the action event for at most this long, then blocks on it (a rank whose player sits behind a long
# gradient step does not burn a core that CPU-heavy env workers need)
_SPIN_S = float(os.environ.get("SRL_SPIN_WAIT_MS", "2")) * 1e-3


class InteractionLoop:
    def __init__(self, runner, cfg, envs, player, rb, actions_dim: Sequence[int], is_continuous: bool,
                 clip_rewards: Optional[Callable] = None):
        self.runner, self.cfg, self.envs, self.player, self.rb = runner, cfg, envs, player, rb
        self.actions_dim = list(actions_dim)
        self.is_continuous = is_continuous
        self.clip_rewards = clip_rewards or (lambda r: r)
        self.device = runner.device
        self.ne = int(cfg.env.num_envs)
        self.cnn_keys = list(cfg.cnn_keys.encoder)
        self.mlp_keys = list(cfg.mlp_keys.encoder)
        self.obs_keys = self.cnn_keys + self.mlp_keys
        self.row_keys = self.obs_keys + ["rewards", "dones", "is_first"]
        self.pipelined = self.device.type == "cuda"
        # reference effect order (act, add, env step, add reset rows, train) instead of training before the env step
        self.serial_order = bool(cfg.algo.get("interaction_serial_order", True))
        self.step_data = TensorDict({}, batch_size=[self.ne], device="cpu")
        self._slot = 0
        self._ring: List[Dict[str, torch.Tensor]] = []
        self.last_train_host_s = 0.0
        self.host_ms: Optional[Dict[str, float]] = None  # host-side breakdown of ``step`` when a dict

    # ------------------------------------------------------------------ setup
    def _obs_tensor(self, k: str, v) -> torch.Tensor:
        a = np.asarray(v)
        t = torch.from_numpy(a).view(self.ne, *a.shape[1:])
        return t.float() if k in self.mlp_keys else t

    def reset(self, seed: int) -> None:
        o = self.envs.reset(seed=seed)[0]
        for k in self.obs_keys:
            self.step_data[k] = self._obs_tensor(k, o[k])
        self.step_data["dones"] = torch.zeros(self.ne, 1)
        self.step_data["rewards"] = torch.zeros(self.ne, 1)
        self.step_data["is_first"] = torch.ones(self.ne, 1)
        self.player.init_states()
        if self.pipelined:
            sd = self.step_data
            # one staging row per slot: every row key packed into ONE pinned byte buffer (64-byte aligned views) and a
            # device twin, so a step is one H2D copy; the player reads the observations from the device twin and the
            # replay add is one device-to-device multi-tensor copy from it
            offs, total = {}, 0
            for k in self.row_keys:
                nb = sd[k].numel() * sd[k].element_size()
                offs[k] = (total, nb)
                total += (nb + 63) // 64 * 64
            self._pstage = [torch.empty(total, dtype=torch.uint8).pin_memory() for _ in range(2)]
            self._dstage = [torch.empty(total, dtype=torch.uint8, device=self.device) for _ in range(2)]

            def views(buf):
                return {k: buf[o:o + nb].view(sd[k].dtype).view(sd[k].shape) for k, (o, nb) in offs.items()}

            self._ring = [views(b) for b in self._pstage]
            self._dring = [views(b) for b in self._dstage]
            width = sum(self.actions_dim) if self.is_continuous else len(self.actions_dim)
            dtype = torch.float32 if self.is_continuous else torch.int64
            shape = (self.ne, width) if self.is_continuous else (width, self.ne)
            self._real_pin = torch.empty(shape, dtype=dtype).pin_memory()
            self._h2d = torch.cuda.Stream(device=self.device)
            self._h2d_ev = torch.cuda.Event()
            self._act_ev = torch.cuda.Event()
            rb_dev = getattr(self.rb, "device", None)
            self._rb_on_device = rb_dev is not None and torch.device(rb_dev).type == "cuda"

    # ------------------------------------------------------------------ acting
    def _random_actions(self):
        real = np.array(self.envs.action_space.sample())
        acts = real
        if not self.is_continuous:
            acts = np.concatenate([np.eye(d, dtype=np.float32)[a] for a, d in
                                   zip(real.reshape(len(self.actions_dim), -1), self.actions_dim)], axis=-1)
        return real, acts

    def _policy_serial(self):
        """CPU (or diagnostic) form: pageable copies, blocking readback."""
        pre = {}
        for k in self.obs_keys:
            v = self.step_data[k][None].to(self.device)
            pre[k] = v / 255.0 if k in self.cnn_keys else v
        mask = {k: v for k, v in pre.items() if k.startswith("mask")} or None
        with torch.no_grad():
            actions = self.player.get_exploration_action(pre, self.is_continuous, mask)
        acts = torch.cat(actions, -1).cpu().numpy()
        if self.is_continuous:
            real = acts
        else:
            real = np.array([a.cpu().argmax(dim=-1).numpy() for a in actions])
        return real, acts

    def _policy_pipelined(self) -> None:
        """Stage the row, act, enqueue the row's replay add; the action comes back via ``_real_pin``."""
        slot = self._slot
        b, d = self._ring[slot], self._dring[slot]
        self._slot ^= 1
        for k in self.row_keys:  # slot last read by work enqueued before the previous step's player
            b[k].copy_(self.step_data[k])
        # the slot's device twin was last read two steps ago (that step's player and replay add), which precede the
        # previous step's player, whose readback the host already waited for: the copy may overlap the training
        main = torch.cuda.current_stream(self.device)
        with torch.cuda.stream(self._h2d):
            self._dstage[slot].copy_(self._pstage[slot], non_blocking=True)
            self._h2d_ev.record(self._h2d)
        main.wait_event(self._h2d_ev)
        with torch.no_grad():
            pre = {k: (d[k][None] / 255.0 if k in self.cnn_keys else d[k][None]) for k in self.obs_keys}
            mask = {k: v for k, v in pre.items() if k.startswith("mask")} or None
            actions = self.player.get_exploration_action(pre, self.is_continuous, mask)
            acts = torch.cat(actions, -1).view(self.ne, -1)
            if self.is_continuous:
                self._real_pin.copy_(acts, non_blocking=True)
            else:
                self._real_pin.copy_(torch.stack([a.argmax(-1) for a in actions]).view(len(self.actions_dim), -1),
                                     non_blocking=True)
            self._act_ev.record(main)
        # device-resident replay storage: one device-to-device copy from the twin; host storage (buffer.device=cpu,
        # memmap): the pinned host row (no H2D + blocking D2H round trip)
        if self._rb_on_device:
            row = TensorDict({**{k: d[k] for k in self.row_keys}, "actions": acts}, batch_size=[self.ne])
        else:
            row = TensorDict({**{k: b[k] for k in self.row_keys}, "actions": acts.cpu()}, batch_size=[self.ne])
        self.rb.add(row[None, ...])

    # ------------------------------------------------------------------ one step
    def _timed(self, fn: Optional[Callable[[], Any]]):
        if fn is None:
            return None

        def run():
            t0 = time.perf_counter()
            try:
                return fn()
            finally:
                self.last_train_host_s += time.perf_counter() - t0

        return run

    def step(self, random_actions: bool, train_fn: Optional[Callable[[], Any]] = None) -> Dict[str, Any]:
        """Act (random or policy), add the row, run ``train_fn`` (launched before the env step on the
        GPU path), step the envs.  Returns the env ``infos``."""
        cfg, ne = self.cfg, self.ne
        train_fn = self._timed(train_fn)
        self.last_train_host_s = 0.0
        hp = self.host_ms  # optional host-side breakdown (bench.py SRL_HOST_TIMES=1)
        t0 = time.perf_counter() if hp is not None else 0.0
        deferred = None
        if self.serial_order:
            deferred, train_fn = train_fn, None
        if random_actions:
            real, acts = self._random_actions()
            self.step_data["actions"] = torch.from_numpy(np.asarray(acts, dtype=np.float32)).view(ne, -1)
            self.rb.add(self.step_data[None, ...])
            out = train_fn() if train_fn is not None else None
        elif self.pipelined:
            self._policy_pipelined()
            if hp is not None:
                t1 = time.perf_counter()
                hp["player_launch"] = hp.get("player_launch", 0.0) + (t1 - t0) * 1e3
            out = train_fn() if train_fn is not None else None
            if hp is not None:
                t2 = time.perf_counter()
            if _SPIN:
                # poll (lower wake-up latency than the blocking event wait), bounded by _SPIN_S
                t_end = time.perf_counter() + _SPIN_S
                while not self._act_ev.query():
                    if time.perf_counter() > t_end:
                        self._act_ev.synchronize()
                        break
            else:
                self._act_ev.synchronize()
            if hp is not None:
                t0 = time.perf_counter()
                hp["action_wait"] = hp.get("action_wait", 0.0) + (t0 - t2) * 1e3
            real = self._real_pin.numpy().copy()
        else:
            real, acts = self._policy_serial()
            self.step_data["actions"] = torch.from_numpy(np.asarray(acts, dtype=np.float32)).view(ne, -1)
            self.rb.add(self.step_data[None, ...])
            out = train_fn() if train_fn is not None else None
        self.last_train_out = out

        o, rewards, dones, truncated, infos = self.envs.step(np.asarray(real).reshape(self.envs.action_space.shape))
        dones = np.logical_or(dones, truncated)
        if hp is not None:
            t1 = time.perf_counter()
            hp["env_step"] = hp.get("env_step", 0.0) + (t1 - t0) * 1e3

        sd = self.step_data
        sd["is_first"] = torch.zeros_like(sd["dones"])
        if "restart_on_exception" in infos:
            for i, roe in enumerate(infos["restart_on_exception"]):
                if roe and not dones[i]:
                    b = self.rb.buffer[i]
                    last = (b._pos - 1) % b.buffer_size
                    b["dones"][last] = torch.ones_like(b["dones"][last])
                    b["is_first"][last] = torch.zeros_like(b["is_first"][last])
                    sd["is_first"][i] = torch.ones_like(sd["is_first"][i])

        real_next_obs = {k: np.array(v, copy=True) for k, v in o.items()}
        if "final_observation" in infos:
            for idx, final_obs in enumerate(infos["final_observation"]):
                if final_obs is not None:
                    for k, v in final_obs.items():
                        real_next_obs[k][idx] = v
        for k in self.obs_keys:
            sd[k] = self._obs_tensor(k, o[k])
        r = torch.from_numpy(np.asarray(rewards)).view(ne, -1).float()
        d = torch.from_numpy(np.asarray(dones)).view(ne, -1).float()
        sd["dones"] = d
        sd["rewards"] = self.clip_rewards(r)

        idxes = d.nonzero(as_tuple=True)[0].tolist()
        if idxes:
            n = len(idxes)
            reset = TensorDict({}, batch_size=[n], device="cpu")
            for k in self.obs_keys:
                v = torch.from_numpy(real_next_obs[k][idxes])
                reset[k] = v.float() if k in self.mlp_keys else v
            reset["dones"] = torch.ones(n, 1)
            reset["actions"] = torch.zeros(n, int(np.sum(self.actions_dim)))
            reset["rewards"] = sd["rewards"][idxes].float()
            reset["is_first"] = torch.zeros_like(reset["dones"])
            self.rb.add(reset[None, ...], idxes)
            sd["rewards"][idxes] = 0.0
            sd["dones"][idxes] = 0.0
            sd["is_first"][idxes] = 1.0
            self.player.init_states(idxes)
        if hp is not None:
            t0 = time.perf_counter()
            hp["bookkeeping"] = hp.get("bookkeeping", 0.0) + (t0 - t1) * 1e3
        if deferred is not None:
            self.last_train_out = deferred()
        if hp is not None:
            hp["train_launch"] = hp.get("train_launch", 0.0) + (time.perf_counter() - t0) * 1e3
            hp["steps"] = hp.get("steps", 0) + 1
        return infos
