"""MineRL 0.4.4 adapter (reference ``sheeprl/envs/minerl.py:1-321``).

MineRL's dict action space is flattened into one ``Discrete`` action: index 0 is no-op, then one
index per binary key, four camera moves (+-15 degrees pitch/yaw) and one index per non-"none" value
of every enum action; jump / sneak / sprint also press forward.  Sticky attack / jump keep those
keys pressed for a number of steps; pitch is clamped to ``pitch_limits``.  Observations: ``rgb``
(CHW), ``life_stats``, (max-)``inventory`` counts, optional ``equipment`` one-hot and ``compass``.
"""
from __future__ import annotations

import copy
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

from sheeprl_prey_amd.envs import spaces
from sheeprl_prey_amd.envs._gate import require
from sheeprl_prey_amd.envs.core import Env

NOOP: Dict[str, Any] = {"camera": (0, 0), "forward": 0, "back": 0, "left": 0, "right": 0, "attack": 0, "sprint": 0,
                        "jump": 0, "sneak": 0, "craft": "none", "nearbyCraft": "none", "nearbySmelt": "none",
                        "place": "none", "equip": "none"}
CAMERA_MOVES = [np.array([-15, 0]), np.array([15, 0]), np.array([0, -15]), np.array([0, 15])]


def build_action_map(action_keys: Sequence[Tuple[str, Optional[Sequence[str]]]]) -> List[Dict[str, Any]]:
    """``action_keys``: (name, enum values or None) in MineRL's action-space order ->
    list of partial MineRL actions, index = discrete action."""
    table: List[Dict[str, Any]] = [{}]
    for name, values in action_keys:
        if values is not None:
            for v in sorted(set(values) - {"none"}):
                table.append({name: v})
        elif name == "camera":
            table.extend({"camera": m} for m in CAMERA_MOVES)
        else:
            entry = {name: 1}
            if name in ("jump", "sneak", "sprint"):
                entry["forward"] = 1
            table.append(entry)
    return table


class StickyKeys:
    """Keeps ``attack`` / ``jump`` pressed for ``sticky_*`` steps after being selected."""

    def __init__(self, sticky_attack: Optional[int] = 30, sticky_jump: Optional[int] = 10):
        self.sticky_attack = sticky_attack or 0
        self.sticky_jump = sticky_jump or 0
        self.reset()

    def reset(self) -> None:
        self.attack_left = self.jump_left = 0

    def __call__(self, act: Dict[str, Any]) -> Dict[str, Any]:
        if self.sticky_attack:
            if act["attack"]:
                self.attack_left = self.sticky_attack
            if self.attack_left > 0:
                act["attack"], act["jump"] = 1, 0
                self.attack_left -= 1
        if self.sticky_jump:
            if act["jump"]:
                self.jump_left = self.sticky_jump
            if self.jump_left > 0:
                act["jump"], act["forward"] = 1, 1
                self.jump_left -= 1
        return act


class MineRLWrapper(Env):
    def __init__(self, id: str, height: int = 64, width: int = 64, pitch_limits: Tuple[int, int] = (-60, 60),
                 seed: Optional[int] = None, sticky_attack: Optional[int] = 30, sticky_jump: Optional[int] = 10,
                 break_speed_multiplier: Optional[int] = 100, multihot_inventory: bool = True, **kwargs: Any):
        require("minerl", "Install minerl==0.4.4 to use `env=minerl`.")
        from minerl.herobraine.hero import mc
        from minerl.herobraine.hero import spaces as mspaces

        from sheeprl_prey_amd.envs.minerl_specs import make_spec, task_kwargs

        self._pitch_limits = pitch_limits
        self.sticky = StickyKeys(sticky_attack, sticky_jump)
        self._env = make_spec(id, break_speed=break_speed_multiplier, resolution=(height, width),
                              **task_kwargs(id, kwargs)).make()
        aspace = self._env.action_space
        keys = [(k, aspace[k].values.tolist() if isinstance(aspace[k], mspaces.Enum) else None) for k in aspace]
        self.action_table = build_action_map(keys)
        self.action_space = spaces.Discrete(len(self.action_table))
        ospace = self._env.observation_space
        all_items = list(mc.ALL_ITEMS)
        if multihot_inventory:
            self.inv_index = {n: i for i, n in enumerate(all_items)}
            self.equip_index = self.inv_index
        else:
            self.inv_index = {n: i for i, n in enumerate(ospace["inventory"])}
            if "equipped_items" in ospace.spaces:
                self.equip_index = {n: i for i, n in
                                    enumerate(ospace["equipped_items"]["mainhand"]["type"].values.tolist())}
        n_inv = len(self.inv_index)
        obs = {"rgb": spaces.Box(0, 255, (3, height, width), np.uint8),
               "life_stats": spaces.Box(0.0, np.array([20.0, 20.0, 300.0]), (3,), np.float32),
               "inventory": spaces.Box(0.0, np.inf, (n_inv,), np.float32),
               "max_inventory": spaces.Box(0.0, np.inf, (n_inv,), np.float32)}
        if "compass" in ospace.spaces:
            obs["compass"] = spaces.Box(-180, 180, (1,), np.float32)
        if "equipped_items" in ospace.spaces:
            obs["equipment"] = spaces.Box(0, 1, (len(self.equip_index),), np.int32)
        self.observation_space = spaces.Dict(obs)
        self._max_inventory = np.zeros(n_inv)
        self._pos = {"pitch": 0.0, "yaw": 0.0}
        self.render_mode = "rgb_array"
        self.action_space.seed(seed)

    def _convert_action(self, action) -> Dict[str, Any]:
        act = copy.deepcopy(NOOP)
        act.update(self.action_table[int(np.asarray(action).reshape(-1)[0])])
        return self.sticky(act)

    def _convert_obs(self, obs: Dict[str, Any]) -> Dict[str, np.ndarray]:
        inv = np.zeros(len(self.inv_index))
        for item, q in obs["inventory"].items():
            inv[self.inv_index[item]] += 1 if item == "air" else q
        self._max_inventory = np.maximum(inv, self._max_inventory)
        ls = obs["life_stats"]
        out = {"rgb": obs["pov"].copy().transpose(2, 0, 1),
               "life_stats": np.array([ls["life"], ls["food"], ls["air"]], dtype=np.float32),
               "inventory": inv, "max_inventory": self._max_inventory.copy()}
        if "equipment" in self.observation_space.spaces:
            e = np.zeros(len(self.equip_index), dtype=np.int32)
            e[self.equip_index.get(obs["equipped_items"]["mainhand"]["type"], self.equip_index["air"])] = 1
            out["equipment"] = e
        if "compass" in self.observation_space.spaces:
            out["compass"] = np.asarray(obs["compass"]["angle"]).reshape(-1)
        return out

    def step(self, action):
        act = self._convert_action(action)
        pitch = self._pos["pitch"] + act["camera"][0]
        yaw = ((self._pos["yaw"] + act["camera"][1]) + 180) % 360 - 180
        if not (self._pitch_limits[0] <= pitch <= self._pitch_limits[1]):
            act["camera"] = np.array([0, act["camera"][1]])
            pitch = self._pos["pitch"]
        obs, reward, done, _ = self._env.step(act)
        self._pos = {"pitch": pitch, "yaw": yaw}
        return self._convert_obs(obs), reward, done, False, {}

    def reset(self, seed: Optional[int] = None, options: Optional[Dict[str, Any]] = None):
        obs = self._env.reset()
        self._max_inventory = np.zeros(len(self.inv_index))
        self.sticky.reset()
        self._pos = {"pitch": 0.0, "yaw": 0.0}
        return self._convert_obs(obs), {}

    def render(self, mode: Optional[str] = "rgb_array"):
        return self._env.render(self.render_mode)

    def close(self) -> None:
        self._env.close()
