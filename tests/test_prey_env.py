"""Native predator-prey cellworld (``prey_d_1``): spaces, dynamics, rewards, determinism, and the
DreamerV3 prey preset + evaluation entry point end to end (CPU)."""
from __future__ import annotations

import math
import os
from pathlib import Path
from unittest import mock

import numpy as np
import pytest

from sheeprl_prey_amd.envs.prey.env import PreyEnv
from sheeprl_prey_amd.envs.prey.world import CELL_SIZE, HexWorld, get_world
from sheeprl_prey_amd.envs.registry import make


def test_spaces_and_reset():
    env = make("prey_d_1")
    assert env.observation_space.shape == (14,) and env.action_space.n == 100
    o, info = env.reset(seed=0)
    assert o.shape == (14,) and o.dtype == np.float32
    np.testing.assert_allclose(o[:3], [0.0, 0.5, math.pi / 2], atol=1e-6)
    assert o[3] == 0 and o[4] == 0


def test_action_grid_mapping():
    env = PreyEnv()
    assert env.map_discrete_to_continuous(0) == (-1.0, -1.0)
    assert env.map_discrete_to_continuous(99) == (1.0, 1.0)
    s, t = env.map_discrete_to_continuous(94)
    assert s == 1.0 and abs(t - (-1 + 4 * 2 / 9)) < 1e-9


def test_world_generation_deterministic_and_connected():
    a, b = HexWorld("03_05"), HexWorld("03_05")
    assert a.n == 331
    np.testing.assert_array_equal(a.occluded, b.occluded)
    assert HexWorld("03_01").occluded.sum() < HexWorld("03_09").occluded.sum()
    w = get_world("00_03")
    start, goal = w.cell_of(np.array([0.0, 0.5])), w.cell_of(np.array([1.0, 0.5]))
    assert not w.occluded[start] and not w.occluded[goal]
    p = w.path(start, goal)
    assert p[0] == start and p[-1] == goal  # goal reachable


def test_visibility_is_symmetric_and_blocked_by_occlusions():
    w = get_world("05_07")
    rng = np.random.default_rng(0)
    pts = w.centers[w.free][rng.choice(len(w.free), 40, replace=False)]
    for i in range(0, 40, 2):
        assert w.is_visible(pts[i], pts[i + 1]) == w.is_visible(pts[i + 1], pts[i])
    mask = w.visible_mask(pts[0], pts)
    assert mask.dtype == bool and mask[0]
    assert all(mask[j] == w.is_visible(pts[0], pts[j]) for j in range(40))
    occ = w.occ_centers[0]
    assert not w.is_valid_location(occ)


def test_same_seed_same_episode():
    def rollout():
        env = PreyEnv(e=4)
        env.reset(seed=7)
        out = []
        for k in range(60):
            o, r, d, t, _ = env.step((k * 37) % 100)
            out.append((o.copy(), r))
            if d or t:
                break
        return out

    a, b = rollout(), rollout()
    assert len(a) == len(b)
    for (oa, ra), (ob, rb) in zip(a, b):
        np.testing.assert_array_equal(oa, ob)
        assert ra == rb


def test_goal_reward_and_time_limit():
    env = PreyEnv(has_predator=False, max_step=5)
    env.reset(seed=0)
    env.prey["loc"] = np.array([1.0 - CELL_SIZE * 0.5, 0.5])
    o, r, d, t, info = env.step(99 - 5)  # full speed, straight
    assert d and r == 100 and info["is success"]
    env.reset(seed=0)
    rewards = []
    for _ in range(10):
        o, r, d, t, _ = env.step(45)  # ~zero speed
        rewards.append(r)
        if t:
            break
    assert t and len(rewards) == 5 and all(x < 0 for x in rewards)


def test_capture_truncates_with_penalty():
    env = PreyEnv(has_predator=True)
    env.reset(seed=1)
    env.pred["loc"] = env.prey["loc"] + np.array([CELL_SIZE * 0.3, 0.0])
    o, r, d, t, info = env.step(45)
    assert t and r == -50 and info["is truncated"]


def test_render_rgb():
    env = PreyEnv(render_mode="rgb_array", render_size=64)
    env.reset(seed=0)
    img = env.render()
    assert img.shape == (64, 64, 3) and img.dtype == np.uint8


@pytest.mark.timeout(240)
def test_dreamer_v3_prey_preset_and_evaluate():
    from sheeprl_prey_amd.cli import run
    from sheeprl_prey_amd.evaluate import evaluate

    with mock.patch.dict(os.environ, {"LT_ACCELERATOR": "cpu", "LT_DEVICES": "1"}):
        run(["exp=dreamer_v3_prey", "dry_run=True", "env.num_envs=1", "env.sync_env=True", "env.capture_video=False",
             "per_rank_batch_size=1", "per_rank_sequence_length=1", "buffer.size=2", "algo.learning_starts=0",
             "algo.horizon=4", "root_dir=prey", "run_name=t", "algo.dense_units=8",
             "algo.world_model.recurrent_model.recurrent_state_size=8",
             "algo.world_model.representation_model.hidden_size=8", "algo.world_model.transition_model.hidden_size=8"])
    ck = sorted(Path("logs", "runs", "prey", "t").rglob("*.ckpt"))[-1]
    rets = evaluate(str(ck), ["env.env_type=test"], episodes=2, render=True)
    assert len(rets) == 2
    assert list((ck.parent / "eval_videos").glob("*.gif"))


def test_observation_and_reward_contract_of_reference_step():
    """Pins the per-step contract of the reference ``prey_env/envs/gymnasium_env_bins.py:152-232``:
    obs = [prey x, y, theta, speed, turning, predator x, y, theta (-1, -1, 0 when not visible),
    3 x (distance, angle) of the nearest occlusions]; reward = -|prey - (1, 0.5)| off the goal."""
    env = PreyEnv()
    o, _ = env.reset(seed=3)
    rng = np.random.default_rng(0)
    for _ in range(40):
        a = int(rng.integers(100))
        o, r, done, trunc, info = env.step(a)
        speed, turning = env.map_discrete_to_continuous(a)
        assert o.shape == (14,) and o.dtype == np.float32
        np.testing.assert_allclose(o[3:5], [speed, turning], atol=1e-6)
        if o[5] == -1.0 and o[6] == -1.0:
            assert o[7] == 0.0  # predator not visible
        assert np.all(o[8::2] >= 0)  # occlusion distances
        if not done and not trunc:
            assert abs(r - (-math.hypot(o[0] - 1.0, o[1] - 0.5))) < 1e-5
        if done or trunc:
            break
