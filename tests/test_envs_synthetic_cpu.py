"""Synthetic Atari-shaped env (envs/synthetic.py): the scalar-sprite fast path reproduces the original numpy
implementation bit for bit (checksums of 300 steps recorded with the round-3 implementation, seed 7)."""
import hashlib

import numpy as np
import pytest

from sheeprl_prey_amd.envs.synthetic import SyntheticAtari


@pytest.mark.parametrize("gray,size,digest,reward", [(True, 84, "aa76bbd236402b3e", 2.0), (False, 64, "ce6d17d653a9239d", 10.0)])
def test_synthetic_atari_frames_match_recorded_checksums(gray, size, digest, reward):
    e = SyntheticAtari("PongNoFrameskip-v4", screen_size=size, grayscale=gray)
    f, _ = e.reset(seed=7)
    assert f.shape == (size, size, 1 if gray else 3) and f.dtype == np.uint8
    h = hashlib.sha256(f.tobytes())
    tot = 0.0
    rng = np.random.default_rng(0)
    for _ in range(300):
        o, r, term, trunc, _ = e.step(int(rng.integers(0, 6)))
        assert not term and not trunc
        h.update(o.tobytes())
        tot += r
    assert h.hexdigest()[:16] == digest
    assert tot == reward


def test_synthetic_atari_truncates_and_resets():
    e = SyntheticAtari("MsPacmanNoFrameskip-v4", screen_size=64, episode_length=5)
    e.reset(seed=1)
    outs = [e.step(0) for _ in range(5)]
    assert [o[3] for o in outs] == [False] * 4 + [True]
    f1, _ = e.reset(seed=1)
    f2, _ = SyntheticAtari("MsPacmanNoFrameskip-v4", screen_size=64).reset(seed=1)
    assert np.array_equal(f1, f2)


def test_synthetic_control_states_renders_and_rewards_pinned():
    """The walker_walk-shaped control env (SyntheticControl): states, renders and rewards of 100 seeded steps pinned
    by checksum (its render caches the tiled floor, which equals the per-call formula it replaced)."""
    from sheeprl_prey_amd.envs.synthetic import SyntheticControl

    e = SyntheticControl(seed=3)
    e.reset(seed=3)
    h = hashlib.sha256(e.render().tobytes())
    tot = 0.0
    rng = np.random.default_rng(0)
    for _ in range(100):
        o, r, term, trunc, _ = e.step(rng.uniform(-1, 1, 6))
        tot += r
        h.update(o.tobytes())
        h.update(e.render().tobytes())
    assert h.hexdigest()[:16] == "11bd4e172c8f129d"
    assert abs(tot - 47.48275099571548) < 1e-9
    s = e.size
    yy, xx = np.mgrid[0:s, 0:s]
    assert np.array_equal(e._floor, np.repeat((((xx // 8 + yy // 8) % 2) * 30 + 40).astype(np.uint8)[..., None], 3, -1))
