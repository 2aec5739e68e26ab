"""Replay-buffer semantics (behaviour pinned by the reference's ``tests/test_data/*``)."""
from __future__ import annotations

import os

import numpy as np
import pytest
import torch

from sheeprl_prey_amd.data.buffers import AsyncReplayBuffer, EpisodeBuffer, ReplayBuffer, SequentialReplayBuffer
from sheeprl_prey_amd.data.tensordict import TensorDict


def td(n, n_envs=1, key="t", fill=None):
    v = torch.rand(n, n_envs, 1) if fill is None else fill.view(n, n_envs, 1)
    return TensorDict({key: v}, batch_size=[n, n_envs])


# ---------------------------------------------------------------- ReplayBuffer
@pytest.mark.parametrize("args", [(-1,), (1, -1), (0,)])
def test_rb_bad_sizes(args):
    with pytest.raises(ValueError):
        ReplayBuffer(*args)


def test_rb_add_partial():
    rb = ReplayBuffer(5, 1)
    a = td(2)
    rb.add(a)
    assert not rb.full and rb._pos == 2
    torch.testing.assert_close(rb["t"][:2], a["t"])


def test_rb_wraparound_sequence():
    rb = ReplayBuffer(5, 1)
    a, b, c = td(2), td(2), td(3)
    for x in (a, b, c):
        rb.add(x)
    assert rb.full and rb._pos == 2
    torch.testing.assert_close(rb["t"][0], c["t"][-2])
    torch.testing.assert_close(rb["t"][1], c["t"][-1])
    torch.testing.assert_close(rb["t"][2:4], b["t"])


@pytest.mark.parametrize("n,size,pos", [(17, 5, 2), (20, 5, 0), (9, 7, 2)])
def test_rb_single_add_larger_than_buffer(n, size, pos):
    rb = ReplayBuffer(size, 1)
    x = td(n)
    rb.add(x)
    assert rb.full and rb._pos == pos
    # the buffer holds the LAST `size` rows, rotated so that row i sits at (i mod size)
    last = x["t"][-size:]
    for j in range(size):
        row = (n - size + j) % size
        torch.testing.assert_close(rb["t"][row], last[j])


def test_rb_sample_shapes():
    rb = ReplayBuffer(5, 2)
    rb.add(td(6, 2))
    s = rb.sample(4)
    assert tuple(s.shape) == (4, 1)
    s = rb.sample(7)
    assert tuple(s.shape) == (7, 1)


def test_rb_sample_next_obs_excludes_write_head():
    for n in (4, 8):
        rb = ReplayBuffer(5, 1, obs_keys=("observations",))
        x = td(n, key="observations", fill=torch.arange(n, dtype=torch.float32))
        rb.add(x)
        s = rb.sample(64, sample_next_obs=True)
        assert tuple(s.shape) == (64, 1)
        assert float(x["observations"][-1]) not in s["observations"].flatten().tolist()
        torch.testing.assert_close(s["next_observations"], s["observations"] + 1)


def test_rb_one_element():
    rb = ReplayBuffer(1, 1, obs_keys=("observations",))
    x = td(1, key="observations")
    rb.add(x)
    assert rb.full
    torch.testing.assert_close(rb.sample(1)["observations"].view(-1), x["observations"].view(-1))
    with pytest.raises(RuntimeError):
        rb.sample(1, sample_next_obs=True)


def test_rb_sample_errors():
    rb = ReplayBuffer(1, 1)
    with pytest.raises(ValueError, match="No sample has been added"):
        rb.sample(1)
    rb.add(td(1))
    with pytest.raises(ValueError, match="Batch size must be greater than 0"):
        rb.sample(-1)


def test_rb_memmap_default_dir_warns():
    with pytest.warns(UserWarning, match="memory-mapped into the `/tmp` folder"):
        rb = ReplayBuffer(10, 4, memmap=True, memmap_dir=None)
    rb.add(TensorDict({"observations": torch.randint(0, 256, (10, 4, 3, 8, 8), dtype=torch.uint8)},
                      batch_size=[10, 4]))
    assert rb.is_memmap


def test_rb_memmap_to_dir(tmp_path):
    d = tmp_path / "memmap_buffer"
    rb = ReplayBuffer(10, 4, memmap=True, memmap_dir=str(d))
    obs = torch.randint(0, 256, (10, 4, 3, 8, 8), dtype=torch.uint8)
    rb.add(TensorDict({"observations": obs}, batch_size=[10, 4]))
    assert rb.is_memmap
    assert any(os.scandir(d))
    torch.testing.assert_close(rb["observations"], obs)


def test_rb_state_dict_roundtrip():
    rb = ReplayBuffer(6, 2)
    rb.add(td(9, 2))
    sd = rb.state_dict()
    rb2 = ReplayBuffer(6, 2)
    rb2.load_state_dict(sd)
    assert rb2._pos == rb._pos and rb2.full == rb.full
    torch.testing.assert_close(rb2["t"], rb["t"])


# ---------------------------------------------------------------- SequentialReplayBuffer
def test_seq_shapes_and_contiguity():
    rb = SequentialReplayBuffer(20, 3)
    rb.add(td(20, 3, fill=torch.arange(60, dtype=torch.float32)))
    s = rb.sample(4, sequence_length=5, n_samples=2)
    assert tuple(s.shape) == (2, 5, 4)
    v = s["t"].squeeze(-1)  # [n, L, B]; stored value = 3*row + env
    diffs = v[:, 1:] - v[:, :-1]
    assert torch.all((diffs == 3) | (diffs == 3 - 60))


def test_seq_never_crosses_write_head():
    rb = SequentialReplayBuffer(10, 1)
    rb.add(td(13, 1, fill=torch.arange(13, dtype=torch.float32)))  # full, head at 3
    s = rb.sample(256, sequence_length=4)
    v = s["t"].squeeze(-1)
    assert torch.all(v[:, 1:] - v[:, :-1] == 1)  # consecutive in insertion order


def test_seq_errors():
    rb = SequentialReplayBuffer(10, 1)
    with pytest.raises(ValueError):
        rb.sample(2, sequence_length=2)
    rb.add(td(3))
    with pytest.raises(ValueError):
        rb.sample(2, sequence_length=5)  # not enough data
    with pytest.raises(ValueError):
        rb.sample(0, sequence_length=2)


# ---------------------------------------------------------------- EpisodeBuffer
def episode(n, start=0.0):
    d = torch.zeros(n, 1, 1)
    d[-1] = 1
    return TensorDict({"t": torch.arange(start, start + n).view(n, 1, 1), "dones": d}, batch_size=[n, 1])


def test_episode_buffer_args():
    with pytest.raises(ValueError):
        EpisodeBuffer(-1, 2)
    with pytest.raises(ValueError):
        EpisodeBuffer(5, -1)
    with pytest.raises(ValueError):
        EpisodeBuffer(2, 5)


def test_episode_buffer_add_and_evict():
    eb = EpisodeBuffer(10, 2)
    eb.add(episode(4))
    eb.add(episode(5, 100))
    assert len(eb) == 9 and eb.full  # full == no room for another sequence_length-long episode
    eb.add(episode(6, 200))  # must evict the oldest episode(s)
    assert len(eb) <= 10
    assert float(eb.buffer[-1]["t"][0]) == 200.0


def test_episode_buffer_rejects_bad_episodes():
    eb = EpisodeBuffer(10, 3)
    with pytest.raises(RuntimeError):
        eb.add(episode(2))  # shorter than the sequence length
    bad = episode(4)
    bad["dones"][-1] = 0
    with pytest.raises(RuntimeError):
        eb.add(bad)  # episode must end with done


def test_episode_buffer_sample_shapes_and_ends():
    eb = EpisodeBuffer(30, 3)
    for i in range(3):
        eb.add(episode(7, 10 * i))
    s = eb.sample(5, n_samples=2)
    assert tuple(s.shape) == (2, 3, 5)
    v = s["t"].squeeze(-1)
    assert torch.all(v[:, 1:] - v[:, :-1] == 1)
    s = eb.sample(64, prioritize_ends=True)
    assert tuple(s.shape)[1:] == (3, 64)


def test_episode_buffer_errors():
    eb = EpisodeBuffer(10, 2)
    with pytest.raises(RuntimeError):
        eb.sample(2)
    eb.add(episode(3))
    with pytest.raises(ValueError):
        eb.sample(0)


# ---------------------------------------------------------------- AsyncReplayBuffer
def test_async_buffer_per_env_and_reset_rows():
    rb = AsyncReplayBuffer(16, 2, sequential=True)
    for i in range(10):
        rb.add(TensorDict({"t": torch.full((1, 2, 1), float(i))}, batch_size=[1, 2]))
    # env 1 only
    rb.add(TensorDict({"t": torch.full((1, 1, 1), 99.0)}, batch_size=[1, 1]), indices=[1])
    assert rb.buffer[0]._pos == 10 and rb.buffer[1]._pos == 11
    s = rb.sample(3, sequence_length=4, n_samples=2)
    assert tuple(s.shape) == (2, 4, 3)
    sd = rb.state_dict()
    rb2 = AsyncReplayBuffer(16, 2, sequential=True)
    rb2.load_state_dict(sd)
    torch.testing.assert_close(rb2.buffer[1]["t"], rb.buffer[1]["t"])


def test_replay_buffer_whole_buffer_adds_after_full():
    """Adding exactly ``buffer_size`` rows again once full (PPO with env.device=True adds a whole
    rollout per update) overwrites every row instead of storing nothing."""
    rb = ReplayBuffer(4, 2, device="cpu")
    for i in range(3):
        rb.add(TensorDict({"a": torch.full((4, 2, 1), float(i))}, batch_size=[4, 2]))
        assert rb["a"].eq(float(i)).all() and rb._pos == 0 and rb.full
    rb.add(TensorDict({"a": torch.full((1, 2, 1), 9.0)}, batch_size=[1, 2]))
    rb.add(TensorDict({"a": torch.arange(4.0).view(4, 1, 1).expand(4, 2, 1)}, batch_size=[4, 2]))
    assert rb["a"][:, 0, 0].tolist() == [3.0, 0.0, 1.0, 2.0] and rb._pos == 1


@pytest.mark.parametrize("serial", [False, True])
def test_dv3_interaction_order_of_reset_rows(serial):
    """``InteractionLoop`` effect order (reference ``dreamer_v3.py:609-709``: act, add the row, env step, add the
    reset rows of finished episodes, then train).  The default launches the gradient steps before the env step
    (so they overlap it): the reset row of an episode ending at this step reaches the replay buffer after that
    step's training.  ``algo.interaction_serial_order=True`` gives the reference order: training sees it."""
    from sheeprl_prey_amd.algos.dreamer_v3.interaction import InteractionLoop
    from sheeprl_prey_amd.config.compose import compose
    from sheeprl_prey_amd.data.buffers import AsyncReplayBuffer
    from sheeprl_prey_amd.parallel.runner import Runner
    from sheeprl_prey_amd.utils.env import make_env, make_vector_env
    from sheeprl_prey_amd.utils.utils import dotdict

    cfg = dotdict(compose(["exp=dreamer_v3", "env=dummy", "env.id=discrete_dummy", "env.num_envs=1", "env.sync_env=True",
                           "env.capture_video=False", "cnn_keys.encoder=[rgb]", f"algo.interaction_serial_order={serial}"]))
    runner = Runner(accelerator="cpu")
    envs = make_vector_env(cfg, [make_env(cfg, 0, 0, None, "train", 0)])

    class _Player:
        def init_states(self, *a):
            pass

    rb = AsyncReplayBuffer(64, 1, device="cpu", sequential=True)
    loop = InteractionLoop(runner, cfg, envs, _Player(), rb, [2], False)
    loop.reset(0)
    seen = []

    def train():
        b = rb.buffer[0]
        seen.append(float(b["dones"][: b._pos].sum()))
        return None

    for _ in range(5):  # the dummy episode ends at the 5th env step (4 steps + the terminal one)
        loop.step(True, train)
    envs.close()
    # dones rows in the buffer when the 5th step's training ran: the reset row only in the serial order
    assert seen[-1] == (1.0 if serial else 0.0), seen


def test_sequential_buffer_sampler_stream_survives_checkpoint():
    """The device-side sampler's (seed, counter) travel with the buffer's state_dict, so a resumed run continues
    the index stream instead of replaying the first draws of the original run."""
    from sheeprl_prey_amd.data.buffers import SequentialReplayBuffer
    from sheeprl_prey_amd.data.tensordict import TensorDict

    rb = SequentialReplayBuffer(8, 1)
    rb.add(TensorDict({"a": torch.arange(4.0).view(4, 1, 1)}, batch_size=[4, 1]))
    rb._draw_seed, rb._draw_counter = 1234567, 42
    rb2 = SequentialReplayBuffer(8, 1)
    rb2.load_state_dict(rb.state_dict())
    assert (rb2._draw_seed, rb2._draw_counter) == (1234567, 42)
