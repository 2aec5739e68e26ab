"""K21: HBM-resident sequential replay sampling with the one-launch multi-key row gather
(``gather.hip``) vs the ATen index path, same draws."""
import pytest
import torch

from sheeprl_prey_amd import ops
from sheeprl_prey_amd.data.buffers import AsyncReplayBuffer, SequentialReplayBuffer
from sheeprl_prey_amd.data.tensordict import TensorDict

pytestmark = pytest.mark.gpu


def _fill(rb, steps, n_envs):
    for t in range(steps):
        rb.add(TensorDict({
            "rgb": torch.randint(0, 256, (1, n_envs, 3, 8, 8), dtype=torch.uint8, device="cuda"),
            "actions": torch.randn(1, n_envs, 5, device="cuda"),
            "rewards": torch.randn(1, n_envs, 1, device="cuda"),
            "odd": torch.randint(0, 256, (1, n_envs, 3), dtype=torch.uint8, device="cuda"),  # 3-byte rows
        }, batch_size=[1, n_envs], device="cuda"))


@pytest.mark.parametrize("n_envs,full", [(1, False), (3, True)])
def test_sequential_gather_kernel_matches_index_path(n_envs, full):
    rb = SequentialReplayBuffer(40, n_envs, device="cuda")
    _fill(rb, 55 if full else 30, n_envs)
    torch.manual_seed(5)
    a = rb.sample(6, sequence_length=9, n_samples=2)
    ops.set_fused(False)
    try:
        torch.manual_seed(5)
        b = rb.sample(6, sequence_length=9, n_samples=2)
    finally:
        ops.set_fused(True)
    assert a.shape == b.shape == torch.Size([2, 9, 6])
    for k in b.keys():
        assert torch.equal(a[k], b[k]), k


def test_async_single_env_sample_has_no_concat_copy():
    rb = AsyncReplayBuffer(32, 1, device="cuda", sequential=True)
    _fill(rb, 20, 1)
    s = rb.sample(4, sequence_length=5, n_samples=1)
    assert s["rgb"].shape == (1, 5, 4, 3, 8, 8) and s["rgb"].dtype == torch.uint8


@pytest.mark.parametrize("full", [False, True])
def test_sequential_sample_into_fused(full):
    """The one-launch device-side sample (gather.hip seq_sample_kernel) writes consecutive rows of one env per
    sample, starting only at valid starts, identically for every key, into [L, B, ...] outputs."""
    from sheeprl_prey_amd.data.buffers import SequentialReplayBuffer
    from sheeprl_prey_amd.data.tensordict import TensorDict

    cap, n_envs, L, B = 64, 3, 8, 256
    rb = SequentialReplayBuffer(cap, n_envs, device="cuda")
    steps = cap + 10 if full else 30
    for t in range(steps):
        row = torch.arange(n_envs, dtype=torch.float32).view(1, n_envs, 1) + 100.0 * t
        rb.add(TensorDict({"a": row, "img": (torch.full((1, n_envs, 2, 4, 4), t % 251, dtype=torch.uint8))},
                          batch_size=[1, n_envs]))
    out = {"a": torch.empty(L, B, 1, device="cuda"), "img": torch.empty(L, B, 2, 4, 4, dtype=torch.uint8, device="cuda")}
    assert rb.sample_into(out, B, L)
    a = out["a"][..., 0].cpu()  # [L, B]: 100 * step + env
    step = torch.div(a, 100, rounding_mode="floor").long()
    env = (a - 100 * step).long()
    assert torch.all(env == env[0:1]), "one env per sample"
    assert torch.all((env >= 0) & (env < n_envs))
    assert torch.all(step[1:] - step[:-1] == 1), "consecutive steps"
    assert torch.equal(out["img"][:, :, 0, 0, 0].cpu().long(), step % 251), "keys gathered from the same rows"
    if full:
        # never across the write head: every sequence ends at or before the newest row
        assert torch.all(step[-1] <= steps - 1) and torch.all(step[0] >= steps - cap)
    else:
        assert torch.all(step[0] >= 0) and torch.all(step[-1] <= steps - 1)
    first = step[0]
    assert first.unique().numel() > 5, "starts are drawn, not constant"
    # a second call draws new starts
    prev = out["a"].clone()
    assert rb.sample_into(out, B, L)
    assert not torch.equal(prev, out["a"])
