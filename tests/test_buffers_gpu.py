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
