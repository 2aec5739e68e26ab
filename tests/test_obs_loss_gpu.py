"""Fused vector-encoder input (ops.symlog_cat, csrc/obs_loss.hip symlog_cat_kernel) against the torch composite of the
reference MLPEncoder (dreamer_v3/agent.py: cat of symlog(obs[k]) over the keys)."""
import pytest
import torch

from sheeprl_prey_amd import ops

pytestmark = pytest.mark.gpu


def test_symlog_cat_matches_eager():
    """The vector encoder's input (cat of symlog(obs[k]) over the keys) in one launch vs the torch ops, incl. zeros and
    negative / large values."""
    from sheeprl_prey_amd.utils.utils import symlog

    g = torch.Generator(device="cuda").manual_seed(3)
    xs = [torch.randn(5, 7, d, device="cuda", generator=g) * 30 for d in (24, 1, 9)]
    xs[0][0, 0, :4] = torch.tensor([0.0, -0.0, 1e-7, -1e6])
    out = ops.symlog_cat(xs)
    ref = torch.cat([symlog(x) for x in xs], -1)
    assert out.shape == ref.shape == (5, 7, 34)
    torch.testing.assert_close(out, ref, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(ops.symlog_cat(xs[:1]), symlog(xs[0]), rtol=1e-6, atol=1e-6)
