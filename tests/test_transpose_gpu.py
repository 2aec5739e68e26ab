"""Batched transpose (csrc/transpose.hip, ops.transpose_many) vs ``.t().contiguous()``: ragged shapes, column
slices of wider weights, preallocated row-block destinations."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_transpose_many_matches_torch():
    from sheeprl_prey_amd import ops

    g = torch.Generator(device="cuda").manual_seed(0)
    W = torch.randn(512, 1030, device="cuda", generator=g)
    xs = [W[:, :1024], W[:, 1024:], torch.randn(1536, 1024, device="cuda", generator=g),
          torch.randn(33, 65, device="cuda", generator=g), torch.randn(1, 7, device="cuda", generator=g)]
    outs = ops.transpose_many(xs)
    for x, y in zip(xs, outs):
        assert y.is_contiguous() and y.shape == (x.shape[1], x.shape[0])
        assert torch.equal(y, x.t())


def test_transpose_many_into_row_blocks():
    from sheeprl_prey_amd import ops

    g = torch.Generator(device="cuda").manual_seed(1)
    W = torch.randn(512, 1024 + 9, device="cuda", generator=g)
    table = torch.empty(1024 + 9, 512, device="cuda")
    res = ops.transpose_many([W[:, 1024:], W[:, :1024]], [table[:9], table[9:]])
    assert res[0].data_ptr() == table.data_ptr()
    assert torch.equal(table, torch.cat((W[:, 1024:], W[:, :1024]), 1).t())
