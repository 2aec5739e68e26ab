"""DreamerV3 critic objective kernel (csrc/dist.hip value_loss2_kernel: both two-hot NLL terms, the discount weights
and the mean in one pass, the logits gradient written in the same pass) against the composite of the reference
(dreamer_v3.py:327-336: TwoHotEncodingDistribution log-probs of the lambda returns and of the target critic's values,
discount-weighted mean) in fp64."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("T,M,K,spread", [(15, 1024, 255, 3.0), (4, 37, 255, 30.0), (6, 100, 64, 0.5)])
def test_value_loss2_matches_fp64_composite(T, M, K, spread):
    from sheeprl_prey_amd import ops
    from sheeprl_prey_amd.ops import reference as ref

    torch.manual_seed(T * M + K)
    logits = (torch.randn(T, M, K, device="cuda") * 2).requires_grad_()
    y1 = torch.randn(T, M, 1, device="cuda") * spread
    y2 = torch.randn(T, M, 1, device="cuda") * spread
    y2[0, :3] = 0.0  # a target exactly on a bin
    w = torch.rand(T, M, 1, device="cuda")
    loss = ops.twohot_value_loss(logits, y1, y2, w)
    loss.backward()
    l64 = logits.detach().double().requires_grad_()
    bins = ops.twohot_bins(K, -20.0, 20.0, device="cuda").double()
    nll = ref.twohot_nll(l64, y1.squeeze(-1).double(), bins) + ref.twohot_nll(l64, y2.squeeze(-1).double(), bins)
    r = torch.mean(nll * w.squeeze(-1).double())
    r.backward()
    torch.testing.assert_close(loss.double(), r.detach(), rtol=2e-5, atol=1e-6)
    torch.testing.assert_close(logits.grad.double(), l64.grad, rtol=1e-4, atol=1e-9)


def test_value_loss2_bitwise_reproducible():
    """The final reduction is a fixed-order tree: two runs on the same inputs give bitwise-equal losses."""
    from sheeprl_prey_amd import ops

    torch.manual_seed(0)
    logits = torch.randn(15, 1024, 255, device="cuda") * 2
    y1, y2 = torch.randn(15, 1024, 1, device="cuda") * 3, torch.randn(15, 1024, 1, device="cuda") * 3
    w = torch.rand(15, 1024, 1, device="cuda")
    a = ops.twohot_value_loss(logits, y1, y2, w)
    b = ops.twohot_value_loss(logits, y1, y2, w)
    assert torch.equal(a, b)
