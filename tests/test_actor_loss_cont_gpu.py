"""DreamerV3 continuous actor objective kernel (csrc/actor_loss.hip actor_loss_cont_kernel) against the eager
truncated-normal objective in fp64 (reference dreamer_v3.py:258-301, agent.py:685-700; TruncatedNormal entropy
from utils/distribution.py): the loss and its gradients w.r.t. the head outputs, lambda returns and baseline."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _eager(pre, lam, base, disc, off, inv, ent_coef, init_std, min_std):
    from sheeprl_prey_amd.utils.distribution import TruncatedNormal

    mean, std = torch.chunk(pre, 2, -1)
    std = 2 * torch.sigmoid((std + init_std) / 2) + min_std
    d = TruncatedNormal(torch.tanh(mean), std, pre.new_full((), -1.0), pre.new_full((), 1.0))
    ent = d.entropy().sum(-1)
    adv = (lam - off) / inv - (base - off) / inv
    return -torch.mean(disc[:-1] * (adv + ent_coef * ent[:-1]))


@pytest.mark.parametrize("T,M,A,spread", [(16, 1024, 6, 1.0), (4, 33, 1, 3.0), (9, 100, 12, 6.0)])
def test_actor_loss_cont_matches_fp64_eager(T, M, A, spread):
    from sheeprl_prey_amd import ops

    torch.manual_seed(T * M + A)
    pre = (torch.randn(T, M, 2 * A, device="cuda") * spread).requires_grad_()
    lam = torch.randn(T - 1, M, device="cuda", requires_grad=True)
    base = torch.randn(T - 1, M, device="cuda", requires_grad=True)
    disc = torch.rand(T, M, device="cuda")
    off, inv = torch.tensor(0.3, device="cuda"), torch.tensor(1.7, device="cuda")
    ent_coef, init_std, min_std = 3e-4 * spread, 0.0, 0.1
    loss = ops.actor_loss_cont(pre, lam, base, disc, off, inv, ent_coef, init_std, min_std)
    assert loss is not None
    loss.backward()
    p64, l64, b64 = (t.detach().double().requires_grad_() for t in (pre, lam, base))
    ref = _eager(p64, l64, b64, disc.double(), off.double(), inv.double(), ent_coef, init_std, min_std)
    ref.backward()
    torch.testing.assert_close(loss.double(), ref.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(lam.grad.double(), l64.grad, rtol=1e-5, atol=1e-10)
    torch.testing.assert_close(base.grad.double(), b64.grad, rtol=1e-5, atol=1e-10)
    scale = float(p64.grad.abs().max())
    torch.testing.assert_close(pre.grad.double(), p64.grad, rtol=1e-3, atol=1e-4 * scale)
    assert float(pre.grad[-1].abs().max()) == 0.0  # the last imagined step is outside the objective
