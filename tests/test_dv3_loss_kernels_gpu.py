"""DreamerV3 actor-phase kernels vs plain fp32 PyTorch:

* ``moments.hip`` (radix-select percentiles + EMA) vs the sort-based ``quantile`` path
  (reference ``dreamer_v3/utils.py:16-41``) -- bitwise, over several EMA updates, with ties / negatives.
* ``actor_loss.hip`` (fused discrete policy objective + its logit gradient) vs the eager
  distribution formulation (reference ``dreamer_v3/dreamer_v3.py:258-301``).
"""
import pytest
import torch
import torch.nn.functional as F

from sheeprl_prey_amd import ops
from sheeprl_prey_amd.algos.dreamer_v3.utils import Moments

pytestmark = pytest.mark.gpu


def _moments_pair():
    native, eager = Moments(None), Moments(None)
    return native.cuda(), eager.cuda()


@pytest.mark.parametrize("n", [1, 2, 7, 1000, 15 * 1024, 65536 + 3])
def test_moments_kernel_matches_sort_path(n):
    torch.manual_seed(n)
    native, eager = _moments_pair()
    for it in range(4):
        if it == 0:
            x = torch.randn(n, device="cuda") * 5 - 1
        elif it == 1:  # heavy ties
            x = torch.randint(-3, 4, (n,), device="cuda").float()
        elif it == 2:  # signed zeros, tiny and huge magnitudes
            x = torch.randn(n, device="cuda") * torch.tensor([1e-30, 1e30, 0.0, -0.0], device="cuda").repeat(n // 4 + 1)[:n]
        else:
            x = torch.rand(15, max(1, n // 15), device="cuda") * 100
        lo_n, inv_n = native.update(x)
        ops.set_fused(False)
        try:
            lo_e, inv_e = eager.update(x)
        finally:
            ops.set_fused(True)
        torch.cuda.synchronize()
        assert torch.equal(native.low, eager.low), (it, native.low.item(), eager.low.item())
        assert torch.equal(native.high, eager.high), (it, native.high.item(), eager.high.item())
        assert torch.equal(lo_n, lo_e) and torch.equal(inv_n, inv_e)


def _eager_actor_loss(mixed, actions, lam, base, disc, off, inv, heads, ent_coef):
    adv = (lam - off) / inv - (base - off) / inv  # [T-1, M, 1]
    lps, ents = [], []
    for z, a in zip(torch.split(mixed, heads, -1), torch.split(actions, heads, -1)):
        logp = F.log_softmax(z, -1)
        lps.append((logp * a).sum(-1, keepdim=True)[:-1])
        ents.append(-(logp.exp() * logp).sum(-1))
    obj = torch.stack(lps, -1).sum(-1) * adv
    ent = ent_coef * torch.stack(ents, -1).sum(-1)
    return -torch.mean(disc[:-1] * (obj + ent.unsqueeze(-1)[:-1]))


@pytest.mark.parametrize("heads,T,M", [((6,), 16, 1024), ((3, 5, 2), 16, 257), ((18,), 4, 64)])
def test_actor_loss_kernel_matches_eager(heads, T, M):
    torch.manual_seed(sum(heads) + T + M)
    A = sum(heads)
    dev = "cuda"
    raw = torch.randn(T, M, A, device=dev) * 3
    mixed = torch.cat([ops.reference.unimix_logits(z, z.shape[-1], 0.01) for z in torch.split(raw, heads, -1)], -1)
    mixed = mixed.detach().requires_grad_(True)
    idx = [torch.randint(0, h, (T, M), device=dev) for h in heads]
    actions = torch.cat([F.one_hot(i, h).float() for i, h in zip(idx, heads)], -1)
    lam = torch.randn(T - 1, M, 1, device=dev) * 10
    base = torch.randn(T - 1, M, 1, device=dev) * 10
    disc = torch.rand(T, M, 1, device=dev)
    off = torch.tensor(-0.7, device=dev)
    inv = torch.tensor(3.3, device=dev)
    ent = 3e-4

    ref = _eager_actor_loss(mixed, actions, lam, base, disc, off, inv, list(heads), ent)
    (g_ref,) = torch.autograd.grad(ref, mixed)

    z = mixed.detach().requires_grad_(True)
    got = ops.actor_loss_discrete(z, actions, lam.reshape(T - 1, M), base.reshape(T - 1, M), disc.reshape(T, M), off, inv,
                                  heads, ent)
    assert got is not None
    (got * 2.0).backward()
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(z.grad, 2.0 * g_ref, rtol=1e-4, atol=1e-8)
    assert torch.all(z.grad[-1] == 0)


def test_actor_loss_kernel_graph_capture():
    T, M, heads = 8, 128, (4,)
    dev = "cuda"
    z = torch.randn(T, M, 4, device=dev, requires_grad=True)
    actions = F.one_hot(torch.randint(0, 4, (T, M), device=dev), 4).float()
    lam, base, disc = torch.randn(T - 1, M, device=dev), torch.randn(T - 1, M, device=dev), torch.rand(T, M, device=dev)
    off, inv = torch.tensor(0.1, device=dev), torch.tensor(2.0, device=dev)

    def step():
        z.grad = None
        loss = ops.actor_loss_discrete(z, actions, lam, base, disc, off, inv, heads, 1e-3)
        loss.backward()
        return loss

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    eager_loss = step().detach().clone()
    eager_grad = z.grad.clone()
    z.grad = torch.zeros_like(z)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        loss = ops.actor_loss_discrete(z, actions, lam, base, disc, off, inv, heads, 1e-3)
        (gz,) = torch.autograd.grad(loss, z)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(loss, eager_loss) and torch.equal(gz, eager_grad)


@pytest.mark.parametrize("u8,symlog,shape", [(True, False, (8, 4, 3, 64, 64)), (False, True, (8, 4, 20)),
                                            (False, False, (5, 3, 1, 16, 16))])
def test_obs_mse_kernel_matches_eager(u8, symlog, shape):
    """K6: observation MSE (image: against the raw uint8 frames / 255; vector: symlog MSE with the
    d < 1e-8 rule) and its gradient vs the reference formulation."""
    torch.manual_seed(len(shape))
    rec = torch.randn(*shape, device="cuda", requires_grad=True)
    if u8:
        raw = torch.randint(0, 256, shape, device="cuda", dtype=torch.uint8)
        tgt = raw.float() / 255.0
    else:
        raw = tgt = torch.randn(*shape, device="cuda") * 3
    dims = tuple(range(2, rec.dim()))
    if symlog:
        d = (rec - torch.sign(tgt) * torch.log1p(tgt.abs())) ** 2
        ref = torch.where(d < 1e-8, torch.zeros_like(d), d).sum(dim=dims)
    else:
        ref = ((rec - tgt) ** 2).sum(dim=dims)
    g = torch.rand_like(ref)
    (gr,) = torch.autograd.grad((ref * g).sum(), rec)
    got = ops.obs_mse(rec, raw, 1.0 / 255.0 if u8 else 1.0, symlog=symlog)
    (gg,) = torch.autograd.grad((got * g).sum(), rec)
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(gg, gr, rtol=1e-5, atol=1e-5)


def test_imag_discount_kernel_matches_torch():
    """K11: imagined continuation discounts (one kernel) vs the reference torch form, bitwise."""
    torch.manual_seed(0)
    T1, M, gamma = 16, 1024, 0.996996996
    logits = torch.randn(T1, M, 1, device="cuda")
    dones = (torch.rand(M, device="cuda") < 0.1).float()
    cg, disc = ops.imag_discount(logits, dones, gamma)
    c = (logits > 0).float()
    c = torch.cat(((1 - dones).reshape(1, -1, 1), c[1:]))
    assert torch.equal(cg, c[1:] * gamma)
    assert torch.equal(disc, torch.cumprod(c * gamma, dim=0) / gamma)
    # skip_first: only the rows 1.. of the logits are given (the trainer never computes row 0)
    cg1, disc1 = ops.imag_discount(logits[1:].contiguous(), dones, gamma, skip_first=True)
    assert torch.equal(cg1, cg) and torch.equal(disc1, disc)


def test_wm_loss_assembly_matches_eager():
    """The fused loss assembly (wm_loss.hip: continue BCE, weighted sum, mean, metric means) vs the
    eager formulation, forward values and the gradients reaching every per-row input."""
    from sheeprl_prey_amd import ops
    from sheeprl_prey_amd.algos.dreamer_v3.loss import reconstruction_loss

    torch.manual_seed(0)
    T, B, S, C, K = 16, 8, 32, 32, 255
    mk = lambda *s: torch.randn(*s, device="cuda", requires_grad=True)  # noqa: E731
    obs, rl, post, prior, cl = mk(T, B), mk(T, B, K), mk(T, B, S * C), mk(T, B, S * C), mk(T, B, 1)
    rew = torch.randn(T, B, 1, device="cuda")
    dones = (torch.rand(T, B, 1, device="cuda") < 0.2).float()
    args = (rew, prior, post, S, C, 0.5, 0.1, 1.0, 1.0)
    fused = reconstruction_loss(obs, rl, *args, cl, None, 1.0, dones=dones)
    g_f = torch.autograd.grad(fused[0], (obs, rl, post, prior, cl))
    ops._FUSED = False
    try:
        eager = reconstruction_loss(obs, rl, *args, cl, 1 - dones, 1.0)
        g_e = torch.autograd.grad(eager[0], (obs, rl, post, prior, cl))
    finally:
        ops._FUSED = True
    for a, b in zip(fused, eager):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)
    for a, b in zip(g_f, g_e):
        torch.testing.assert_close(a, b, rtol=1e-3, atol=1e-6)
