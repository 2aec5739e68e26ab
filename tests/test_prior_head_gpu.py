"""One-launch imagination prior head (``prior_head.hip``): LayerNorm + act, output Linear, unimix categorical
sample, against an fp64 reference of the same math (``ops/reference.py`` semantics: unimix, then the
inverse-CDF draw with the given uniforms).  A draw is checked by interval membership in the fp64 CDF (a uniform
within rounding distance of a boundary may legitimately pick either neighbour)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ref_cdf(x, gamma, beta, eps, W, b, alpha, C=32):
    xd = x.double()
    y = F.silu(F.layer_norm(xd, (x.shape[1],), gamma.double(), beta.double(), eps))
    l = y @ W.double().t() + (b.double() if b is not None else 0.0)
    l = l.view(x.shape[0], -1, C)
    p = torch.softmax(l, -1)
    if alpha > 0:
        p = (1 - alpha) * p + alpha / C
        p = p.clamp(1.1920928955078125e-07, 1 - 1.1920928955078125e-07)
        p = torch.softmax(p.log(), -1)
    return p.cumsum(-1)


@pytest.mark.parametrize("M,K,N,strided,bias", [(1024, 512, 1024, True, True), (40, 512, 256, False, True),
                                                (64, 1024, 512, True, False), (16, 256, 1024, False, True)])
def test_prior_head_matches_fp64(M, K, N, strided, bias):
    from sheeprl_prey_amd import ops

    C = ops._ext()
    torch.manual_seed(0)
    dev = "cuda"
    G = N // 32
    xs = torch.randn(M, K + 64 if strided else K, device=dev)
    x = xs[:, :K]
    gamma = 1 + 0.1 * torch.randn(K, device=dev)
    beta = 0.1 * torch.randn(K, device=dev)
    W = torch.randn(N, K, device=dev) / K ** 0.5
    b = 0.1 * torch.randn(N, device=dev) if bias else None
    u = torch.rand(M * G, device=dev)
    out = torch.full((M, N + 8), -1.0, device=dev)
    idx = torch.full((M, G + 3), -7, dtype=torch.int32, device=dev)
    ok = C.prior_head(x, gamma, beta, 1e-3, ops._act_code("silu"), W, b, u, 0.01,
                      out[:, 2:2 + N], idx[:, 1:1 + G], 5)
    assert ok
    torch.cuda.synchronize()
    s = out[:, 2:2 + N].view(M, G, 32)
    assert torch.equal(s.sum(-1), torch.ones(M, G, device=dev))  # exact one-hots
    assert torch.all((s == 0) | (s == 1))
    assert torch.all(out[:, :2] == -1) and torch.all(out[:, 2 + N:] == -1)  # nothing outside the view
    pick = s.argmax(-1)
    assert torch.equal(idx[:, 1:1 + G].long(), 5 + torch.arange(G, device=dev) * 32 + pick)
    assert torch.all(idx[:, 0] == -7) and torch.all(idx[:, 1 + G:] == -7)
    cdf = _ref_cdf(x, gamma, beta, 1e-3, W, b, 0.01)
    uu = u.double().view(M, G, 1)
    hi = cdf.gather(-1, pick.unsqueeze(-1))
    lo = torch.where(pick.unsqueeze(-1) > 0, cdf.gather(-1, (pick - 1).clamp_min(0).unsqueeze(-1)), torch.zeros_like(hi))
    tol = 1e-5
    assert torch.all(lo <= uu + tol) and torch.all(uu <= hi + tol), "draw outside its fp64 CDF interval"
    # the reference's own draw agrees except within rounding distance of a boundary
    ref_pick = (cdf < uu).sum(-1).clamp_max(31)
    near = ((cdf - uu).abs() < tol).any(-1)
    assert torch.equal(pick[~near], ref_pick[~near])


def test_imagination_prior_head_matches_three_launch_path():
    """imagine_discrete with the fused prior head vs SRL_PRIOR_HEAD off (LayerNorm kernel + GEMM + sampler), same
    uniforms: the sampled paths agree up to rare rounding flips and the indices describe the one-hots exactly."""
    from sheeprl_prey_amd.algos.dreamer_v3.agent import RSSM
    from tests.test_dreamer_gpu import _build

    tr = _build(graphs=False)
    wm, actor = tr.world_model, tr.actor
    M, S, H, Hz = 256, 32 * 32, 64, 6
    g = torch.Generator(device="cuda").manual_seed(3)
    post = F.one_hot(torch.randint(0, 32, (M, 32), device="cuda", generator=g), 32).float().view(M, S)
    h = torch.randn(M, H, device="cuda", generator=g)
    outs = []
    for on in (False, True):
        RSSM._prior_head_ok = on
        try:
            torch.manual_seed(7)
            outs.append(wm.rssm.imagine_discrete(post, h, actor, Hz, indices=True))
        finally:
            RSSM._prior_head_ok = True
    (t0, a0, i0), (t1, a1, i1) = outs
    A = a1.shape[-1]
    hot = torch.zeros(Hz + 1, M, A + S, device="cuda")
    hot.scatter_(2, i1.long(), 1.0)
    torch.testing.assert_close(hot[:, :, A:], t1[:, :, :S])
    same = (t0[:, :, :S] == t1[:, :, :S]).all(-1).all(0) & (a0 == a1).all(-1).all(0)
    frac = same.float().mean().item()
    assert frac > 0.95, frac
    torch.testing.assert_close(t1[:, same], t0[:, same], rtol=1e-4, atol=1e-4)
