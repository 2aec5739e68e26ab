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


@pytest.mark.parametrize("M,K,A,bias", [(1024, 512, 6, True), (37, 256, 1, False), (100, 1024, 8, True)])
def test_head_linear_sample_matches_gemm_then_sample(M, K, A, bias):
    """``tn_head_linear_sample_fwd`` (head Linear folded into the truncated-normal sampler, csrc/truncnorm.hip) vs
    the library GEMM + ``tn_head_sample_fwd``, on the same uniforms; the head product against fp64."""
    from sheeprl_prey_amd import ops

    C = ops._ext()
    torch.manual_seed(M + K)
    ys = torch.randn(M, K + 8, device="cuda")
    y = ys[:, :K]  # row-strided
    W = torch.randn(2 * A, K, device="cuda") / K ** 0.5
    b = torch.randn(2 * A, device="cuda") if bias else None
    u = torch.rand(M, A, device="cuda").clamp(1e-6, 1 - 1e-6)
    outs = []
    for fused in (True, False):
        pre = torch.empty(M, 2 * A, device="cuda")
        loc, scale = torch.empty(M, A, device="cuda"), torch.empty(M, A, device="cuda")
        x = torch.full((M, A + 3), -9.0, device="cuda")[:, :A]
        if fused:
            assert C.tn_head_linear_sample_fwd(y, W, b, u, 0.0, 0.1, -1.0, 1.0, pre, loc, scale, x)
        else:
            torch.addmm(b if bias else torch.zeros(2 * A, device="cuda"), y, W.t(), out=pre)
            C.tn_head_sample_fwd(pre, u, 0.0, 0.1, -1.0, 1.0, loc, scale, x)
        outs.append((pre, loc, scale, x))
    (p1, l1, s1, x1), (p0, l0, s0, x0) = outs
    ref = y.double() @ W.double().t() + (b.double() if bias else 0.0)
    torch.testing.assert_close(p1.double(), ref, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(l1, l0, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(s1, s0, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(x1, x0, rtol=1e-4, atol=1e-4)
    # outside the kernel's LDS budget (2A x K fp32 > 64 KB): nothing launched, the caller keeps GEMM + sample
    W2 = torch.randn(2 * 9, 1024, device="cuda")
    y2 = torch.randn(4, 1024, device="cuda")
    p2, l2, s2, x2 = (torch.empty(4, 18, device="cuda"), torch.empty(4, 9, device="cuda"), torch.empty(4, 9, device="cuda"),
                      torch.empty(4, 9, device="cuda"))
    assert not C.tn_head_linear_sample_fwd(y2, W2, None, torch.rand(4, 9, device="cuda"), 0.0, 0.1, -1.0, 1.0, p2, l2, s2, x2)


@pytest.mark.parametrize("M,N,G,nA", [(1024, 512, 32, 6), (33, 256, 8, 1), (64, 1024, 16, 12)])
def test_onehot_gather_ln_dense_columns(M, N, G, nA):
    """``onehot_gather_ln`` with dense input columns (``xa @ Wa`` added in-kernel: the recurrent layer's action part
    of the continuous rollout) vs the one-hot-expanded dense layer in fp64: pre-norm values, statistics, output."""
    import torch.nn.functional as F

    from sheeprl_prey_amd import ops

    C = ops._ext()
    torch.manual_seed(M + N)
    K = G * 32
    table = torch.randn(K, N, device="cuda") / 8
    idx = (torch.randint(0, 32, (M, G), device="cuda") + torch.arange(G, device="cuda") * 32).int()
    xa = torch.randn(M, nA + 2, device="cuda")[:, :nA]
    Wa = torch.randn(nA, N, device="cuda") / 3
    gamma, beta = 1 + 0.1 * torch.randn(N, device="cuda"), 0.1 * torch.randn(N, device="cuda")
    z, y = torch.empty(M, N, device="cuda"), torch.empty(M, N, device="cuda")
    mean, rstd = torch.empty(M, device="cuda"), torch.empty(M, device="cuda")
    assert C.onehot_gather_ln(None, idx, G, 0, table, None, gamma, beta, 1e-3, ops._act_code("silu"), True, z, y, mean,
                              rstd, None, xa, Wa)
    onehot = torch.zeros(M, K, device="cuda", dtype=torch.float64).scatter_(1, idx.long(), 1.0)
    zr = onehot @ table.double() + xa.double() @ Wa.double()
    yr = F.silu(F.layer_norm(zr, (N,), gamma.double(), beta.double(), 1e-3))
    torch.testing.assert_close(z.double(), zr, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(y.double(), yr, rtol=1e-4, atol=1e-4)


def test_head_linear_sample_with_layernorm_prologue():
    """The trunk's last LayerNorm + SiLU folded in front of the head (``ln_w`` ...): normalised row, statistics,
    head outputs and samples vs ``ln_act_fwd_into`` + the unfused head."""
    from sheeprl_prey_amd import ops

    C = ops._ext()
    torch.manual_seed(11)
    M, K, A = 1024, 512, 6
    z = torch.randn(M, K + 16, device="cuda")[:, :K] * 2 + 0.5
    g, bb = 1 + 0.1 * torch.randn(K, device="cuda"), 0.1 * torch.randn(K, device="cuda")
    W, b = torch.randn(2 * A, K, device="cuda") / K ** 0.5, torch.randn(2 * A, device="cuda")
    u = torch.rand(M, A, device="cuda").clamp(1e-6, 1 - 1e-6)
    act = ops._act_code("silu")
    y1, m1, r1 = torch.empty(M, K, device="cuda"), torch.empty(M, device="cuda"), torch.empty(M, device="cuda")
    p1, l1, s1, x1 = (torch.empty(M, 2 * A, device="cuda"), torch.empty(M, A, device="cuda"), torch.empty(M, A, device="cuda"),
                      torch.empty(M, A, device="cuda"))
    assert C.tn_head_linear_sample_fwd(z, W, b, u, 0.0, 0.1, -1.0, 1.0, p1, l1, s1, x1, ln_w=g, ln_b=bb, ln_eps=1e-3, act=act,
                                       y_out=y1, mean=m1, rstd=r1)
    y0, m0, r0 = torch.empty(M, K, device="cuda"), torch.empty(M, device="cuda"), torch.empty(M, device="cuda")
    C.ln_act_fwd_into(z, z.stride(0), y0, K, g, bb, m0, r0, M, K, 1, 1e-3, act)
    p0, l0, s0, x0 = (torch.empty(M, 2 * A, device="cuda"), torch.empty(M, A, device="cuda"), torch.empty(M, A, device="cuda"),
                      torch.empty(M, A, device="cuda"))
    torch.addmm(b, y0, W.t(), out=p0)
    C.tn_head_sample_fwd(p0, u, 0.0, 0.1, -1.0, 1.0, l0, s0, x0)
    for a_, b_ in ((y1, y0), (m1, m0), (r1, r0), (p1, p0), (l1, l0), (s1, s0)):
        torch.testing.assert_close(a_, b_, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(x1, x0, rtol=1e-3, atol=1e-3)


def test_ln_gru_into_writes_back_the_summed_input():
    """``ln_gru_into(..., x2=, write_sum=True)`` (the continuous rollout's split GRU input GEMM): same next state and
    statistics as the kernel on the materialised sum, and ``x`` holds the sum afterwards (the backward reads it)."""
    from sheeprl_prey_amd import ops

    C = ops._ext()
    torch.manual_seed(3)
    for M, H in ((1024, 512), (33, 256), (16, 1024)):
        x = torch.randn(M, 3 * H, device="cuda")
        x2s = torch.randn(M, 3 * H + 40, device="cuda")[:, 8:8 + 3 * H]  # row-strided addend
        h = torch.randn(M, H, device="cuda")
        g, b = 1 + 0.1 * torch.randn(3 * H, device="cuda"), 0.1 * torch.randn(3 * H, device="cuda")
        ref_x = x + x2s
        o0, m0, r0 = torch.empty(M, H, device="cuda"), torch.empty(M, device="cuda"), torch.empty(M, device="cuda")
        C.ln_gru_into(ref_x.clone(), h, g, b, 1e-3, o0, mean=m0, rstd=r0)
        o1, m1, r1 = torch.empty(M, H, device="cuda"), torch.empty(M, device="cuda"), torch.empty(M, device="cuda")
        C.ln_gru_into(x, h, g, b, 1e-3, o1, mean=m1, rstd=r1, x2=x2s, write_sum=True)
        torch.testing.assert_close(x, ref_x, rtol=0, atol=0)
        for a_, b_ in ((o1, o0), (m1, m0), (r1, r0)):
            torch.testing.assert_close(a_, b_, rtol=1e-6, atol=1e-6)
