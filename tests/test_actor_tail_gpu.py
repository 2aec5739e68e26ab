"""Fused rollout actor tail (csrc/actor_tail.hip): act(LN(pre)) + head + unimix one-hot sample in one launch, vs the
three-launch path (ln_act, F.linear, unimix_sample_into) and vs fp64 for the LayerNorm / head values."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,N,A,sample", [(1024, 512, 9, True), (300, 256, 16, True), (77, 1024, 4, False), (64, 512, 16, True)])
def test_actor_tail_matches_unfused(M, N, A, sample):
    from sheeprl_prey_amd import ops

    C = ops._ext()
    g = torch.Generator(device="cuda").manual_seed(0)
    pre = torch.randn(M, N + 8, device="cuda", generator=g)[:, 4:4 + N]  # row-strided
    pre = torch.randn(M, N, device="cuda", generator=g) if N % 4 or pre.stride(0) % 4 else pre
    gam = 1 + 0.1 * torch.randn(N, device="cuda", generator=g)
    bet = 0.1 * torch.randn(N, device="cuda", generator=g)
    Wh = torch.randn(A, N, device="cuda", generator=g) / N ** 0.5
    bh = torch.randn(A, device="cuda", generator=g)
    uni = torch.rand(M, device="cuda", generator=g) if sample else None
    y = torch.empty(M, N, device="cuda")
    mean, rstd = torch.empty(M, device="cuda"), torch.empty(M, device="cuda")
    out = torch.zeros(M, A + 3, device="cuda")
    idx = torch.zeros(M, 2, dtype=torch.int32, device="cuda")
    logits = torch.empty(M, A, device="cuda")
    ok = C.actor_tail(pre, y, gam, bet, mean, rstd, 1e-3, ops._act_code("silu"), Wh, bh, uni, 0.01, out[:, :A], idx[:, 1:],
                      5, logits)
    assert ok
    yd = F.silu(F.layer_norm(pre.double(), (N,), gam.double(), bet.double(), 1e-3))
    torch.testing.assert_close(y.double(), yd, rtol=1e-5, atol=2e-5)
    ld = yd @ Wh.double().t() + bh.double()
    torch.testing.assert_close(logits.double(), ld, rtol=1e-5, atol=5e-5)
    # the sampler on the kernel's own logits: identical to the standalone unimix kernel
    ref = torch.zeros(M, A, device="cuda")
    ridx = torch.zeros(M, 1, dtype=torch.int32, device="cuda")
    C.unimix_sample_into(logits, uni, A, 0.01, ref, ridx, 5)
    assert torch.equal(out[:, :A], ref)
    assert torch.equal(idx[:, 1:], ridx)
    assert torch.all(out[:, A:] == 0)
    assert torch.equal(out[:, :A].sum(1), torch.ones(M, device="cuda"))


def test_player_tail_draw_matches_eager():
    """The discrete player's fused draw (Actor._tail_sample: last LayerNorm + head + unimix sample in one launch)
    against the eager trunk + head + unimix sampler fed the same uniforms."""
    from sheeprl_prey_amd import ops
    from tests.test_dreamer_gpu import _build

    actor = _build(graphs=False).actor
    M = 9
    state = torch.randn(1, M, actor.model.model[0].in_features, device="cuda")
    torch.manual_seed(3)
    a = actor._tail_sample(state)
    assert a is not None and a.shape == (1, M, 5)
    torch.manual_seed(3)
    u = torch.rand(M, device="cuda")
    with torch.no_grad():
        logits = actor.mlp_heads[0](actor.model(state.view(M, -1)))
        ref = ops.unimix_sample(logits, 5, actor._unimix, sample=True, uniform=u)[1]
    assert torch.equal(a.view(M, 5).sum(-1), torch.ones(M, device="cuda"))
    assert torch.equal(a.view(M, 5), ref)
