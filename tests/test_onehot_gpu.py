"""One-hot first layers as row gathers (ops/onehot.py, csrc/onehot.hip) vs the dense fp32 layer:
``act(LN(x W^T + b))`` with the first S input columns exact one-hots, forward and backward."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _onehot(M, G, C, gen):
    k = torch.randint(0, C, (M, G), device="cuda", generator=gen)
    return F.one_hot(k, C).float().view(M, G * C), k


@pytest.mark.parametrize("N,Kd,ln,bias", [(512, 512, True, False), (4096, 512, False, True), (1024, 96, True, True), (1000, 64, True, True),
                                          (256, 0, True, False)])
def test_gather_first_layer_matches_dense(N, Kd, ln, bias):
    from sheeprl_prey_amd.ops import onehot as oh
    from sheeprl_prey_amd.utils.model import LayerNorm

    g = torch.Generator(device="cuda").manual_seed(0)
    M, G, C = 300, 32, 32
    S = G * C
    z, k = _onehot(M, G, C, g)
    h = torch.randn(M, Kd, device="cuda", generator=g)
    x = torch.cat((z, h), 1).requires_grad_(True)
    lin = torch.nn.Linear(S + Kd, N, bias=bias).cuda()
    norm = LayerNorm(N, eps=1e-3, act="silu").cuda() if ln else None
    if norm is not None:
        with torch.no_grad():
            norm.weight.add_(0.1 * torch.randn(N, device="cuda", generator=g))
            norm.bias.add_(0.1 * torch.randn(N, device="cuda", generator=g))
    idx = torch.empty(M, G, dtype=torch.int32, device="cuda")
    oh.onehot_index(z, C, idx, 7)  # offset 7: idx = 7 + g*C + k
    assert torch.equal(idx.long() - 7, k + torch.arange(G, device="cuda") * C)
    y = oh.first_layer(x, idx, G, 7, lin, norm, S)
    ref = F.linear(x.double(), lin.weight.double(), None if lin.bias is None else lin.bias.double())
    if norm is not None:
        ref = F.silu(F.layer_norm(ref, (N,), norm.weight.double(), norm.bias.double(), 1e-3))
    torch.testing.assert_close(y.double(), ref, rtol=2e-5, atol=2e-5)
    gy = torch.randn_like(y)
    (y * gy).sum().backward()
    grads = [x.grad.clone(), lin.weight.grad.clone()] + ([norm.weight.grad.clone()] if norm is not None else [])
    for p in [x, lin.weight] + ([norm.weight] if norm is not None else []):
        p.grad = None
    (ref * gy.double()).sum().backward()
    refs = [x.grad, lin.weight.grad] + ([norm.weight.grad] if norm is not None else [])
    for a, b in zip(grads, refs):
        torch.testing.assert_close(a.double(), b.double(), rtol=1e-4, atol=1e-4)
    oh.check_onehot_error()


def test_gather_rejects_out_of_range_index():
    from sheeprl_prey_amd.ops import onehot as oh

    M, G, N = 8, 4, 64
    lin = torch.nn.Linear(G * 8, N, bias=False).cuda()
    idx = torch.full((M, G), 10_000, dtype=torch.int32, device="cuda")
    x = torch.zeros(M, G * 8, device="cuda")
    y = oh.gather_first_layer(x, idx, G, 0, lin, None, G * 8)
    torch.cuda.synchronize()
    assert torch.equal(y, torch.zeros_like(y))
    with pytest.raises(RuntimeError, match="outside its weight table"):
        oh.check_onehot_error()


@pytest.mark.parametrize("graphs", [False, True])
def test_dv3_onehot_heads_match_dense(graphs):
    """A DreamerV3 step with the one-hot gathers (rollout, imagination heads, world-model heads) vs the
    dense first layers from the same state and RNG: same losses and updated weights to fp32 rounding."""
    import copy

    from tests.test_dreamer_gpu import _build, _data

    tr = _build(graphs=False)
    data = _data()
    tr.train_step(data)
    torch.cuda.synchronize()
    opts = (tr.world_optimizer, tr.actor_optimizer, tr.critic_optimizer)
    snap = [(o.flat_param.clone(), o.exp_avg.clone(), o.exp_avg_sq.clone(), o.scalars.clone()) for o in opts]
    msnap = copy.deepcopy(tr.moments.state_dict())
    results = []
    for on in (False, True):
        for o, (p, m, v, sc) in zip(opts, snap):
            o.flat_param.copy_(p); o.exp_avg.copy_(m); o.exp_avg_sq.copy_(v); o.scalars.copy_(sc)
        tr.moments.load_state_dict(msnap)
        tr.onehot_heads = on
        tr.graphed.enabled = graphs
        tr.graphed.graph = None
        tr.graphed._calls = 0
        tr.graphed.warmup = 0
        torch.manual_seed(321)
        torch.cuda.manual_seed(321)
        out = tr.train_step(data)
        torch.cuda.synchronize()
        results.append(({k: float(v) for k, v in out.items()}, [o.flat_param.clone() for o in opts]))
    (o0, p0), (o1, p1) = results
    # the actor-side values go through the Moments percentiles of the lambda returns and the sampled imagined
    # actions, which amplify rounding-level logit differences (observed 4e-4 relative): looser bound there
    tol = {"Loss/policy_loss": 1e-3, "Grads/actor": 1e-3}
    bad = {k: (o0[k], o1[k]) for k in ("Loss/world_model_loss", "Loss/observation_loss", "Loss/reward_loss",
                                        "Loss/continue_loss", "Grads/world_model", "Loss/policy_loss", "Loss/value_loss",
                                        "Grads/actor", "Grads/critic")
           if abs(o0[k] - o1[k]) > tol.get(k, 2e-4) * max(1.0, abs(o0[k]))}
    assert not bad, bad
    for a, b in zip(p0, p1):
        torch.testing.assert_close(b, a, rtol=1e-4, atol=2e-5)


@pytest.mark.parametrize("record", [False, True])
def test_imagine_gather_matches_dense_rollout(record):
    """The rollout with the one-hot gathers vs the same rollout with dense first layers, same uniforms:
    the sampled paths agree up to rare rounding flips, and matching rows agree in h."""
    from tests.test_dreamer_gpu import _build

    tr = _build(graphs=False)
    wm, actor = tr.world_model, tr.actor
    M, S, H, Hz = 256, 32 * 32, 64, 6
    g = torch.Generator(device="cuda").manual_seed(3)
    post = F.one_hot(torch.randint(0, 32, (M, 32), device="cuda", generator=g), 32).float().view(M, S)
    h = torch.randn(M, H, device="cuda", generator=g)
    outs = []
    for gather in (False, True):
        torch.manual_seed(7)
        outs.append(wm.rssm.imagine_discrete(post, h, actor, Hz, record=record, indices=True, gather=gather))
    (t0, a0), (t1, a1) = outs[0][:2], outs[1][:2]
    idx0, idx1 = outs[0][-1], outs[1][-1]
    assert torch.equal(idx0, idx1) or (idx0 == idx1).float().mean() > 0.95
    # the indices describe the sampled one-hots exactly
    A = a1.shape[-1]
    hot = torch.zeros(Hz + 1, M, A + S, device="cuda")
    hot.scatter_(2, idx1.long(), 1.0)
    torch.testing.assert_close(hot[:, :, A:], t1[:, :, :S])
    torch.testing.assert_close(hot[:, :, :A], a1)
    same = (t0[:, :, :S] == t1[:, :, :S]).all(-1).all(0) & (a0 == a1).all(-1).all(0)
    frac = same.float().mean().item()
    assert frac > 0.95, (frac, [(t0[i, :, :S] == t1[i, :, :S]).all(-1).float().mean().item() for i in range(Hz + 1)])
    torch.testing.assert_close(t1[:, same], t0[:, same], rtol=1e-4, atol=1e-4)
    if record:
        r0, r1 = outs[0][2], outs[1][2]
        torch.testing.assert_close(r1.y[-1][:, same], r0.y[-1][:, same], rtol=1e-4, atol=1e-4)
