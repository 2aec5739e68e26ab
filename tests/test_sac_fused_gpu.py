"""The fused SAC gradient step (csrc/sac_fused.hip, algos/sac/fused.py) against fp64 PyTorch references of the
same math (reference sac/agent.py:53-152 actor, sac/agent.py:256-275 critics, sac/loss.py:10-26 losses,
sac/sac.py:34-78 the update).  The kernels draw their own Gaussian noise and return it, so every reference is
evaluated on exactly that noise."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _C():
    from sheeprl_prey_amd import ops

    return ops._ext()


def _actor(OD, A, H, seed):
    from sheeprl_prey_amd.algos.sac.agent import SACActor

    torch.manual_seed(seed)
    low = -np.linspace(1.0, 2.0, A)
    high = np.linspace(0.5, 3.0, A)
    a = SACActor(OD, A, hidden_size=H, action_low=low, action_high=high).cuda()
    with torch.no_grad():  # spread the raw log-std so both clamp bounds are exercised
        a.fc_logstd.weight.mul_(6.0)
        a.fc_logstd.bias.uniform_(-6.0, 3.0)
    return a


def _actor_w(a):
    m = a.model.model
    return [m[0].weight, m[0].bias, m[2].weight, m[2].bias, a.fc_mean.weight, a.fc_mean.bias, a.fc_logstd.weight,
            a.fc_logstd.bias, a.action_scale, a.action_bias]


def _critic_w(crit):
    e = crit.model
    return [e.layers[0].weight, e.layers[0].bias, e.layers[1].weight, e.layers[1].bias, e.head.weight, e.head.bias]


def _ref_heads(w, obs):
    W1, b1, W2, b2, Wm, bm, Ws, bs = w[:8]
    h1 = torch.relu(obs @ W1.T + b1)
    h2 = torch.relu(h1 @ W2.T + b2)
    return h2 @ Wm.T + bm, h2 @ Ws.T + bs


def _ref_sample(w, obs, eps):
    from sheeprl_prey_amd.ops import reference as ref

    mean, raw = _ref_heads(w, obs)
    return ref.squashed_gaussian(mean, raw, eps, w[8], w[9], 0, -5.0, 2.0)


def _ref_q(cw, obs, act):
    W1, b1, W2, b2, W3, b3 = cw
    x = torch.cat([obs, act], -1)
    h1 = torch.relu(torch.einsum("mi,nhi->nmh", x, W1) + b1[:, None])
    h2 = torch.relu(torch.einsum("nmh,nkh->nmk", h1, W2) + b2[:, None])
    return (torch.einsum("nmh,noh->nmo", h2, W3) + b3[:, None]).squeeze(-1).T  # [M, n]


def _d(ts):
    return [t.detach().double() for t in ts]


@pytest.mark.parametrize("OD,A,H,M", [(24, 6, 256, 1), (24, 6, 256, 37), (32, 1, 128, 256), (17, 17, 256, 100)])
def test_fused_player_matches_reference(OD, A, H, M):
    C = _C()
    a = _actor(OD, A, H, seed=OD + A + M)
    w = _actor_w(a)
    obs = torch.randn(M, OD, device="cuda") * 2
    ctr = torch.zeros(2, dtype=torch.int64, device="cuda")
    ticket = torch.zeros(1, dtype=torch.int32, device="cuda")
    act = torch.empty(M, A, device="cuda")
    logp = torch.empty(M, device="cuda")
    eps = torch.empty(M, A, device="cuda")
    C.sac_fused_act(obs, w, -5.0, 2.0, ctr[1:], ticket, 12345, act, logp, eps)
    torch.cuda.synchronize()
    a_ref, lp_ref = _ref_sample(_d(w), obs.double(), eps.double())
    torch.testing.assert_close(act.double(), a_ref, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(logp.double(), lp_ref.squeeze(-1), rtol=1e-4, atol=2e-3)
    assert int(ctr[1]) == 1 and int(ctr[0]) == 0 and int(ticket) == 0
    eps2 = torch.empty_like(eps)
    C.sac_fused_act(obs, w, -5.0, 2.0, ctr[1:], ticket, 12345, act, None, eps2)
    assert int(ctr[1]) == 2 and not torch.equal(eps, eps2)


def test_fused_noise_is_standard_normal():
    C = _C()
    a = _actor(8, 16, 128, seed=3)
    M = 8192
    obs = torch.randn(M, 8, device="cuda")
    ctr = torch.zeros(1, dtype=torch.int64, device="cuda")
    ticket = torch.zeros(1, dtype=torch.int32, device="cuda")
    act = torch.empty(M, 16, device="cuda")
    eps = torch.empty(M, 16, device="cuda")
    C.sac_fused_act(obs, _actor_w(a), -5.0, 2.0, ctr, ticket, 99, act, None, eps)
    e = eps.double().flatten()
    assert abs(float(e.mean())) < 0.02 and abs(float(e.std()) - 1.0) < 0.02
    assert abs(float((e ** 3).mean())) < 0.06 and abs(float((e ** 4).mean()) - 3.0) < 0.15
    # neighbouring elements are uncorrelated
    assert abs(float((eps[:, 0].double() * eps[:, 1].double()).mean())) < 0.04
    assert int(ticket) == 0 and int(ctr) == 1


@pytest.mark.parametrize("OD,A,H,n,Hc,M", [(24, 6, 256, 2, 256, 256), (17, 3, 128, 3, 128, 45), (32, 8, 256, 2, 512, 64)])
def test_fused_target_matches_reference(OD, A, H, n, Hc, M):
    from sheeprl_prey_amd.algos.sac.agent import SACCriticEnsemble

    C = _C()
    a = _actor(OD, A, H, seed=n * M)
    crit = SACCriticEnsemble(OD + A, n=n, hidden_size=Hc).cuda()
    obs = torch.randn(M, OD, device="cuda")
    rew = torch.randn(M, device="cuda")
    done = (torch.rand(M, device="cuda") < 0.2).float()
    log_alpha = torch.tensor([-0.9], device="cuda")
    ctr = torch.tensor([5], dtype=torch.int64, device="cuda")
    y = torch.empty(M, device="cuda")
    act = torch.empty(M, A, device="cuda")
    logp = torch.empty(M, device="cuda")
    eps = torch.empty(M, A, device="cuda")
    C.sac_fused_target(obs, rew, done, log_alpha, _actor_w(a), -5.0, 2.0, _critic_w(crit), ctr, 77, 0.99, y, act, logp, eps)
    torch.cuda.synchronize()
    a_ref, lp_ref = _ref_sample(_d(_actor_w(a)), obs.double(), eps.double())
    torch.testing.assert_close(act.double(), a_ref, rtol=1e-4, atol=1e-4)
    q = _ref_q(_d(_critic_w(crit)), obs.double(), act.double())  # the kernel's own actions
    y_ref = rew.double() + (1 - done.double()) * 0.99 * (q.min(-1)[0] - log_alpha.double().exp() * logp.double())
    torch.testing.assert_close(y.double(), y_ref, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(logp.double(), lp_ref.squeeze(-1), rtol=1e-4, atol=2e-3)
    assert int(ctr) == 5  # the target launch only reads the update counter


def _actor_ws(M, OD, H, A, n):
    C = _C()
    zp, nb = C.sac_fused_zp(A), C.sac_fused_blocks(M)
    e = lambda *s: torch.full(s, float("nan"), device="cuda")  # noqa: E731  (poisoned: every read must be written first)
    ws = [e(M, (OD + 15) // 16 * 16), e(M, H), e(M, H), e(M, zp), e(M, H), e(M, H), e(n, M), e(n, M, A), e(nb, 2)]
    return ws, torch.zeros(nb, dtype=torch.int32, device="cuda")


@pytest.mark.parametrize("reduce_min", [True, False])
@pytest.mark.parametrize("OD,A,H,n,Hc,M", [(24, 6, 256, 2, 256, 256), (17, 3, 128, 3, 256, 50), (32, 1, 256, 2, 128, 16)])
def test_fused_actor_update_matches_autograd(reduce_min, OD, A, H, n, Hc, M):
    """Policy loss mean(alpha logp - min/mean_c Q_c(s, a)) and the alpha loss: losses, every actor gradient and
    the log-alpha gradient vs fp64 autograd on the kernel's own noise."""
    from sheeprl_prey_amd.algos.sac.agent import SACCriticEnsemble

    C = _C()
    a = _actor(OD, A, H, seed=M + n)
    crit = SACCriticEnsemble(OD + A, n=n, hidden_size=Hc).cuda()
    obs = torch.randn(M, OD, device="cuda")
    log_alpha = torch.tensor([-0.4], device="cuda")
    te = torch.tensor([-float(A)], device="cuda")
    ctr = torch.tensor([3], dtype=torch.int64, device="cuda")
    ws, cnt = _actor_ws(M, OD, H, A, n)
    w = _actor_w(a)
    grads = [torch.full_like(p, float("nan")) for p in w[:8]] + [torch.full((1,), float("nan"), device="cuda")]
    losses = torch.empty(2, device="cuda")
    acc = torch.zeros(3, 2, dtype=torch.float64, device="cuda")
    qf = torch.tensor([0.25], device="cuda")
    act = torch.empty(M, A, device="cuda")
    logp = torch.empty(M, device="cuda")
    eps = torch.empty(M, A, device="cuda")
    q = torch.empty(M, n, device="cuda")
    C.sac_fused_actor(obs, log_alpha, te, w, -5.0, 2.0, _critic_w(crit), ctr, 11, reduce_min, ws, cnt, grads, qf, losses,
                      acc, act, logp, eps, q)
    torch.cuda.synchronize()
    assert int(ctr) == 4 and int(cnt.abs().sum()) == 0

    wd = [t.clone().requires_grad_() for t in _d(w[:8])] + _d(w[8:])
    la = log_alpha.double().clone().requires_grad_()
    a_ref, lp_ref = _ref_sample(wd, obs.double(), eps.double())
    q_ref = _ref_q(_d(_critic_w(crit)), obs.double(), a_ref)
    torch.testing.assert_close(q.double(), q_ref.detach(), rtol=1e-4, atol=1e-4)
    q_red = q_ref.min(-1, keepdim=True)[0] if reduce_min else q_ref.mean(-1, keepdim=True)
    pl = (la.detach().exp() * lp_ref - q_red).mean()
    al = (-la * (lp_ref.detach() + te.double())).mean()
    g_ref = torch.autograd.grad(pl, wd[:8]) + torch.autograd.grad(al, [la])
    torch.testing.assert_close(losses[0].double(), pl.detach(), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(losses[1].double(), al.detach(), rtol=1e-4, atol=1e-4)
    names = ["W1", "b1", "W2", "b2", "Wm", "bm", "Ws", "bs", "log_alpha"]
    for nm, g, r in zip(names, grads, g_ref):
        scale = float(r.abs().max()) + 1e-6
        torch.testing.assert_close(g.double(), r.reshape(g.shape), rtol=2e-3, atol=2e-4 * scale,
                                   msg=lambda m, nm=nm: f"{nm}: {m}")
    # metric sums: value (given), policy and alpha losses, one count each
    torch.testing.assert_close(acc[:, 1], torch.ones(3, dtype=torch.float64, device="cuda"))
    torch.testing.assert_close(acc[:, 0].float(), torch.stack([qf[0], losses[0], losses[1]]))


def test_fused_critic_wgrad_into_slab_matches_autograd_path():
    from sheeprl_prey_amd import ops
    from sheeprl_prey_amd.algos.sac.agent import SACCriticEnsemble

    C = _C()
    torch.manual_seed(5)
    n, H, OD, A, M = 2, 256, 24, 6, 200
    crit = SACCriticEnsemble(OD + A, n=n, hidden_size=H).cuda()
    obs, act, y = torch.randn(M, OD, device="cuda"), torch.rand(M, A, device="cuda") * 2 - 1, torch.randn(M, device="cuda")
    cw = _critic_w(crit)
    loss_ref, _ = ops.sac_critic_loss(crit.model, obs, act, y)
    g_ref = torch.autograd.grad(loss_ref, cw)
    lossp, _q, *saved = C.sac_critic_fwd(obs, act, y, *cw)
    outs = [torch.full_like(p, float("nan")) for p in cw]
    loss = torch.empty(1, device="cuda")
    C.sac_fused_critic_wgrad(saved, torch.ones(1, device="cuda"), OD + A, outs, lossp, loss)
    torch.testing.assert_close(loss[0], loss_ref.detach(), rtol=1e-5, atol=1e-6)
    for a_, b_ in zip(outs, g_ref):
        torch.testing.assert_close(a_, b_, rtol=1e-5, atol=1e-7)


def _adam_ref(p, g, m, v, t, lr, b1, b2, eps, wd):
    g = g + wd * p
    m = m + (1 - b1) * (g - m)
    v = v * b2 + (1 - b2) * g * g
    p = p - lr / (1 - b1 ** t) * m / (v.sqrt() / (1 - b2 ** t) ** 0.5 + eps)
    return p, m, v


def test_adam_multi_matches_flat_adam_and_ema():
    from sheeprl_prey_amd import ops

    C = _C()
    torch.manual_seed(0)
    sizes, hyper = [4096 + 64, 4], [[3e-4, 0.9, 0.999, 1e-4, 0.0, 0.0], [1e-2, 0.8, 0.99, 1e-8, 0.01, 0.0]]
    slabs = []
    for n in sizes:
        slabs.append([torch.randn(n, device="cuda"), torch.randn(n, device="cuda"), torch.randn(n, device="cuda") * 0.1,
                      torch.rand(n, device="cuda") * 0.1, torch.tensor([3.0, 1.0, 0.0, 0.0], device="cuda")])
    target = torch.randn(sizes[0], device="cuda")
    ema_w = torch.tensor([0.005], device="cuda")
    ref = [[t.double().clone() for t in s[:4]] for s in slabs]
    tgt_ref = target.double().clone()
    tickets = torch.zeros(4, dtype=torch.int32, device="cuda")
    guard = ops.fault_block(torch.device("cuda"))
    guard.zero_()
    for step in range(3):
        C.sac_adam_multi([slabs[0] + [target, ema_w], slabs[1]], hyper, guard, tickets)
        for r, h in zip(ref, hyper):
            r[0], r[2], r[3] = _adam_ref(r[0], r[1], r[2], r[3], 4 + step, *h[:5])
        tgt_ref = tgt_ref + 0.005 * (ref[0][0] - tgt_ref)
    torch.cuda.synchronize()
    for s, r in zip(slabs, ref):
        torch.testing.assert_close(s[0].double(), r[0], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(s[2].double(), r[2], rtol=1e-4, atol=1e-7)
        torch.testing.assert_close(s[3].double(), r[3], rtol=1e-4, atol=1e-9)
        assert float(s[4][0]) == 6.0 and float(s[4][3]) == 0.0
    torch.testing.assert_close(target.double(), tgt_ref, rtol=1e-5, atol=1e-6)
    assert int(tickets.abs().sum()) == 0
    # a recorded fault: no parameter / moment update, the step count stays, skip flag set, one skip counted per slab
    before = [s[0].clone() for s in slabs]
    guard[1] = 1
    skipped = int(guard[2])
    C.sac_adam_multi([slabs[0], slabs[1]], hyper, guard, tickets)
    torch.cuda.synchronize()
    for s, b in zip(slabs, before):
        assert torch.equal(s[0], b) and float(s[4][0]) == 6.0 and float(s[4][3]) == 1.0
    assert int(guard[2]) == skipped + 2
    guard.zero_()


def test_fused_trainer_selected_and_metrics_accumulate():
    """exp=sac selects the fused update (DroQ keeps autograd); the device-side loss sums give the same
    per-interval means as per-step recording."""
    from sheeprl_prey_amd.utils.metric import MeanMetric, MetricAggregator
    from tests.test_sac_gpu import _batch, _sac

    tr, _ = _sac(False)
    assert tr.fused is not None
    tr_d, _ = _sac(False, droq=True)
    assert tr_d.fused is None
    keys = ("Loss/value_loss", "Loss/policy_loss", "Loss/alpha_loss")
    agg = MetricAggregator({k: MeanMetric() for k in keys})
    seen = {k: [] for k in keys}
    for i in range(5):
        tr.train(_batch(seed=i), do_ema=True, aggregator=agg)
        torch.cuda.synchronize()
        seen["Loss/value_loss"].append(float(tr._st["qf_loss"]))
        seen["Loss/policy_loss"].append(float(tr._st["actor_loss"]))
        seen["Loss/alpha_loss"].append(float(tr._st["alpha_loss"]))
    got = agg.compute()
    for k in keys:
        assert abs(got[k] - float(np.mean(seen[k]))) <= 1e-5 * max(1.0, abs(got[k])), (k, got[k], seen[k])
    agg.reset()
    assert float(tr.fused.acc.abs().sum()) == 0.0
