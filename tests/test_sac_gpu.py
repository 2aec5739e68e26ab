"""SAC family on the GPU: fused squashed-Gaussian kernel vs the fp32 PyTorch reference, and the
captured (hipGraph) critic/actor updates vs the eager ones."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("A", [1, 2, 6, 17, 64])
def test_squashed_gaussian_kernel_matches_reference(mode, A):
    from sheeprl_prey_amd import ops
    from sheeprl_prey_amd.ops import reference as ref

    torch.manual_seed(A)
    R = 1000
    lo, hi = (-5.0, 2.0) if mode == 0 else (-10.0, 2.0)
    mean = torch.randn(R, A, device="cuda", requires_grad=True)
    raw = (torch.randn(R, A, device="cuda") * 3).requires_grad_()
    eps = torch.randn(R, A, device="cuda")
    scale = torch.rand(A, device="cuda") + 0.5
    bias = torch.randn(A, device="cuda")
    a, lp = ops.squashed_gaussian(mean, raw, scale, bias, mode, lo, hi, eps=eps)
    m2 = mean.detach().clone().requires_grad_()
    r2 = raw.detach().clone().requires_grad_()
    a2, lp2 = ref.squashed_gaussian(m2, r2, eps, scale, bias, mode, lo, hi)
    torch.testing.assert_close(a, a2, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(lp, lp2, rtol=1e-4, atol=1e-3)
    ga = torch.randn_like(a)
    gl = torch.randn_like(lp)
    torch.autograd.backward([a, lp], [ga, gl])
    torch.autograd.backward([a2, lp2], [ga, gl])
    torch.testing.assert_close(mean.grad, m2.grad, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(raw.grad, r2.grad, rtol=1e-3, atol=1e-3)


def _sac(graphs: bool, droq: bool = False, seed: int = 0):
    from sheeprl_prey_amd.algos.sac.agent import build_agent
    from sheeprl_prey_amd.algos.sac.sac import SACTrainer
    from sheeprl_prey_amd.config.compose import compose
    from sheeprl_prey_amd.envs import spaces
    from sheeprl_prey_amd.parallel.flat_optim import build_optimizer
    from sheeprl_prey_amd.parallel.runner import Runner
    from sheeprl_prey_amd.utils.utils import dotdict

    cfg = dotdict(compose(["exp=droq" if droq else "exp=sac", "fabric.accelerator=cuda",
                           f"fabric.cuda_graphs={graphs}"]))
    torch.manual_seed(seed)
    runner = Runner(**dict(cfg.fabric))
    act = spaces.Box(-2.0, 2.0, (3,))
    agent = build_agent(runner, cfg, 11, act, dropout=0.0, layer_norm=droq)
    qf = build_optimizer(cfg.algo.critic.optimizer, agent.critic.parameters())
    ao = build_optimizer(cfg.algo.actor.optimizer, agent.actor.parameters())
    al = build_optimizer(cfg.algo.alpha.optimizer, [agent.log_alpha])
    return SACTrainer(runner, cfg, agent, ao, qf, al, actor_q_reduce="mean" if droq else "min"), agent


def _batch(B=256, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return {
        "observations": torch.randn(B, 11, device="cuda", generator=g),
        "next_observations": torch.randn(B, 11, device="cuda", generator=g),
        "actions": torch.rand(B, 3, device="cuda", generator=g) * 4 - 2,
        "rewards": torch.randn(B, 1, device="cuda", generator=g),
        "dones": (torch.rand(B, 1, device="cuda", generator=g) < 0.05).float(),
    }


@pytest.mark.parametrize("droq", [False, True])
def test_sac_graph_matches_eager(droq):
    """Same init, same batches, same RNG seed before every update: the hipGraph replays must
    reproduce the eager updates (Philox offsets are replayed graph-safely)."""
    from sheeprl_prey_amd.utils.metric import MeanMetric, MetricAggregator

    res = []
    for graphs in (False, True):
        tr, agent = _sac(graphs, droq)
        agg = MetricAggregator({k: MeanMetric() for k in ("Loss/value_loss", "Loss/policy_loss", "Loss/alpha_loss")})
        for i in range(6):
            torch.manual_seed(100 + i)
            tr.train(_batch(seed=i), do_ema=(i % 2 == 0), aggregator=agg)
        torch.cuda.synchronize()
        if graphs:
            assert tr.critic_step.mode == "single" and tr.critic_step._impl.graph is not None
        res.append((torch.cat([p.detach().reshape(-1) for p in agent.parameters()]),
                    torch.cat([p.detach().reshape(-1) for p in agent.critic_target.parameters()]), agg.compute()))
    (p0, t0, m0), (p1, t1, m1) = res
    torch.testing.assert_close(p1, p0, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(t1, t0, rtol=1e-4, atol=1e-5)
    for k in m0:
        assert abs(m0[k] - m1[k]) <= 1e-3 * max(1.0, abs(m0[k])), (k, m0[k], m1[k])


def test_sac_graph_learns_a_bandit():
    """Q regression on a fixed reward must converge under the captured update."""
    tr, agent = _sac(True)
    b = _batch()
    b["dones"] = torch.ones_like(b["dones"])  # pure regression to the reward
    first = last = None
    for i in range(300):
        d = dict(b)
        out = dict(tr.critic_step({**d, "ema_w": tr.ema_weight(True, "cuda")}))
        v = float(out["Loss/value_loss"])
        first = v if first is None else first
        last = v
    assert last < 0.2 * first, (first, last)


@pytest.mark.parametrize("n,H,obs_dim,act_dim,M", [(2, 256, 17, 6, 256), (2, 128, 24, 8, 100), (3, 256, 3, 1, 64)])
def test_sac_twin_q_target_kernel_matches_eager(n, H, obs_dim, act_dim, M):
    """K15: the fused target (n target critics, min, entropy term, Bellman target) vs the eager
    ensemble evaluation (reference ``sac/agent.py:256-275``)."""
    from sheeprl_prey_amd import ops
    from sheeprl_prey_amd.algos.sac.agent import SACCriticEnsemble

    torch.manual_seed(n * H + M)
    crit = SACCriticEnsemble(obs_dim + act_dim, n=n, hidden_size=H).cuda()
    obs = torch.randn(M, obs_dim, device="cuda")
    act = torch.rand(M, act_dim, device="cuda") * 2 - 1
    logp = torch.randn(M, 1, device="cuda")
    rew = torch.randn(M, 1, device="cuda")
    done = (torch.rand(M, 1, device="cuda") < 0.2).float()
    log_alpha = torch.tensor([-1.3], device="cuda")
    gamma = 0.99
    with torch.no_grad():
        q = crit(obs, act)
        ref = rew + (1 - done) * gamma * (q.min(-1, keepdim=True)[0] - log_alpha.exp() * logp)
        got = ops.sac_twin_q_target(crit.model, obs, act, logp, rew, done, log_alpha, gamma)
    assert got is not None and got.shape == ref.shape
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("n,H,obs_dim,act_dim,M", [(2, 256, 24, 6, 256), (2, 128, 17, 8, 100), (3, 512, 3, 1, 64),
                                                   (2, 256, 10, 6, 33)])
def test_sac_critic_fused_loss_and_grads_match_eager(n, H, obs_dim, act_dim, M):
    """K15: the fused twin-Q critic update (forward + MSE loss + backward, csrc/sac_critic.hip) vs the
    eager ensemble + ``critic_loss`` autograd (reference sac/agent.py:256-275, sac/loss.py:15-20)."""
    from sheeprl_prey_amd import ops
    from sheeprl_prey_amd.algos.sac.agent import SACCriticEnsemble
    from sheeprl_prey_amd.algos.sac.loss import critic_loss

    torch.manual_seed(7 * n + H + M)
    crit = SACCriticEnsemble(obs_dim + act_dim, n=n, hidden_size=H).cuda()
    obs = torch.randn(M, obs_dim, device="cuda")
    act = torch.rand(M, act_dim, device="cuda") * 2 - 1
    y = torch.randn(M, 1, device="cuda")
    params = list(crit.parameters())
    q_ref = crit(obs, act)
    loss_ref = critic_loss(q_ref, y, n)
    g_ref = torch.autograd.grad(loss_ref * 0.7, params)
    res = ops.sac_critic_loss(crit.model, obs, act, y)
    assert res is not None
    loss, q = res
    torch.testing.assert_close(q, q_ref.detach(), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(loss, loss_ref.detach(), rtol=1e-4, atol=1e-5)
    g = torch.autograd.grad(loss * 0.7, params)
    names = [nm for nm, _ in crit.named_parameters()]
    for nm, a, b in zip(names, g, g_ref):
        torch.testing.assert_close(a, b, rtol=1e-3, atol=1e-5, msg=lambda m, nm=nm: f"{nm}: {m}")
