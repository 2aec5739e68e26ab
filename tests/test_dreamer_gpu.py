"""DreamerV3 train step on the GPU: fused + hipGraph path vs eager path."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _build(graphs: bool, seed: int = 0, continuous: bool = False, cnn_mult: int = 8, extra=()):
    from sheeprl_prey_amd.algos.dreamer_v3.agent import build_models
    from sheeprl_prey_amd.algos.dreamer_v3.dreamer_v3 import DreamerV3Trainer
    from sheeprl_prey_amd.algos.dreamer_v3.utils import Moments
    from sheeprl_prey_amd.config.compose import compose
    from sheeprl_prey_amd.envs import spaces
    from sheeprl_prey_amd.parallel.flat_optim import build_optimizer
    from sheeprl_prey_amd.parallel.runner import Runner
    from sheeprl_prey_amd.utils.utils import dotdict

    cfg = dotdict(compose([
        "exp=dreamer_v3", "env=dummy", "cnn_keys.encoder=[rgb]", "cnn_keys.decoder=[rgb]", "algo.dense_units=64",
        "algo.mlp_layers=2", f"algo.world_model.encoder.cnn_channels_multiplier={cnn_mult}",
        "algo.world_model.recurrent_model.recurrent_state_size=64", "algo.world_model.representation_model.hidden_size=64",
        "algo.world_model.transition_model.hidden_size=64", "algo.horizon=5", "fabric.accelerator=cuda",
        f"fabric.cuda_graphs={graphs}", *extra,
    ]))
    torch.manual_seed(seed)
    runner = Runner(**dict(cfg.fabric))
    obs_space = spaces.Dict({"rgb": spaces.Box(0, 255, (3, 64, 64), "uint8")})
    adim = [3] if continuous else [5]
    wm, actor, critic, target = build_models(runner, adim, continuous, cfg, obs_space)
    opts = [build_optimizer(c, m.parameters()) for c, m in
            ((cfg.algo.world_model.optimizer, wm), (cfg.algo.actor.optimizer, actor), (cfg.algo.critic.optimizer, critic))]
    trainer = DreamerV3Trainer(runner, cfg, wm, actor, critic, target, *opts, Moments(None).cuda(), continuous, adim)
    return trainer


def _data(T=16, B=4, seed=1, continuous=False):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return {
        "rgb": torch.randint(0, 255, (T, B, 3, 64, 64), dtype=torch.uint8, device="cuda", generator=g),
        "actions": (torch.rand(T, B, 3, device="cuda", generator=g) * 2 - 1) if continuous else
        torch.nn.functional.one_hot(torch.randint(0, 5, (T, B), device="cuda", generator=g), 5).float(),
        "rewards": torch.randn(T, B, 1, device="cuda", generator=g),
        "dones": (torch.rand(T, B, 1, device="cuda", generator=g) < 0.1).float(),
        "is_first": (torch.rand(T, B, 1, device="cuda", generator=g) < 0.1).float(),
    }


def test_dv3_train_step_graph_runs_and_learns():
    tr = _build(graphs=True)
    losses = []
    data = _data()
    for i in range(8):
        out = tr.train_step(data)
        losses.append(float(out["Loss/world_model_loss"]))
    assert tr.graphed.graph is not None, "hipGraph was not captured"
    assert all(l == l for l in losses)
    assert losses[-1] < losses[0], losses


def test_dv3_graph_matches_eager_losses():
    """Same seed, same data: eager and graphed steps must agree (same RNG streams are not
    guaranteed across capture, so compare the deterministic world-model loss of step 1)."""
    a = _build(graphs=False, seed=3)
    b = _build(graphs=True, seed=3)
    data = _data(seed=7)
    torch.manual_seed(11)
    la = float(a.train_step(data)["Loss/observation_loss"])
    torch.manual_seed(11)
    lb = float(b.train_step(data)["Loss/observation_loss"])
    assert abs(la - lb) / abs(la) < 1e-4


@pytest.mark.parametrize("impl", ["persist", "scan4", "scan9"])
@pytest.mark.parametrize("H,D,hid,B,T", [(64, 64, 64, 4, 16), (512, 512, 512, 16, 8), (96, 80, 48, 3, 5),
                                         (256, 1024, 256, 16, 8)])  # the prey preset: deter 256, dense 1024
def test_fused_rssm_scan_matches_python_scan(H, D, hid, B, T, impl):
    """The fused scans (persist: one persistent launch per direction; scan4: 4+4 MFMA launches/step;
    scan9: 9+9 launches/step; batched weight grads) vs the python step loop, same noise.  D = 1024 (the prey
    preset) runs the persistent scan's wide-input form (fwd_kernel_big / bwd_kernel_big)."""
    _check_scan_vs_python(H, D, hid, B, T, impl)


def test_persistent_scan_prey_shape_T64():
    """The fork's own preset (exp=dreamer_v3_prey: deter 256, dense 1024, hidden 256, stoch 32x32) through the
    persistent scan's wide-input form over a whole B 16 x T 64 sequence, fwd + bwd vs the python loop."""
    _check_scan_vs_python(256, 1024, 256, 16, 64, "persist", tol=(5e-3, 5e-4), gtol=(5e-3, 5e-3))


@pytest.mark.parametrize("impl", ["persist", "scan4"])
def test_fused_rssm_scan_full_shape_T64(impl):
    """Atari-100k shape over the whole sequence (B 16, T 64, H = D = hid = 512): the fast
    sigmoid/tanh forms and the in-launch hand-offs must hold through 64 recurrent steps, fwd + bwd."""
    _check_scan_vs_python(512, 512, 512, 16, 64, impl, tol=(5e-3, 5e-4), gtol=(5e-3, 5e-3))


def test_fused_rssm_scan_xl_shape():
    """DreamerV3-XL recurrent shape (deter 4096, dense 1024, hidden 1024; reference
    ``configs/exp/dreamer_v3_XL_crafter.yaml``): beyond the register/LDS-resident scans, the
    per-step scan with the skinny split-K weight-streaming GEMMs, fwd + bwd vs the python loop."""
    _check_scan_vs_python(4096, 1024, 1024, 16, 6, "persist", tol=(5e-3, 5e-4), gtol=(5e-3, 5e-3), expect="scan9")


def _check_scan_vs_python(H, D, hid, B, T, impl, tol=(2e-3, 2e-4), gtol=(3e-3, 3e-3), expect=None):
    import copy

    from sheeprl_prey_amd.algos.dreamer_v3.agent import RSSM, RecurrentModel, init_weights
    from sheeprl_prey_amd.models.models import MLP

    torch.manual_seed(0)
    S, A, E = 32 * 32, 6, 200
    rec = RecurrentModel(S + A, H, D)
    rep = MLP(H + E, S, [hid], activation=torch.nn.SiLU, norm_layer=[torch.nn.LayerNorm], norm_args=[{"normalized_shape": hid}])
    tr = MLP(H, S, [hid], activation=torch.nn.SiLU, norm_layer=[torch.nn.LayerNorm], norm_args=[{"normalized_shape": hid}])
    rssm = RSSM(rec.apply(init_weights), rep.apply(init_weights), tr.apply(init_weights), {"validate_args": False}).cuda()
    for p in rssm.parameters():  # non-trivial LN affine params
        if p.dim() == 1:
            p.data.add_(0.1 * torch.randn_like(p))
    rssm_ref = copy.deepcopy(rssm)
    rssm_ref.fused_scan = False
    rssm.scan_impl = impl
    emb = torch.randn(T, B, E, device="cuda")
    act = torch.nn.functional.one_hot(torch.randint(0, A, (T, B), device="cuda"), A).float()
    first = (torch.rand(T, B, 1, device="cuda") < 0.2).float()
    first[0] = 1
    uni = torch.rand(T, 2 * B * 32, device="cuda")
    # python scan consumes one uniform per posterior categorical: feed it the posterior half
    uni_post = uni.view(T, 2, B * 32)[:, 1].reshape(T, B, 32)
    e1, e2 = emb.clone().requires_grad_(), emb.clone().requires_grad_()
    out1 = rssm.scan_dynamic(e1, act, first, uniform=uni)
    out2 = rssm_ref.scan_dynamic(e2, act, first, uniform=uni_post)
    fn = {"persist": "RSSMPersistFnBackward", "scan4": "RSSMScan4FnBackward", "scan9": "RSSMScanFnBackward"}[expect or impl]
    assert type(out1[0].grad_fn).__name__ == fn
    names = ["h", "post", "post_logits", "prior_logits"]
    for n, a, b in zip(names, out1, out2):
        torch.testing.assert_close(a, b, rtol=tol[0], atol=tol[1], msg=lambda m: f"{n}: {m}")
    sync = out1[0].grad_fn.saved_tensors[34] if (expect or impl) == "persist" else None  # hand-off counters + error word
    gs = [torch.randn_like(o) for o in out1]
    sum((o * g).sum() for o, g in zip(out1, gs)).backward()
    sum((o * g).sum() for o, g in zip(out2, gs)).backward()
    if sync is not None:
        from sheeprl_prey_amd.ops.rssm import scanp_error

        assert scanp_error(sync) == 0, "a persistent-scan hand-off timed out"
    torch.testing.assert_close(e1.grad, e2.grad, rtol=gtol[0], atol=gtol[1])
    for (n, p1), p2 in zip(rssm.named_parameters(), rssm_ref.parameters()):
        torch.testing.assert_close(p1.grad, p2.grad, rtol=gtol[0], atol=gtol[1], msg=lambda m: f"{n}: {m}")


@pytest.mark.parametrize("continuous", [False, True])
def test_dv3_segmented_graph_matches_single_graph(continuous):
    """Multi-rank execution mode (one hipGraph per phase, collectives between replays) forced on one
    rank must reproduce the single-graph step - for continuous actors too, whose actor loss
    back-propagates through the imagination graph recorded in the previous phase's capture."""
    a = _build(graphs=True, seed=5, continuous=continuous)
    b = _build(graphs=True, seed=5, continuous=continuous)
    from sheeprl_prey_amd.algos.dreamer_v3.dreamer_v3 import DreamerV3Trainer

    b2 = DreamerV3Trainer(b.runner, b.cfg, b.world_model, b.actor, b.critic, b.target_critic, b.world_optimizer,
                          b.actor_optimizer, b.critic_optimizer, b.moments, continuous, b.actions_dim, force_segmented=True)
    data = _data(seed=9, continuous=continuous)
    la, lb = [], []
    for i in range(5):
        torch.manual_seed(100 + i)
        la.append(float(a.train_step(data)["Loss/world_model_loss"]))
        torch.manual_seed(100 + i)
        lb.append(float(b2.train_step(data)["Loss/world_model_loss"]))
    assert b2.seg.graphs is not None and a.graphed.graph is not None
    assert la[-1] < la[0] and lb[-1] < lb[0]
    # both executions train (identical math; RNG streams differ once graphs replay)
    assert abs(la[1] - lb[1]) / abs(la[1]) < 1e-3, (la, lb)
    for k in ("Loss/policy_loss", "Loss/value_loss"):
        assert torch.isfinite(b2.seg.static_out[k]).all()


@pytest.mark.parametrize("merge", [True, False])
def test_imagine_discrete_matches_reference_loop(monkeypatch, merge):
    """Buffer-resident no-grad imagination (RSSM.imagine_discrete) vs the reference loop
    (RSSM.imagination + Actor per step).  imagine_discrete draws every uniform of the rollout in one
    launch, U [H+1, M*(heads + groups)] (actions first, then the prior groups, per step); the
    reference loop is fed the same slices in its call order, so the sampled trajectories agree up to
    rare category flips from GEMM rounding.  merge: every GEMM over h_{t+1} as one (the default) or separate."""
    from sheeprl_prey_amd import ops
    from sheeprl_prey_amd.algos.dreamer_v3.agent import RSSM

    monkeypatch.setattr(RSSM, "_merge_h_ok", "1" if merge else "0")
    tr = _build(graphs=False)
    wm, actor = tr.world_model, tr.actor
    M, S, H, Hz = 96, 32 * 32, 64, 4
    g = torch.Generator(device="cuda").manual_seed(3)
    post = torch.nn.functional.one_hot(torch.randint(0, 32, (M, 32), device="cuda", generator=g), 32).float().view(M, S)
    h = torch.randn(M, H, device="cuda", generator=g)
    assert wm.rssm.imagine_fast_ok(actor)
    torch.manual_seed(7)
    traj, acts = wm.rssm.imagine_discrete(post, h, actor, Hz)
    torch.manual_seed(7)
    U = torch.rand(Hz + 1, M * (1 + S // 32), device="cuda")
    feed = iter([U[t, :M] if i == 0 else U[t, M:] for t in range(Hz + 1) for i in range(2)])
    real = ops.unimix_sample

    def fed(logits, classes, unimix=0.01, sample=True, uniform=None, forced=None):
        return real(logits, classes, unimix, sample=sample, uniform=next(feed) if sample else None)

    monkeypatch.setattr(ops, "unimix_sample", fed)
    with torch.no_grad():
        prior, hh = post, h
        lat = torch.cat((prior, hh), -1)
        ref_t, ref_a = [lat], [torch.cat(actor(lat)[0], -1)]
        for _ in range(Hz):
            prior, hh = wm.rssm.imagination(prior, hh, ref_a[-1])
            prior = prior.reshape(M, S)
            lat = torch.cat((prior, hh), -1)
            ref_t.append(lat)
            ref_a.append(torch.cat(actor(lat)[0], -1))
    ref_t, ref_a = torch.stack(ref_t), torch.stack(ref_a)
    assert traj.shape == ref_t.shape and acts.shape == ref_a.shape
    torch.testing.assert_close(traj[0], ref_t[0])
    # rows whose sampled prefix matched must match exactly in h (one-step GEMM rounding only)
    same_rows = (traj[:, :, :S] == ref_t[:, :, :S]).all(-1).all(0) & (acts == ref_a).all(-1).all(0)
    assert same_rows.float().mean() > 0.95, same_rows.float().mean()
    torch.testing.assert_close(traj[:, same_rows], ref_t[:, same_rows], rtol=1e-4, atol=1e-4)


def test_player_graphed_steps_and_resets():
    from sheeprl_prey_amd.algos.dreamer_v3.agent import PlayerDV3

    tr = _build(graphs=True)
    wm, actor = tr.world_model, tr.actor
    player = PlayerDV3(wm.encoder, wm.rssm, actor, [5], 0.0, 3, 32, 64, torch.device("cuda"), discrete_size=32)
    player.use_graphs = True
    player.init_states()
    h0 = player.recurrent_state.clone()
    z0 = player.stochastic_state.clone()
    buf_ptr = player.recurrent_state.data_ptr()
    for _ in range(5):
        obs = {"rgb": torch.rand(1, 3, 3, 64, 64, device="cuda")}
        acts = player.get_exploration_action(obs, False)
        a = acts[0]
        assert a.shape == (1, 3, 5)
        assert torch.all(a.sum(-1) == 1)
    # expl_amount 0: the capture without the exploration ops
    assert set(player._graphed) == {False} and player._graphed[False].graph is not None
    assert player.recurrent_state.data_ptr() == buf_ptr, "state must stay in the captured buffers"
    # a nonzero amount switches to the exploring capture over the same state buffers
    player.expl_amount = 0.5
    for _ in range(4):
        obs = {"rgb": torch.rand(1, 3, 3, 64, 64, device="cuda")}
        a = player.get_exploration_action(obs, False)[0]
        assert a.shape == (1, 3, 5) and torch.all(a.sum(-1) == 1)
    assert set(player._graphed) == {False, True} and player._graphed[True].graph is not None
    assert player.recurrent_state.data_ptr() == buf_ptr
    player.expl_amount = 0.0
    assert not torch.equal(player.recurrent_state, h0)
    player.init_states([1])
    torch.testing.assert_close(player.recurrent_state[:, 1], h0[:, 1])
    torch.testing.assert_close(player.stochastic_state[:, 1], z0[:, 1])
    assert torch.all(player.actions[:, 1] == 0)
    player.init_states()
    assert player.recurrent_state.data_ptr() == buf_ptr
    torch.testing.assert_close(player.recurrent_state, h0)
    # the single-env test episode after training on 3 envs (utils.test): new state shapes, captures dropped
    player.num_envs = 1
    player.init_states()
    assert player._graphed is None and player.recurrent_state.shape[1] == 1
    a = player.get_greedy_action({"rgb": torch.rand(1, 1, 3, 64, 64, device="cuda")}, False)[0]
    assert a.shape == (1, 1, 5) and torch.all(a.sum(-1) == 1)


@pytest.mark.parametrize("graphs", [False, True])
def test_dv3_forward_reuse_matches_recompute(graphs):
    """Recorded actor trunk + reused critic forward (``reuse_forwards``) vs the reference-shaped second
    forwards: same losses and the same updated weights after one step from the same state/RNG."""
    import copy

    tr = _build(graphs=False)
    data = _data()
    tr.train_step(data)  # move off the initial state (Moments, Adam moments)
    torch.cuda.synchronize()
    opts = (tr.world_optimizer, tr.actor_optimizer, tr.critic_optimizer)
    snap = [(o.flat_param.clone(), o.exp_avg.clone(), o.exp_avg_sq.clone(), o.scalars.clone()) for o in opts]
    msnap = copy.deepcopy(tr.moments.state_dict())
    results = []
    for reuse in (False, True):
        for o, (p, m, v, sc) in zip(opts, snap):
            o.flat_param.copy_(p); o.exp_avg.copy_(m); o.exp_avg_sq.copy_(v); o.scalars.copy_(sc)
        tr.moments.load_state_dict(msnap)
        tr.reuse_forwards = reuse
        tr.graphed.enabled = graphs
        tr.graphed.graph = None
        tr.graphed._calls = 0
        torch.manual_seed(123)
        torch.cuda.manual_seed(123)
        if graphs:
            tr.graphed.warmup = 0
        out = tr.train_step(data)
        torch.cuda.synchronize()
        results.append(({k: float(v) for k, v in out.items()}, [o.flat_param.clone() for o in opts]))
    (o0, p0), (o1, p1) = results
    for k in ("Loss/policy_loss", "Loss/value_loss", "Grads/actor", "Grads/critic"):
        assert abs(o0[k] - o1[k]) <= 1e-4 * max(1.0, abs(o0[k])), (k, o0[k], o1[k])
    for a, b in zip(p0, p1):
        torch.testing.assert_close(b, a, rtol=1e-4, atol=1e-5)


def test_persistent_scan_timeout_is_loud():
    """A starved hand-off must not pass silently: with every wait bounded to one poll the persistent
    scan's waits time out, the grid drains, the sticky health word records the waits and the host check
    raises; with the default bound a step is healthy again."""
    from sheeprl_prey_amd.ops import rssm as R

    tr = _build(graphs=False)
    data = _data()
    tr.train_step(data)
    torch.cuda.synchronize()
    assert R.check_scan_health() == 0
    from sheeprl_prey_amd import ops

    ops.skipped_updates(reset=True)
    opts = (tr.world_optimizer, tr.actor_optimizer, tr.critic_optimizer)
    try:
        R.set_scan_spin_max(1)
        before = [(o.flat_param.clone(), o.exp_avg.clone(), o.exp_avg_sq.clone(), float(o.scalars[0])) for o in opts]
        tr.train_step(data)
        torch.cuda.synchronize()
        # the faulted step's updates were skipped on the device: weights, moments and step counts bit-unchanged
        for o, (p, m, v, t) in zip(opts, before):
            assert torch.equal(o.flat_param, p) and torch.equal(o.exp_avg, m) and torch.equal(o.exp_avg_sq, v)
            assert float(o.scalars[0]) == t
        assert ops.skipped_updates(reset=True) == 3
        with pytest.raises(RuntimeError, match="hand-off wait timed out"):
            R.check_scan_health()
    finally:
        R.set_scan_spin_max(0)
    assert R.check_scan_health() == 0  # the check cleared the word
    p0 = tr.world_optimizer.flat_param.clone()
    tr.train_step(data)
    torch.cuda.synchronize()
    assert R.check_scan_health() == 0
    assert not torch.equal(tr.world_optimizer.flat_param, p0)  # healthy again: the update is applied
    assert ops.skipped_updates() == 0


@pytest.mark.parametrize("graphs,n_act", [(False, 2), (True, 2), (True, 100)])
def test_dv3_vector_obs_train_step(graphs, n_act):
    """Vector observations only (no CNN encoder / decoder: the CartPole-style config), fused ops, with and without
    the captured step: finite losses that decrease on a fixed batch.  n_act = 100: the fork's prey_d_1 action space
    (Discrete(100)), whose actor categorical runs on the wide (one wave per categorical) unimix kernels."""
    from sheeprl_prey_amd.algos.dreamer_v3.agent import build_models
    from sheeprl_prey_amd.algos.dreamer_v3.dreamer_v3 import DreamerV3Trainer
    from sheeprl_prey_amd.algos.dreamer_v3.utils import Moments
    from sheeprl_prey_amd.config.compose import compose
    from sheeprl_prey_amd.envs import spaces
    from sheeprl_prey_amd.parallel.flat_optim import build_optimizer
    from sheeprl_prey_amd.parallel.runner import Runner
    from sheeprl_prey_amd.utils.utils import dotdict

    cfg = dotdict(compose([
        "exp=dreamer_v3", "env=dummy", "cnn_keys.encoder=[]", "cnn_keys.decoder=[]", "mlp_keys.encoder=[state]",
        "mlp_keys.decoder=[state]", "algo.dense_units=64", "algo.mlp_layers=2",
        "algo.world_model.recurrent_model.recurrent_state_size=64", "algo.world_model.representation_model.hidden_size=64",
        "algo.world_model.transition_model.hidden_size=64", "algo.horizon=5", "fabric.accelerator=cuda",
        f"fabric.cuda_graphs={graphs}",
    ]))
    torch.manual_seed(0)
    runner = Runner(**dict(cfg.fabric))
    obs_space = spaces.Dict({"state": spaces.Box(-10, 10, (4,), "float32")})
    wm, actor, critic, target = build_models(runner, [n_act], False, cfg, obs_space)
    opts = [build_optimizer(c, m.parameters()) for c, m in
            ((cfg.algo.world_model.optimizer, wm), (cfg.algo.actor.optimizer, actor), (cfg.algo.critic.optimizer, critic))]
    tr = DreamerV3Trainer(runner, cfg, wm, actor, critic, target, *opts, Moments(None).cuda(), False, [n_act])
    g = torch.Generator(device="cuda").manual_seed(1)
    T, B = 16, 4
    data = {
        "state": torch.randn(T, B, 4, device="cuda", generator=g),
        "actions": torch.nn.functional.one_hot(torch.randint(0, n_act, (T, B), device="cuda", generator=g), n_act).float(),
        "rewards": torch.randn(T, B, 1, device="cuda", generator=g),
        "dones": (torch.rand(T, B, 1, device="cuda", generator=g) < 0.1).float(),
        "is_first": (torch.rand(T, B, 1, device="cuda", generator=g) < 0.1).float(),
    }
    losses = [float(tr.train_step(data)["Loss/world_model_loss"]) for _ in range(8)]
    assert all(l == l and abs(l) < 1e6 for l in losses), losses
    assert losses[-1] < losses[0], losses
    if graphs:
        assert tr.graphed.graph is not None
