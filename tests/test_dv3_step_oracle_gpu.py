"""Whole-train-step oracle at the headline bench shape (B 16 x T 64, H 15, dense 512, cnn mult 32, deter 512,
stoch 32x32, 9 actions; ``exp=dreamer_v3_100k_ms_pacman``), and the same step with a multi-discrete [3, 2] action
space (two actor heads: the ``nh > 1`` branches of the imagination kernels, the per-head unimix and the
multi-head actor loss; reference ``tests/test_algos/test_algos.py:562-564`` runs every algorithm on
``multidiscrete_dummy``).

The fused + hipGraph-replayed ``DreamerV3Trainer`` step (HIP kernels, recorded-forward reuse, one-hot
gathers, device-side clipping) is compared with the SAME step run eagerly through the fp32 reference
ops (``fabric.fused_ops=False`` / ``ops.set_fused(False)``: ``ops/reference.py`` + stock torch modules, the
reference's ``dreamer_v3.py:51-351`` math), from the same weights, optimiser state and batch.

Discrete samples are the one thing two correct implementations do not share: a categorical draw whose
uniform falls within rounding distance of a CDF boundary flips, and the flip propagates through the
recurrence.  So the eager run is teacher-forced (``DreamerV3Trainer.teacher``) with the fused run's
posterior / prior / action samples; everything else - every forward, every straight-through and data
gradient, the losses, Moments, the lambda returns, the clip norms - is computed independently.

Compared: all 13 step metrics, and the first Adam moment of each flat slab (world model, actor, critic).
From a zero optimiser state, ``exp_avg = (1 - beta1) * clip_coef * grad`` exactly, so it is the clipped
gradient slab each optimiser applied.  The per-slab and per-parameter errors are printed (``-s``)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

T, B = 64, 16


def _build(adim):
    from sheeprl_prey_amd.algos.dreamer_v3.agent import build_models
    from sheeprl_prey_amd.algos.dreamer_v3.dreamer_v3 import DreamerV3Trainer
    from sheeprl_prey_amd.algos.dreamer_v3.utils import Moments
    from sheeprl_prey_amd.config.compose import compose
    from sheeprl_prey_amd.envs import spaces
    from sheeprl_prey_amd.parallel.flat_optim import build_optimizer
    from sheeprl_prey_amd.parallel.runner import Runner
    from sheeprl_prey_amd.utils.utils import dotdict

    cfg = dotdict(compose(["exp=dreamer_v3_100k_ms_pacman", "env=synthetic_atari", "cnn_keys.encoder=[rgb]",
                           "cnn_keys.decoder=[rgb]", "fabric.accelerator=cuda", "fabric.cuda_graphs=True"]))
    runner = Runner(**dict(cfg.fabric))
    torch.manual_seed(0)
    obs_space = spaces.Dict({"rgb": spaces.Box(0, 255, (3, 64, 64), "uint8")})
    wm, actor, critic, target = build_models(runner, adim, False, cfg, obs_space)
    opts = [build_optimizer(c, m.parameters()) for c, m in
            ((cfg.algo.world_model.optimizer, wm), (cfg.algo.actor.optimizer, actor), (cfg.algo.critic.optimizer, critic))]
    moments = Moments(None, cfg.algo.actor.moments.decay, cfg.algo.actor.moments.max,
                      cfg.algo.actor.moments.percentile.low, cfg.algo.actor.moments.percentile.high).cuda()
    tr = DreamerV3Trainer(runner, cfg, wm, actor, critic, target, *opts, moments, False, adim)
    return tr, opts, moments


def _data(adim):
    g = torch.Generator(device="cuda").manual_seed(1)
    acts = torch.cat([torch.nn.functional.one_hot(torch.randint(0, a, (T, B), device="cuda", generator=g), a).float()
                      for a in adim], -1)
    return {
        "rgb": torch.randint(0, 255, (T, B, 3, 64, 64), dtype=torch.uint8, device="cuda", generator=g),
        "actions": acts,
        "rewards": torch.randn(T, B, 1, device="cuda", generator=g),
        "dones": (torch.rand(T, B, 1, device="cuda", generator=g) < 0.02).float(),
        "is_first": (torch.rand(T, B, 1, device="cuda", generator=g) < 0.02).float(),
    }


def _state(tr, opts, moments):
    t = {}
    for j, o in enumerate(opts):
        for k in ("flat_param", "exp_avg", "exp_avg_sq", "scalars"):
            t[(j, k)] = getattr(o, k)
    t["target"] = tr.target_flat
    for n, b in moments.named_buffers():
        t[("moments", n)] = b
    return t


def _rel(a: torch.Tensor, b: torch.Tensor) -> float:
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


@pytest.mark.parametrize("adim", [[9], [3, 2]], ids=["discrete9", "multidiscrete3x2"])
def test_dv3_fused_graphed_step_matches_eager_reference_step(adim):
    from sheeprl_prey_amd import ops
    from sheeprl_prey_amd.algos.dreamer_v3.dreamer_v3 import METRIC_KEYS

    tr, opts, moments = _build(adim)
    data = _data(adim)
    tr.update_target(1.0)
    snap = {k: v.detach().clone() for k, v in _state(tr, opts, moments).items()}
    for _ in range(3):  # 2 warm-up steps, then capture (+ one replay)
        tr.train_step(data)
    assert tr.graphed.graph is not None

    def restore():
        for k, v in _state(tr, opts, moments).items():
            v.copy_(snap[k])

    # ---- fused + graphed
    restore()
    torch.cuda.manual_seed(5)
    out_f = {k: v.detach().clone() for k, v in tr.train_step(data).items()}
    m_f = [o.exp_avg.clone() for o in opts]
    st = tr._st
    S = 32 * 32
    teacher = {"posteriors": st["posteriors"].reshape(T, B, S).clone(),
               "priors": st["imagined_trajectories"][..., :S].clone(),
               "actions": st["imagined_actions"].clone()}
    assert torch.equal(teacher["posteriors"].sum(-1), torch.full((T, B), 32.0, device="cuda"))  # exact one-hots
    # ---- eager reference ops, teacher-forced samples
    restore()
    ops.set_fused(False)
    tr.graphed.enabled = False
    tr.teacher = teacher
    try:
        out_e = {k: v.detach().clone() for k, v in tr.train_step(data).items()}
        torch.cuda.synchronize()
    finally:
        ops.set_fused(True)
        tr.graphed.enabled = True
        tr.teacher = None
    m_e = [o.exp_avg.clone() for o in opts]
    # the eager run consumed the forced samples (same discrete latents / actions as the fused run; the eager
    # straight-through value (onehot + p) - p is the one-hot up to one rounding)
    torch.testing.assert_close(tr._st["imagined_actions"], teacher["actions"], rtol=0, atol=1e-6)

    assert set(METRIC_KEYS) <= set(out_f) and set(METRIC_KEYS) <= set(out_e)
    report = []
    for k in METRIC_KEYS:
        a, b = float(out_f[k]), float(out_e[k])
        err = abs(a - b) / max(abs(b), 1e-3)
        report.append((k, a, b, err))
    for name, o, a, b in zip(("world_model", "actor", "critic"), opts, m_f, m_e):
        worst = max((_rel(a[off:off + p.numel()], b[off:off + p.numel()]), i)
                    for i, (p, off) in enumerate(zip(o.params, o.offsets))
                    if float(b[off:off + p.numel()].norm()) > 1e-6 * float(b.norm()))
        report.append((f"grad slab {name}", float(a.norm()), float(b.norm()), _rel(a, b), worst))
    for r in report:
        print("ORACLE", r)
    for k, a, b, err in report[:len(METRIC_KEYS)]:
        assert err < 2e-3, (k, a, b, err)
    for name, na, nb, err, (worst, i) in report[len(METRIC_KEYS):]:
        assert err < 2e-3, (name, err)
        assert worst < 1e-2, (name, "parameter", i, worst)
