"""CPU unit tests: config composition, models, fused-op oracles, flat optimisers, logger, envs."""
from __future__ import annotations

import math
import os

import numpy as np
import pytest
import torch
import torch.nn as nn

from sheeprl_prey_amd import ops
from sheeprl_prey_amd.config.compose import compose
from sheeprl_prey_amd.models.ensemble import EnsembleMLP
from sheeprl_prey_amd.models.models import CNN, MLP
from sheeprl_prey_amd.parallel.flat_optim import FlatAdam, build_optimizer, flatten_like

CONFIG_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "sheeprl_prey_amd", "configs")
PRESETS = sorted(f[:-5] for f in os.listdir(os.path.join(CONFIG_DIR, "exp")) if f.endswith(".yaml") and f != "default.yaml")


# ---------------------------------------------------------------- config
@pytest.mark.parametrize("exp", PRESETS)
def test_every_preset_composes(exp):
    cfg = compose([f"exp={exp}"])
    assert cfg["algo"]["name"] != "???"
    assert "fabric" in cfg and "env" in cfg and "buffer" in cfg
    assert isinstance(cfg["total_steps"], int)


def test_cli_style_overrides():
    cfg = compose(["exp=ppo", "algo.optimizer.lr=0.5", "+new_key=3", "env.num_envs=7"])
    assert cfg["algo"]["optimizer"]["lr"] == 0.5
    assert cfg["new_key"] == 3
    assert cfg["env"]["num_envs"] == 7
    assert cfg["algo"]["name"] == "ppo"


def test_dv3_100k_preset_values():
    cfg = compose(["exp=dreamer_v3_100k_ms_pacman"])
    a = cfg["algo"]
    assert a["world_model"]["recurrent_model"]["recurrent_state_size"] == 512
    assert a["dense_units"] == 512 and a["mlp_layers"] == 2
    assert cfg["per_rank_batch_size"] == 16 and cfg["per_rank_sequence_length"] == 64
    assert a["replay_ratio"] if "replay_ratio" in a else a["train_every"] == 1


# ---------------------------------------------------------------- models
def test_mlp_shapes_and_errors():
    with pytest.raises(ValueError):
        MLP(10)
    m = MLP(10, 3, (16, 16), norm_layer=nn.LayerNorm, norm_args={"normalized_shape": 16})
    assert m(torch.rand(4, 10)).shape == (4, 3)
    assert m(torch.rand(2, 5, 10)).shape == (2, 5, 3)
    m2 = MLP((2, 5), 4, (8,), flatten_dim=1)
    assert m2(torch.rand(3, 2, 5)).shape == (3, 4)


def test_cnn_shapes():
    c = CNN(3, [8, 16], layer_args={"kernel_size": 3, "stride": 2})
    assert c(torch.rand(2, 3, 32, 32)).shape == (2, 16, 7, 7)
    with pytest.raises(ValueError):
        CNN(3, [], layer_args={"kernel_size": 3})


def test_ensemble_equals_separate_mlps():
    torch.manual_seed(0)
    n, d, h = 3, 7, 16
    ens = EnsembleMLP(n, d, (h, h), 1, activation="relu", layer_norm=True)
    x = torch.randn(5, d)
    y = ens(x)  # [n, 5, 1]
    for i in range(n):
        z = x
        for j, lin in enumerate(ens.layers):
            z = z @ lin.weight[i].T + lin.bias[i]
            z = torch.nn.functional.layer_norm(z, (h,), ens.norms[j].weight[i], ens.norms[j].bias[i])
            z = torch.relu(z)
        z = z @ ens.head.weight[i].T + ens.head.bias[i]
        torch.testing.assert_close(y[i], z)


def test_ensemble_member_grads_are_independent():
    ens = EnsembleMLP(2, 4, (8,), 1)
    x = torch.randn(6, 4)
    y = ens(x)
    y[0].sum().backward()
    assert ens.layers[0].weight.grad[1].abs().sum() == 0
    assert ens.layers[0].weight.grad[0].abs().sum() > 0


# ---------------------------------------------------------------- op oracles
@pytest.mark.parametrize("mode", [0, 1])
def test_squashed_gaussian_oracle_matches_torch_distributions(mode):
    torch.manual_seed(0)
    mean = torch.randn(6, 3, requires_grad=True)
    raw = torch.randn(6, 3, requires_grad=True) * 3
    eps = torch.randn(6, 3)
    scale, bias = torch.tensor([1.0, 2.0, 0.5]), torch.tensor([0.0, 1.0, -1.0])
    lo, hi = (-5.0, 2.0) if mode == 0 else (-10.0, 2.0)
    a, lp = ops.squashed_gaussian(mean, raw, scale, bias, mode, lo, hi, eps=eps)
    ls = raw.clamp(lo, hi) if mode == 0 else lo + 0.5 * (hi - lo) * (torch.tanh(raw) + 1)
    dist = torch.distributions.Normal(mean, ls.exp())
    x = mean + ls.exp() * eps
    y = torch.tanh(x)
    lp_ref = (dist.log_prob(x) - torch.log(scale * (1 - y.pow(2)) + 1e-6)).sum(-1, keepdim=True)
    torch.testing.assert_close(a, y * scale + bias)
    # (x-mean)/std recomputed by Normal.log_prob loses digits for std ~ e^-10; the oracle uses eps directly
    torch.testing.assert_close(lp, lp_ref, rtol=1e-4, atol=1e-3)


def test_gae_oracle():
    from sheeprl_prey_amd.ops import reference as ref

    T, B = 5, 2
    r, v, d = torch.rand(T, B, 1), torch.rand(T, B, 1), (torch.rand(T, B, 1) > 0.7).float()
    nv = torch.rand(B, 1)
    ret, adv = ref.gae(r, v, d, nv, 0.99, 0.95)
    # explicit recursion
    last = torch.zeros(B, 1)
    exp = torch.zeros(T, B, 1)
    for t in reversed(range(T)):
        nxt = nv if t == T - 1 else v[t + 1]
        delta = r[t] + 0.99 * nxt * (1 - d[t]) - v[t]
        last = delta + 0.99 * 0.95 * (1 - d[t]) * last
        exp[t] = last
    torch.testing.assert_close(adv, exp)
    torch.testing.assert_close(ret, exp + v)


# ---------------------------------------------------------------- flat optimisers
def test_flat_adam_matches_torch_adam():
    torch.manual_seed(0)
    a = nn.Sequential(nn.Linear(5, 7), nn.Tanh(), nn.Linear(7, 3))
    b = nn.Sequential(nn.Linear(5, 7), nn.Tanh(), nn.Linear(7, 3))
    b.load_state_dict(a.state_dict())
    oa = torch.optim.Adam(a.parameters(), lr=1e-2, eps=1e-5, weight_decay=0.01)
    ob = build_optimizer({"_target_": "torch.optim.Adam", "lr": 1e-2, "eps": 1e-5, "weight_decay": 0.01},
                         b.parameters())
    for _ in range(5):
        x = torch.randn(8, 5)
        for m, o in ((a, oa), (b, ob)):
            o.zero_grad()
            m(x).pow(2).mean().backward()
            o.step()
    for pa, pb in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(pa, pb, rtol=1e-5, atol=1e-6)
    sd = ob.state_dict()
    assert set(sd["state"][0]) == {"step", "exp_avg", "exp_avg_sq"}


def test_flat_clip_matches_torch():
    torch.manual_seed(1)
    a = nn.Linear(4, 4)
    b = nn.Linear(4, 4)
    b.load_state_dict(a.state_dict())
    oa = torch.optim.SGD(a.parameters(), lr=0.1)
    ob = build_optimizer({"_target_": "torch.optim.SGD", "lr": 0.1}, b.parameters())
    x = torch.randn(3, 4) * 10
    for m, o in ((a, oa), (b, ob)):
        o.zero_grad()
        m(x).pow(2).sum().backward()
    torch.nn.utils.clip_grad_norm_(a.parameters(), 0.5)
    ob.clip_grad_norm_(0.5)
    oa.step()
    ob.step()
    for pa, pb in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(pa, pb, rtol=1e-5, atol=1e-6)


def test_shared_slab_optimisers():
    enc, head = nn.Linear(3, 4), nn.Linear(4, 1)
    critic = nn.Sequential(enc, head)
    o_all = FlatAdam(critic.parameters(), lr=0.1)
    o_enc = FlatAdam(enc.parameters(), lr=0.1)
    assert o_enc.flat_param.data_ptr() == o_all.flat_param.data_ptr()
    o_enc.zero_grad()
    enc(torch.randn(2, 3)).sum().backward()
    o_enc.step()
    # writes through the shared storage
    torch.testing.assert_close(enc.weight.view(-1), o_all.flat_param[: enc.weight.numel()])
    with pytest.raises(ValueError):
        FlatAdam(list(head.parameters()) + [nn.Parameter(torch.zeros(2))], lr=0.1)


def test_flatten_like_target_ema():
    src = nn.Linear(3, 2)
    tgt = nn.Linear(3, 2)
    opt = FlatAdam(src.parameters(), lr=0.1)
    flat = flatten_like(tgt, opt)
    before = tgt.weight.detach().clone()
    flat.lerp_(opt.flat_param, 0.25)
    torch.testing.assert_close(tgt.weight, before + 0.25 * (src.weight - before))


# ---------------------------------------------------------------- logger
def test_tfevents_roundtrip(tmp_path):
    from sheeprl_prey_amd.utils.logger import TensorBoardLogger, read_events

    lg = TensorBoardLogger(str(tmp_path), name="run")
    lg.log_metrics({"Loss/a": 1.5, "Loss/b": -2.0}, 3)
    lg.log_metrics({"Loss/a": 0.5}, 4)
    lg.finalize("success")
    files = [os.path.join(dp, f) for dp, _, fs in os.walk(lg.log_dir) for f in fs if "tfevents" in f]
    assert files
    ev = read_events(files[0])
    assert ("Loss/a", 1.5, 3) in [(t, round(v, 4), s) for t, v, s in ev]
    assert ("Loss/a", 0.5, 4) in [(t, round(v, 4), s) for t, v, s in ev]


# ---------------------------------------------------------------- envs
def test_vector_env_autoreset_and_final_info():
    from sheeprl_prey_amd.envs.registry import make
    from sheeprl_prey_amd.envs.core import RecordEpisodeStatistics
    from sheeprl_prey_amd.envs.vector import SyncVectorEnv

    envs = SyncVectorEnv([lambda: RecordEpisodeStatistics(make("CartPole-v1")) for _ in range(2)])
    envs.reset(seed=0)
    saw_final = False
    for _ in range(600):
        _, _, term, trunc, info = envs.step(envs.action_space.sample())
        if np.any(term | trunc):
            assert "final_observation" in info and "final_info" in info
            idx = int(np.nonzero(term | trunc)[0][0])
            assert info["final_info"][idx]["episode"]["l"] > 0
            saw_final = True
            break
    envs.close()
    assert saw_final


def test_make_env_dict_obs_and_frame_stack():
    from sheeprl_prey_amd.utils.env import make_env
    from sheeprl_prey_amd.utils.utils import dotdict

    cfg = dotdict(compose(["exp=dreamer_v3", "env=dummy", "env.id=discrete_dummy", "cnn_keys.encoder=[rgb]",
                           "env.frame_stack=2", "env.screen_size=32"]))
    env = make_env(cfg, 0, 0, None, "test")()
    o, _ = env.reset(seed=0)
    assert set(o) == {"rgb"}
    assert o["rgb"].shape == env.observation_space["rgb"].shape == (2, 3, 32, 32)


def test_mask_velocities_requires_known_env():
    from sheeprl_prey_amd.envs.registry import make
    from sheeprl_prey_amd.envs.wrappers import MaskVelocityWrapper

    from sheeprl_prey_amd.envs.dummy import ContinuousDummyEnv

    w = MaskVelocityWrapper(make("CartPole-v1"))
    o, _ = w.reset(seed=0)
    o, *_ = w.step(0)
    assert o[1] == 0 and o[3] == 0
    with pytest.raises(NotImplementedError):
        MaskVelocityWrapper(ContinuousDummyEnv(size=(4,)))


def test_gemm_tuning_modes_cpu():
    """parallel/gemm_tuning: YAML booleans map to modes; without a GPU nothing is enabled; the
    committed MI355X TunableOp results file exists and carries its validators."""
    import os

    from sheeprl_prey_amd.parallel import gemm_tuning

    assert gemm_tuning.configure(False) is False
    assert gemm_tuning.configure("off") is False
    assert gemm_tuning.configure("use") is False  # no GPU in the CPU suite
    assert os.path.exists(gemm_tuning.RESULTS)
    head = open(gemm_tuning.RESULTS).read().splitlines()[:5]
    assert any(line.startswith("Validator,GCN_ARCH_NAME,gfx950") for line in head)


def test_bf16_mixed_setup_module_hooks():
    """bf16-mixed runs the set-up module's forward under autocast, returns fp32, keeps fp32 grads,
    and a deep copy (target network) keeps using its own weights."""
    import copy

    from sheeprl_prey_amd.parallel.runner import Runner

    r = Runner(accelerator="cpu", precision="bf16-mixed")
    torch.manual_seed(0)
    m = r.setup_module(torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.Tanh(), torch.nn.Linear(16, 3)))
    x = torch.randn(5, 8)
    y = m(x)
    assert y.dtype == torch.float32
    with torch.autocast("cpu", dtype=torch.bfloat16):
        want = m[2](m[1](m[0](x))).float()
    torch.testing.assert_close(y, want)
    y.sum().backward()
    assert m[0].weight.grad.dtype == torch.float32
    c = copy.deepcopy(m)
    with torch.no_grad():
        m[0].weight.zero_()
    torch.testing.assert_close(c(x), y.detach())
    with pytest.raises(ValueError):
        Runner(precision="64-true")


def test_optimizer_fault_guard_skips_update_eager():
    """The fault-block contract of the flat optimiser kernels (``ops/csrc/optim.hip``), on the eager oracle:
    with word 0 (scan health) or 1 (gather error) set, norm/advance flag the step as skipped, count it in word 2
    and Adam leaves the parameters, moments and step count untouched; a clean block updates as usual."""
    from sheeprl_prey_amd import ops

    torch.manual_seed(0)
    p, g = torch.randn(16), torch.randn(16)
    m, v = torch.zeros(16), torch.zeros(16)
    scalars = torch.tensor([0.0, 1.0, 0.0, 0.0])
    guard = torch.zeros(4, dtype=torch.int32)
    for word in (0, 1):
        guard[word] = 4
        p0 = p.clone()
        ops.flat_grad_norm(g, scalars, 1.0, guard)
        ops.flat_adam(p, g, m, v, scalars, 1e-2, 0.9, 0.999, 1e-8, 0.0, False)
        assert torch.equal(p, p0) and float(scalars[0]) == 0.0 and float(scalars[3]) == 1.0
        ops.flat_advance(scalars, guard)
        assert float(scalars[0]) == 0.0
        guard[word] = 0
    assert int(guard[2]) == 4
    ops.flat_grad_norm(g, scalars, 1.0, guard)
    ops.flat_adam(p, g, m, v, scalars, 1e-2, 0.9, 0.999, 1e-8, 0.0, False)
    assert float(scalars[0]) == 1.0 and float(scalars[3]) == 0.0 and not torch.equal(p, p0)
    assert int(guard[2]) == 4


def test_runner_fused_ops_knob_routes_ops():
    """``fabric.fused_ops`` is wired: a Runner built with it off routes the ops through the eager oracles."""
    from sheeprl_prey_amd import ops
    from sheeprl_prey_amd.parallel.runner import Runner

    try:
        Runner(accelerator="cpu", fused_ops=False)
        assert not ops.fused_enabled()
        Runner(accelerator="cpu", fused_ops=True)
        assert ops.fused_enabled()
    finally:
        ops.set_fused(True)


def test_collective_log_records_and_counts_per_phase():
    """``CollectiveLog`` wraps the torch.distributed entry points: (step, phase, op, numel, dtype) per call."""
    import torch.distributed as dist

    from sheeprl_prey_amd.parallel.collectives import CollectiveLog, set_phase, step_boundary

    calls = []
    orig = dist.all_reduce
    with CollectiveLog() as log:
        assert dist.all_reduce is not orig and dist.all_reduce.__wrapped__ is orig
        step_boundary()
        set_phase("wm")
        # wrappers around stand-ins: no process group needed
        wrapped = log._wrap("all_reduce", lambda t, **kw: calls.append(t.numel()))
        wrapped(torch.zeros(7))
        wrapped(torch.zeros(3))
        set_phase("coll_lambda")
        log._wrap("all_gather_into_tensor", lambda o, t, **kw: None)(torch.zeros(4), torch.zeros(2))
    assert dist.all_reduce is orig
    assert calls == [7, 3]
    assert log.sequence(1) == [("wm", "all_reduce", 7, "float32"), ("wm", "all_reduce", 3, "float32"),
                               ("coll_lambda", "all_gather_into_tensor", 4, "float32")]
    assert log.per_phase(1) == {"wm": {"all_reduce": 2}, "coll_lambda": {"all_gather_into_tensor": 1}}
    set_phase("-")


def test_heartbeat_ends_a_stalled_process():
    """``Heartbeat``: a process whose main loop stops beating exits with status 3 (a rank stuck in a device wait
    never returns to Python, so the daemon thread ends it); one that keeps beating is left alone."""
    import subprocess
    import sys

    code = ("import time, sys; sys.path.insert(0, {root!r});"
            "from sheeprl_prey_amd.parallel.collectives import Heartbeat;"
            "h = Heartbeat(1.0, 'probe');"
            "[(h.beat('ok'), time.sleep(0.2)) for _ in range({n})];"
            "time.sleep({idle}); print('survived')")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    stalled = subprocess.run([sys.executable, "-c", code.format(root=root, n=2, idle=10)], capture_output=True, text=True,
                             timeout=60)
    assert stalled.returncode == 3 and "heartbeat: no progress" in stalled.stderr and "survived" not in stalled.stdout
    alive = subprocess.run([sys.executable, "-c", code.format(root=root, n=10, idle=0)], capture_output=True, text=True,
                           timeout=60)
    assert alive.returncode == 0 and "survived" in alive.stdout


def test_imag_discount_skip_first_matches_full_rows():
    """``ops.imag_discount(..., skip_first=True)`` on the continue logits of rows 1.. equals the full-row form
    (row 0 of the continue head is replaced by ``1 - done``, reference ``dreamer_v3.py:267-268``)."""
    from sheeprl_prey_amd import ops

    torch.manual_seed(0)
    logits = torch.randn(6, 10, 1)
    dones = (torch.rand(10) < 0.3).float()
    cg, disc = ops.imag_discount(logits, dones, 0.99)
    cg1, disc1 = ops.imag_discount(logits[1:], dones, 0.99, skip_first=True)
    assert torch.equal(cg, cg1) and torch.equal(disc, disc1)


def test_built_extension_links():
    """The in-tree HIP extension, when built, imports on the CPU host too (every launcher the bindings declare is
    defined: an undefined symbol otherwise surfaces only on the GPU box)."""
    import glob
    import importlib
    import os

    import sheeprl_prey_amd

    root = os.path.dirname(sheeprl_prey_amd.__file__)
    if not glob.glob(os.path.join(root, "ops", "_C*.so")):
        pytest.skip("extension not built")
    m = importlib.import_module("sheeprl_prey_amd.ops._C")
    for name in ("prior_head", "actor_tail", "conv_up_small", "set_up_last_form", "flat_grad_norm"):
        assert hasattr(m, name), name


def test_sidestream_scope_is_inert_on_cpu_and_outside_scopes():
    """ops/sidestream.py: on CPU tensors and outside a scope ``param_grads`` runs its function in line and returns
    its gradients, nothing is queued or left to join; the scope counter nests and unwinds on exceptions."""
    import torch

    from sheeprl_prey_amd.ops import sidestream as ss

    x = torch.ones(3)
    p = torch.nn.Parameter(torch.zeros(3))
    (g,) = ss.param_grads(x.device, lambda: (x * 2,), [p], x)
    assert torch.equal(g, torch.full((3,), 2.0)) and not ss._pending and not ss._queue
    with ss.scope():
        (g,) = ss.param_grads(x.device, lambda: (x * 3,), [p], x)  # CPU inside a scope: still in line
    assert torch.equal(g, torch.full((3,), 3.0)) and not ss._queue and p.grad is None
    ss.join()
    assert not ss.active(torch.device("cpu"))
    with ss.scope():
        with ss.scope():
            assert ss._depth == 2
            assert not ss.active(torch.device("cpu"))  # CPU: never a side stream
        try:
            with ss.scope():
                raise RuntimeError("boom")
        except RuntimeError:
            pass
        assert ss._depth == 1
    assert ss._depth == 0


def test_imagination_merge_policy():
    """SRL_IMAG_MERGE policy: "auto" merges the h_{t+1} GEMMs for recurrent states <= 1024 only (XL measured slower
    merged), "1" / "0" force it."""
    from sheeprl_prey_amd.algos.dreamer_v3.agent import RSSM

    assert RSSM.merge_enabled("auto", 512) and RSSM.merge_enabled("auto", 1024)
    assert not RSSM.merge_enabled("auto", 4096)
    assert RSSM.merge_enabled("1", 4096) and not RSSM.merge_enabled("0", 256)
    assert RSSM.merge_enabled(True, 4096) and not RSSM.merge_enabled(False, 256)


def test_reduce_workspace_is_gpu_only():
    """The one-launch column-sum workspace is a GPU-process setup: a no-op (False) for CPU devices."""
    from sheeprl_prey_amd import ops

    assert ops.init_reduce_workspace("cpu") is False


def test_heartbeat_startup_grace_scales_with_the_step_timeout():
    """The start-up grace defaults to a multiple of the step timeout (a short step timeout keeps a short start-up
    limit); an explicit grace wins."""
    from sheeprl_prey_amd.parallel.collectives import Heartbeat

    h = Heartbeat(0.0)  # disabled: no thread, the limits are still computed
    assert h.startup_grace_s == 0.0
    h = Heartbeat(30.0)
    try:
        assert h.startup_grace_s == 120.0
    finally:
        h.stop()
    h = Heartbeat(30.0, startup_grace_s=10.0)
    try:
        assert h.startup_grace_s == 10.0
    finally:
        h.stop()


def test_phased_step_eager_replay_api():
    """On the CPU a PhasedStep runs eagerly: no captured inputs to draw into, replay() is a no-op, the phases and
    collectives run in order."""
    from sheeprl_prey_amd.parallel.graphs import PhasedStep, quiesce_for_capture

    class R:
        device = torch.device("cpu")
        world_size = 1

    order = []
    ps = PhasedStep(R(), [lambda d: order.append("a"), lambda d: order.append("b") or {"x": d["x"] + 1}],
                    [lambda dry=False: order.append("c")])
    assert ps.mode == "eager" and not ps.enabled
    assert ps.captured_inputs() is None and ps.replay() is None
    out = ps({"x": torch.zeros(2)})
    assert order == ["a", "c", "b"] and torch.equal(out["x"], torch.ones(2))
    quiesce_for_capture()  # no device, no process group: returns at once
