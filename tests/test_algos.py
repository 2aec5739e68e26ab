"""End-to-end algorithm tests (CPU, gloo) - the reference's ``tests/test_algos/test_algos.py``
strategy: run the real CLI in-process with ``dry_run=True`` and tiny models, then check the
checkpoint key set and the saved ``.hydra/config.yaml``.  ``devices=2`` runs two gloo ranks
(spawned processes) exercising the gradient all-reduce / all-gather / decoupled paths.
"""
from __future__ import annotations

import collections
import contextlib
import os
from pathlib import Path
from unittest import mock

import pytest
import torch

from sheeprl_prey_amd.cli import run

STD = [
    "dry_run=True",
    "env.num_envs=1",
    "env.sync_env=True",
    "env.capture_video=False",
]


def _run(args, devices: int):
    with mock.patch.dict(os.environ, {"LT_ACCELERATOR": "cpu", "LT_DEVICES": str(devices)}, clear=False):
        run(list(args))


def _check_ckpt(root: str, run_name: str, keys: set, rb: bool) -> dict:
    base = Path("logs", "runs", root, run_name)
    versions = sorted(base.iterdir())
    ck_dir = versions[-1] / "checkpoint"
    assert ck_dir.is_dir(), f"no checkpoint dir under {versions[-1]}"
    ckpts = sorted(ck_dir.glob("*.ckpt"))
    assert ckpts, "no checkpoint written"
    state = torch.load(ckpts[-1], map_location="cpu", weights_only=True)
    want = set(keys) | ({"rb"} if rb else set())
    assert set(state.keys()) == want, f"checkpoint keys {sorted(state)} != {sorted(want)}"
    assert (versions[-1] / ".." / ".hydra" / "config.yaml").resolve().exists() or \
        (base / ".hydra" / "config.yaml").exists()
    return state


SAC_KEYS = {"agent", "qf_optimizer", "actor_optimizer", "alpha_optimizer", "update", "last_log", "last_checkpoint",
            "batch_size"}


@pytest.mark.timeout(180)
@pytest.mark.parametrize("devices", [1, 2])
@pytest.mark.parametrize("checkpoint_buffer", [True, False])
def test_sac(devices, checkpoint_buffer):
    _run(STD + ["exp=sac", "env=dummy", "env.id=continuous_dummy_vec", "per_rank_batch_size=1",
                f"buffer.size={devices}", "algo.learning_starts=0", "algo.per_rank_gradient_steps=1",
                "algo.hidden_size=8", "root_dir=sac", f"run_name=r{devices}{int(checkpoint_buffer)}",
                f"buffer.checkpoint={checkpoint_buffer}"], devices)
    st = _check_ckpt("sac", f"r{devices}{int(checkpoint_buffer)}", SAC_KEYS, checkpoint_buffer)
    if checkpoint_buffer and devices == 2:
        assert isinstance(st["rb"], list) and len(st["rb"]) == 2


@pytest.mark.timeout(180)
@pytest.mark.parametrize("devices", [1, 2])
def test_droq(devices):
    _run(STD + ["exp=droq", "env=dummy", "env.id=continuous_dummy_vec", "per_rank_batch_size=1",
                f"buffer.size={devices}", "algo.learning_starts=0", "algo.per_rank_gradient_steps=1",
                "algo.hidden_size=8", "root_dir=droq", "run_name=r", "buffer.checkpoint=True"], devices)
    _check_ckpt("droq", "r", SAC_KEYS, True)


@pytest.mark.timeout(180)
@pytest.mark.parametrize("devices", [1, 2])
def test_sac_ae(devices):
    _run(STD + ["exp=sac_ae", "env.id=Pendulum-v1", "per_rank_batch_size=1", f"buffer.size={devices}",
                "algo.learning_starts=0", "algo.per_rank_gradient_steps=1", "root_dir=sac_ae", "run_name=r",
                "mlp_keys.encoder=[state]", "cnn_keys.encoder=[rgb]", "env.screen_size=64", "algo.hidden_size=4",
                "algo.dense_units=4", "algo.cnn_channels_multiplier=2", "algo.actor.network_frequency=1",
                "algo.decoder.update_freq=1", "buffer.checkpoint=True"], devices)
    _check_ckpt("sac_ae", "r", SAC_KEYS | {"encoder", "decoder", "encoder_optimizer", "decoder_optimizer"}, True)


@pytest.mark.timeout(180)
@pytest.mark.parametrize("devices", [2, 3])
def test_sac_decoupled(devices):
    _run(STD + ["exp=sac_decoupled", "env=dummy", "env.id=continuous_dummy_vec", "per_rank_batch_size=1",
                "algo.learning_starts=0", "algo.per_rank_gradient_steps=1", "algo.hidden_size=8",
                "root_dir=sac_dec", f"run_name=r{devices}", "buffer.checkpoint=True"], devices)
    _check_ckpt("sac_dec", f"r{devices}", SAC_KEYS, True)


PPO_KEYS = {"agent", "optimizer", "scheduler", "update", "batch_size", "last_log", "last_checkpoint"}


@pytest.mark.timeout(180)
@pytest.mark.parametrize("devices", [1, 2])
@pytest.mark.parametrize("env_id", ["discrete_dummy", "multidiscrete_dummy", "continuous_dummy"])
def test_ppo(devices, env_id):
    _run(STD + ["exp=ppo", "env=dummy", f"env.id={env_id}", f"algo.rollout_steps={devices}",
                "per_rank_batch_size=1", "root_dir=ppo", f"run_name={env_id}{devices}"], devices)
    _check_ckpt("ppo", f"{env_id}{devices}", PPO_KEYS, False)


DV3_KEYS = {"world_model", "actor", "critic", "target_critic", "world_optimizer", "actor_optimizer",
            "critic_optimizer", "expl_decay_steps", "moments", "update", "batch_size", "last_log", "last_checkpoint"}

TINY_DREAMER = [
    "per_rank_sequence_length=1", "per_rank_batch_size=1", "algo.learning_starts=0", "algo.horizon=8",
    "algo.per_rank_gradient_steps=1", "algo.dense_units=8", "algo.world_model.encoder.cnn_channels_multiplier=2",
    "algo.world_model.recurrent_model.recurrent_state_size=8", "algo.world_model.representation_model.hidden_size=8",
    "algo.world_model.transition_model.hidden_size=8", "algo.layer_norm=True", "algo.train_every=1",
    "cnn_keys.encoder=[rgb]", "cnn_keys.decoder=[rgb]",
]


@pytest.mark.timeout(240)
@pytest.mark.parametrize("devices", [1, 2])
@pytest.mark.parametrize("env_id", ["discrete_dummy", "multidiscrete_dummy", "continuous_dummy"])
def test_dreamer_v3(devices, env_id):
    _run(STD + ["exp=dreamer_v3", "env=dummy", f"env.id={env_id}", f"buffer.size={devices}", "root_dir=dv3",
                f"run_name={env_id}{devices}", "buffer.checkpoint=True"] + TINY_DREAMER, devices)
    _check_ckpt("dv3", f"{env_id}{devices}", DV3_KEYS, True)


@pytest.mark.timeout(300)
def test_resume_dreamer_v3_two_cli_runs():
    """Checkpoint -> resume through two separate ``python sheeprl.py`` processes (reference
    ``tests/test_algos/test_cli.py:39-79``): the second run restores world model, actor, critics,
    optimisers, Moments and the replay buffer, then keeps training and checkpoints again."""
    import subprocess
    import sys

    repo = Path(__file__).resolve().parents[1]
    env = dict(os.environ, LT_ACCELERATOR="cpu", LT_DEVICES="1",
               PYTHONPATH=os.pathsep.join([str(repo), os.environ.get("PYTHONPATH", "")]))
    tiny = [a for a in TINY_DREAMER if not a.startswith("per_rank_sequence_length")]
    first = [sys.executable, str(repo / "sheeprl.py"), "exp=dreamer_v3", "env=dummy", "dry_run=True", "env.capture_video=False",
             "buffer.size=10", "buffer.checkpoint=True", "per_rank_sequence_length=1", "root_dir=dv3_ckpt",
             "run_name=a"] + tiny
    subprocess.run(first, check=True, env=env, timeout=240)
    ck = sorted(Path("logs", "runs", "dv3_ckpt", "a").rglob("*.ckpt"))[-1]
    saved = torch.load(ck, map_location="cpu", weights_only=True)
    assert set(saved) == DV3_KEYS | {"rb"}
    second = [sys.executable, str(repo / "sheeprl.py"), "exp=dreamer_v3", f"checkpoint.resume_from={ck}", "root_dir=dv3_resume",
              "run_name=b"]
    subprocess.run(second, check=True, env=env, timeout=240)
    resumed = sorted(Path("logs", "runs", "dv3_resume", "b").rglob("*.ckpt"))
    assert resumed, "the resumed run wrote no checkpoint"
    state = torch.load(resumed[-1], map_location="cpu", weights_only=True)
    assert set(state) == DV3_KEYS | {"rb"}
    assert state["update"] >= saved["update"]


def test_sac_default_env_needs_box2d_message():
    """``exp=sac`` defaults to LunarLanderContinuous-v2 (reference ``configs/exp/sac.yaml:15``); Box2D is not
    in the image, so the run must stop with an actionable message instead of an unknown-id error."""
    with pytest.raises(ModuleNotFoundError, match="Box2D"):
        _run(STD + ["exp=sac"], 1)


def test_fsdp_rejected():
    with pytest.raises(ValueError, match="FSDP"):
        _run(["exp=ppo", "env=dummy", "fabric.strategy=fsdp", "dry_run=True"], 1)


def test_resume_sac(tmp_path):
    args = STD + ["exp=sac", "env=dummy", "env.id=continuous_dummy_vec", "per_rank_batch_size=1", "buffer.size=4",
                  "algo.learning_starts=0", "algo.per_rank_gradient_steps=1", "algo.hidden_size=8",
                  "root_dir=resume", "run_name=a", "buffer.checkpoint=True"]
    _run(args, 1)
    ck = sorted(Path("logs", "runs", "resume", "a").rglob("*.ckpt"))[-1]
    _run(STD + ["exp=sac", "env=dummy", "env.id=continuous_dummy_vec", f"checkpoint.resume_from={ck}",
                "root_dir=resume", "run_name=b"], 1)
    assert list(Path("logs", "runs", "resume", "b").rglob("*.ckpt"))


@pytest.mark.timeout(180)
@pytest.mark.parametrize("devices", [1, 2, 3])
@pytest.mark.parametrize("env_id", ["discrete_dummy", "continuous_dummy"])
def test_ppo_decoupled(devices, env_id):
    args = STD + ["exp=ppo_decoupled", "env=dummy", f"env.id={env_id}", f"algo.rollout_steps={devices}",
                  "per_rank_batch_size=1", "algo.update_epochs=1", "root_dir=ppo_dec", f"run_name={env_id}{devices}"]
    if devices == 1:
        with pytest.raises(RuntimeError, match="greater than 1"):
            _run(args, devices)
        return
    _run(args, devices)
    _check_ckpt("ppo_dec", f"{env_id}{devices}", PPO_KEYS, False)


@pytest.mark.timeout(240)
@pytest.mark.parametrize("devices", [2, 3])
@pytest.mark.parametrize("env_id", ["discrete_dummy", "continuous_dummy"])
def test_ppo_actor_fleet(devices, env_id):
    """N-1 actor ranks -> 1 learner over gloo: fixed-shape rollout slabs gathered on the learner, the
    weights broadcast back; the learner checkpoints with the coupled PPO key set."""
    _run(STD + ["exp=ppo_decoupled", "algo.topology=actor_fleet", "env=dummy", f"env.id={env_id}", "algo.rollout_steps=4",
                "per_rank_batch_size=4", "algo.update_epochs=1", "root_dir=ppo_fleet", f"run_name={env_id}{devices}"],
         devices)
    _check_ckpt("ppo_fleet", f"{env_id}{devices}", PPO_KEYS, False)


@pytest.mark.timeout(240)
@pytest.mark.parametrize("lag", [1, 2])
def test_ppo_actor_fleet_weight_lag(lag):
    """``algo.weight_lag``: the actors post the weight receives asynchronously and keep rolling out with weights
    up to ``lag`` updates old; over several updates the collective counts must still match (no hang) and the
    learner finishes and checkpoints."""
    n_updates = 4
    _run(["env.num_envs=1", "env.sync_env=True", "env.capture_video=False", "exp=ppo_decoupled",
          "algo.topology=actor_fleet", "env=dummy", "env.id=discrete_dummy", "algo.rollout_steps=4", "per_rank_batch_size=4",
          "algo.update_epochs=1", f"algo.weight_lag={lag}", f"total_steps={4 * 2 * n_updates}", "metric.log_every=8",
          "checkpoint.every=1000000", "root_dir=ppo_fleet_lag", f"run_name=l{lag}"], 3)
    _check_ckpt("ppo_fleet_lag", f"l{lag}", PPO_KEYS, False)


@pytest.mark.timeout(180)
@pytest.mark.parametrize("devices", [1, 2])
def test_ppo_recurrent(devices):
    _run(STD + ["exp=ppo_recurrent", "algo.rollout_steps=2", "per_rank_batch_size=1", "per_rank_sequence_length=2",
                "algo.update_epochs=2", "root_dir=ppo_rec", f"run_name=r{devices}"], devices)
    _check_ckpt("ppo_rec", f"r{devices}", PPO_KEYS, False)


def test_pad_sequence_and_masked_losses():
    from sheeprl_prey_amd.algos.ppo_recurrent.ppo_recurrent import masked_losses
    from sheeprl_prey_amd.data.tensordict import TensorDict, pad_sequence
    from sheeprl_prey_amd.utils.utils import dotdict

    a = TensorDict({"x": torch.arange(3.0).view(3, 1)}, batch_size=[3])
    b = TensorDict({"x": torch.arange(5.0).view(5, 1)}, batch_size=[5])
    p = pad_sequence([a, b])
    assert tuple(p.shape) == (5, 2) and p["mask"].sum() == 8 and p["x"][4, 0] == 0
    # masked losses == losses over the gathered valid entries
    torch.manual_seed(0)
    shape = (5, 2, 1)
    lp, olp, adv, v, ov, ret, ent = (torch.randn(shape) for _ in range(7))
    m = p["mask"].unsqueeze(-1).float()
    cfg = dotdict({"algo": {"normalize_advantages": True, "clip_coef": 0.2, "clip_vloss": True, "loss_reduction": "mean"}})
    pg, vl, el = masked_losses(lp, olp, adv, v, ov, ret, ent, m, cfg)
    sel = p["mask"].unsqueeze(-1)
    A = adv[sel]
    A = (A - A.mean()) / (A.std() + 1e-8)
    r = (lp[sel] - olp[sel]).exp()
    pg_ref = (-torch.min(A * r, A * r.clamp(0.8, 1.2))).mean()
    pred = ov[sel] + (v[sel] - ov[sel]).clamp(-0.2, 0.2)
    torch.testing.assert_close(pg, pg_ref)
    torch.testing.assert_close(vl, (pred - ret[sel]).pow(2).mean())
    torch.testing.assert_close(el, -ent[sel].mean())


DV1_KEYS = {"world_model", "actor", "critic", "world_optimizer", "actor_optimizer", "critic_optimizer",
            "expl_decay_steps", "update", "batch_size", "last_log", "last_checkpoint"}
DV2_KEYS = DV1_KEYS | {"target_critic"}
P2E1_KEYS = {"world_model", "actor_task", "critic_task", "ensembles", "world_optimizer", "actor_task_optimizer",
             "critic_task_optimizer", "ensemble_optimizer", "expl_decay_steps", "update", "batch_size",
             "actor_exploration", "critic_exploration", "actor_exploration_optimizer", "critic_exploration_optimizer",
             "last_log", "last_checkpoint"}
P2E2_KEYS = P2E1_KEYS | {"target_critic_task", "target_critic_exploration"}
SMALL_WM = ["algo.dense_units=8", "algo.world_model.encoder.cnn_channels_multiplier=2",
            "algo.world_model.recurrent_model.recurrent_state_size=8", "cnn_keys.encoder=[rgb]", "cnn_keys.decoder=[rgb]",
            "algo.learning_starts=0", "algo.per_rank_gradient_steps=1"]
DV2_EXTRA = ["algo.world_model.representation_model.hidden_size=8", "algo.world_model.transition_model.hidden_size=8"]
ENVS3 = ["discrete_dummy", "multidiscrete_dummy", "continuous_dummy"]


@pytest.mark.timeout(180)
@pytest.mark.parametrize("env_id", ENVS3)
@pytest.mark.parametrize("checkpoint_buffer", [True, False])
def test_dreamer_v1(env_id, checkpoint_buffer):
    name = f"{env_id}{int(checkpoint_buffer)}"
    _run(STD + ["exp=dreamer_v1", "env=dummy", f"env.id={env_id}", "per_rank_batch_size=1", "per_rank_sequence_length=1",
                "buffer.size=1", "algo.horizon=2", "root_dir=dv1", f"run_name={name}",
                f"buffer.checkpoint={checkpoint_buffer}"] + SMALL_WM, 1)
    _check_ckpt("dv1", name, DV1_KEYS, checkpoint_buffer)


@pytest.mark.timeout(180)
@pytest.mark.parametrize("env_id", ENVS3)
@pytest.mark.parametrize("buffer_type", ["sequential", "episode"])
def test_dreamer_v2(env_id, buffer_type):
    name = f"{env_id}{buffer_type}"
    _run(STD + ["exp=dreamer_v2", "env=dummy", f"env.id={env_id}", "per_rank_batch_size=1", "per_rank_sequence_length=1",
                "buffer.size=2", "algo.horizon=8", "root_dir=dv2", f"run_name={name}", f"buffer.type={buffer_type}",
                "buffer.checkpoint=True", "algo.world_model.use_continues=True"] + SMALL_WM + DV2_EXTRA, 1)
    _check_ckpt("dv2", name, DV2_KEYS, True)


@pytest.mark.timeout(180)
@pytest.mark.parametrize("env_id", ENVS3)
def test_p2e_dv1(env_id):
    _run(STD + ["exp=p2e_dv1", "env=dummy", f"env.id={env_id}", "per_rank_batch_size=2", "per_rank_sequence_length=2",
                "buffer.size=1", "algo.horizon=8", "root_dir=p2e1", f"run_name={env_id}", "buffer.checkpoint=True",
                "algo.ensembles.n=3"] + SMALL_WM, 1)
    _check_ckpt("p2e1", env_id, P2E1_KEYS, True)


@pytest.mark.timeout(180)
@pytest.mark.parametrize("env_id", ENVS3)
def test_p2e_dv2(env_id):
    _run(STD + ["exp=p2e_dv2", "env=dummy", f"env.id={env_id}", "per_rank_batch_size=2", "per_rank_sequence_length=2",
                "buffer.size=1", "algo.horizon=8", "root_dir=p2e2", f"run_name={env_id}", "buffer.checkpoint=True",
                "algo.ensembles.n=3"] + SMALL_WM + DV2_EXTRA, 1)
    _check_ckpt("p2e2", env_id, P2E2_KEYS, True)


@pytest.mark.timeout(240)
@pytest.mark.parametrize("algo", ["dreamer_v1", "dreamer_v2", "p2e_dv2"])
def test_dreamers_two_ranks(algo):
    extra = DV2_EXTRA if algo != "dreamer_v1" else []
    _run(STD + [f"exp={algo}", "env=dummy", "env.id=discrete_dummy", "per_rank_batch_size=1",
                "per_rank_sequence_length=1", "buffer.size=2", "algo.horizon=4", "root_dir=dr2", f"run_name={algo}",
                "buffer.checkpoint=True"] + (["algo.ensembles.n=2"] if "p2e" in algo else []) + SMALL_WM + extra, 2)
    keys = {"dreamer_v1": DV1_KEYS, "dreamer_v2": DV2_KEYS, "p2e_dv2": P2E2_KEYS}[algo]
    _check_ckpt("dr2", algo, keys, True)


@pytest.mark.timeout(240)
@pytest.mark.parametrize("algo", ["p2e_dv1", "p2e_dv2"])
@pytest.mark.parametrize("env_id", ["discrete_dummy", "continuous_dummy"])
def test_p2e_explores_then_switches(algo, env_id):
    """Not a dry run: 3 exploration updates (ensemble + exploration actor/critic phases), then the task phases."""
    extra = DV2_EXTRA if algo == "p2e_dv2" else []
    args = ["dry_run=False", "env.num_envs=1", "env.sync_env=True", "env.capture_video=False", f"exp={algo}",
            "env=dummy", f"env.id={env_id}", "per_rank_batch_size=2", "per_rank_sequence_length=2", "buffer.size=16",
            "algo.horizon=3", "total_steps=5", "exploration_steps=3", "algo.train_every=1", "checkpoint.every=0",
            "metric.log_every=1", "algo.ensembles.n=3", "root_dir=p2e_x", f"run_name={algo}{env_id}",
            "algo.per_rank_pretrain_steps=1"] + SMALL_WM + extra
    _run(args, 1)
    import json

    rows = [json.loads(l) for l in open(next(Path("logs", "runs", "p2e_x", f"{algo}{env_id}").rglob("metrics.jsonl")))]
    keys = set().union(*[r.keys() for r in rows])
    assert {"Loss/ensemble_loss", "Loss/policy_loss_exploration", "Loss/value_loss_exploration",
            "Loss/policy_loss_task", "Rewards/intrinsic"} <= keys, keys


@contextlib.contextmanager
def record_autocast():
    """Counts, per module class, the forwards that actually ran inside an enabled autocast region."""
    from sheeprl_prey_amd.parallel import runner as R

    seen = collections.Counter()
    orig = R._AutocastHooks.pre

    def pre(self, module, args):
        orig(self, module, args)
        if torch.is_autocast_enabled(self.device_type):
            seen[type(module).__name__] += 1

    with mock.patch.object(R._AutocastHooks, "pre", pre):
        yield seen


@pytest.mark.parametrize("algo", ["ppo", "sac"])
def test_bf16_mixed_precision(algo):
    """``fabric.precision=bf16-mixed`` (Fabric's mixed-precision plugin in the reference): the forwards the
    algorithm calls run under autocast (for SAC the actor and the critics, children of an agent that has
    no forward of its own) and the run trains and checkpoints as usual."""
    env = ["env=dummy", "env.id=discrete_dummy"] if algo == "ppo" else ["env.id=Pendulum-v1", "algo.learning_starts=0",
                                                                       "buffer.size=1", "algo.hidden_size=8"]
    extra = ["algo.rollout_steps=1"] if algo == "ppo" else ["algo.per_rank_gradient_steps=1"]
    with record_autocast() as seen:
        _run(STD + [f"exp={algo}", "fabric.precision=bf16-mixed", "per_rank_batch_size=1", f"root_dir={algo}_bf16",
                    "run_name=r"] + env + extra, 1)
    _check_ckpt(f"{algo}_bf16", "r", PPO_KEYS if algo == "ppo" else SAC_KEYS, False)
    want = {"PPOAgent"} if algo == "ppo" else {"SACActor", "SACCriticEnsemble"}
    assert want <= set(seen), f"forwards run under autocast: {dict(seen)}"


@pytest.mark.parametrize("alias,ok", [("bf16", True), ("32", True), ("32-true", True), ("16-mixed", False),
                                      ("64-true", False), ("bf16-true", False)])
def test_precision_aliases(alias, ok):
    from sheeprl_prey_amd.parallel.runner import _autocast_dtype

    if ok:
        assert _autocast_dtype(alias) in (None, torch.bfloat16)
        assert (_autocast_dtype(alias) is torch.bfloat16) == alias.startswith("bf16")
    else:
        with pytest.raises(ValueError, match="precision"):
            _autocast_dtype(alias)


def test_unsupported_precision_rejected():
    with pytest.raises(ValueError, match="precision"):
        _run(STD + ["exp=ppo", "env=dummy", "env.id=discrete_dummy", "fabric.precision=16-mixed"], 1)
