"""The same CLI dry runs as ``test_algos.py`` on one MI355X (fused HIP ops, hipGraph-captured updates)."""
from __future__ import annotations

import os
from unittest import mock

import pytest

from sheeprl_prey_amd.cli import run
from tests.test_algos import DV3_KEYS, PPO_KEYS, SAC_KEYS, STD, TINY_DREAMER, _check_ckpt

pytestmark = pytest.mark.gpu

GPU = ["fabric.accelerator=cuda", "fabric.cuda_graphs=True"]


def _run(args):
    with mock.patch.dict(os.environ, {"LT_ACCELERATOR": "cuda", "LT_DEVICES": "1"}, clear=False):
        run(list(args) + GPU)


def test_sac_gpu():
    _run(STD + ["exp=sac", "env=dummy", "env.id=continuous_dummy_vec", "per_rank_batch_size=4", "buffer.size=8",
                "algo.learning_starts=0", "algo.per_rank_gradient_steps=4", "root_dir=sac", "run_name=g",
                "buffer.checkpoint=True"])
    _check_ckpt("sac", "g", SAC_KEYS, True)


def test_sac_gpu_graphed_player_pendulum():
    """A short non-dry SAC run on the native Pendulum: random-action steps, then the hipGraph-replayed
    player and the single pinned row copy per env step (sac.py gpu_row path), several logs."""
    _run(["env.num_envs=2", "env.sync_env=True", "env.capture_video=False", "exp=sac", "env=gym",
          "env.id=Pendulum-v1", "total_steps=400", "algo.learning_starts=100", "per_rank_batch_size=32",
          "metric.log_every=100", "checkpoint.every=0", "root_dir=sac_pend", "run_name=g"])
    _check_ckpt("sac_pend", "g", SAC_KEYS, False)


def test_droq_gpu():
    _run(STD + ["exp=droq", "env=dummy", "env.id=continuous_dummy_vec", "per_rank_batch_size=4", "buffer.size=8",
                "algo.learning_starts=0", "algo.per_rank_gradient_steps=4", "root_dir=droq", "run_name=g",
                "buffer.checkpoint=True"])
    _check_ckpt("droq", "g", SAC_KEYS, True)


def test_sac_ae_gpu():
    _run(STD + ["exp=sac_ae", "env.id=Pendulum-v1", "per_rank_batch_size=2", "buffer.size=4",
                "algo.learning_starts=0", "algo.per_rank_gradient_steps=4", "root_dir=sac_ae", "run_name=g",
                "mlp_keys.encoder=[state]", "cnn_keys.encoder=[rgb]", "env.screen_size=64", "algo.hidden_size=16",
                "algo.dense_units=16", "algo.cnn_channels_multiplier=2", "algo.actor.network_frequency=1",
                "algo.decoder.update_freq=1", "buffer.checkpoint=True"])
    _check_ckpt("sac_ae", "g", SAC_KEYS | {"encoder", "decoder", "encoder_optimizer", "decoder_optimizer"}, True)


@pytest.mark.parametrize("env_id", ["discrete_dummy", "continuous_dummy"])
def test_ppo_gpu(env_id):
    _run(STD + ["exp=ppo", "env=dummy", f"env.id={env_id}", "algo.rollout_steps=4", "per_rank_batch_size=2",
                "root_dir=ppo", f"run_name={env_id}"])
    _check_ckpt("ppo", env_id, PPO_KEYS, False)


@pytest.mark.parametrize("fused", [True, False])
def test_ppo_device_env_gpu(fused):
    """env.device=True: CartPole on the GPU, one-launch rollout (or the graph-captured per-op one
    when the agent is outside the fused kernels: LayerNorm MLPs) and the fused update."""
    extra = [] if fused else ["algo.layer_norm=True"]
    _run(STD + ["exp=ppo", "env.id=CartPole-v1", "env.device=True", "mlp_keys.encoder=[state]",
                "algo.rollout_steps=16", "per_rank_batch_size=8", "env.num_envs=3", "root_dir=ppo_dev",
                f"run_name=f{int(fused)}"] + extra)
    _check_ckpt("ppo_dev", f"f{int(fused)}", PPO_KEYS, False)


@pytest.mark.parametrize("env_id", ["discrete_dummy", "multidiscrete_dummy", "continuous_dummy"])
def test_dreamer_v3_gpu(env_id):
    _run(STD + ["exp=dreamer_v3", "env=dummy", f"env.id={env_id}", "buffer.size=4", "root_dir=dv3",
                f"run_name={env_id}", "buffer.checkpoint=True"] + TINY_DREAMER)
    _check_ckpt("dv3", env_id, DV3_KEYS, True)


from tests.test_algos import DV1_KEYS, DV2_KEYS, DV2_EXTRA, P2E1_KEYS, P2E2_KEYS, SMALL_WM  # noqa: E402

# short real runs (not dry runs): the replay must hold a full sequence before the first update
SHORT = ["dry_run=False", "env.num_envs=1", "env.sync_env=True", "env.capture_video=False", "per_rank_batch_size=4",
         "per_rank_sequence_length=4", "buffer.size=64", "algo.horizon=4", "total_steps=12", "algo.train_every=1",
         "checkpoint.every=0", "metric.log_every=1", "algo.per_rank_pretrain_steps=2", "buffer.checkpoint=True"]
WM_GPU = [a for a in SMALL_WM if not a.startswith("algo.learning_starts")] + ["algo.learning_starts=6"]


def test_dreamer_v1_gpu():
    _run(SHORT + ["exp=dreamer_v1", "env=dummy", "env.id=continuous_dummy", "root_dir=dv1", "run_name=g"] + WM_GPU)
    _check_ckpt("dv1", "g", DV1_KEYS, True)


@pytest.mark.parametrize("env_id", ["discrete_dummy", "continuous_dummy"])
def test_dreamer_v2_gpu(env_id):
    _run(SHORT + ["exp=dreamer_v2", "env=dummy", f"env.id={env_id}", "root_dir=dv2", f"run_name={env_id}"]
         + WM_GPU + DV2_EXTRA)
    _check_ckpt("dv2", env_id, DV2_KEYS, True)


@pytest.mark.parametrize("algo", ["p2e_dv1", "p2e_dv2"])
def test_p2e_gpu_explore_phases(algo):
    """Exploration (7-phase captured step) until update 9, then the task step."""
    import json
    from pathlib import Path

    extra = DV2_EXTRA if algo == "p2e_dv2" else []
    _run(SHORT + [f"exp={algo}", "env=dummy", "env.id=discrete_dummy", "exploration_steps=9", "algo.ensembles.n=4",
                  "root_dir=p2e_g", f"run_name={algo}"] + WM_GPU + extra)
    rows = [json.loads(l) for l in open(next(Path("logs", "runs", "p2e_g", algo).rglob("metrics.jsonl")))]
    keys = set().union(*[r.keys() for r in rows])
    assert {"Loss/ensemble_loss", "Loss/policy_loss_exploration", "Loss/policy_loss_task"} <= keys


def test_dreamer_v3_continuous_graph_capture():
    """Continuous DV3 (truncated-normal actor, differentiable imagination) through a captured hipGraph."""
    _run(SHORT + ["exp=dreamer_v3", "env=dummy", "env.id=continuous_dummy", "root_dir=dv3c", "run_name=g",
                  "algo.dense_units=8", "algo.world_model.encoder.cnn_channels_multiplier=2",
                  "algo.world_model.recurrent_model.recurrent_state_size=8",
                  "algo.world_model.representation_model.hidden_size=8",
                  "algo.world_model.transition_model.hidden_size=8", "cnn_keys.encoder=[rgb]", "cnn_keys.decoder=[rgb]",
                  "algo.learning_starts=6", "algo.per_rank_gradient_steps=1"])
    from tests.test_algos import DV3_KEYS

    _check_ckpt("dv3c", "g", DV3_KEYS, True)


@pytest.mark.parametrize("algo", ["ppo", "dreamer_v3"])
def test_bf16_mixed_gpu(algo):
    """``fabric.precision=bf16-mixed`` on the GPU: autocast forwards (fused fp32 kernels step aside),
    hipGraph capture of the train step, checkpoint written."""
    from tests.test_algos import record_autocast

    with record_autocast() as seen:
        if algo == "ppo":
            _run(STD + ["exp=ppo", "env=dummy", "env.id=discrete_dummy", "algo.rollout_steps=4", "per_rank_batch_size=2",
                        "fabric.precision=bf16-mixed", "root_dir=ppo_bf16", "run_name=g"])
            _check_ckpt("ppo_bf16", "g", PPO_KEYS, False)
        else:
            _run(STD + ["exp=dreamer_v3", "env=dummy", "env.id=discrete_dummy", "buffer.size=4", "root_dir=dv3_bf16",
                        "run_name=g", "fabric.precision=bf16-mixed"] + TINY_DREAMER)
            _check_ckpt("dv3_bf16", "g", DV3_KEYS, False)
    # every sub-model the step calls ran its forward under autocast (the world model has no forward of its own)
    want = {"PPOAgent"} if algo == "ppo" else {"MultiEncoder", "RecurrentModel", "MLP", "MultiDecoder", "Actor"}
    assert want <= set(seen), f"forwards run under autocast: {dict(seen)}"


def test_dreamer_v3_prey_preset_gpu():
    """The fork's own preset (exp=dreamer_v3_prey) on the native prey_d_1 cellworld through the CLI on the GPU:
    vector observations, the Discrete(100) actor on the wide-categorical unimix kernels, captured train steps.
    Scaled down (dense 256, 16-step sequences: the persistent scan); the preset's dense 1024 runs the 4-launch scan,
    whose shape tests/test_dreamer_gpu.py covers."""
    _run(["exp=dreamer_v3_prey", "env.sync_env=True", "env.capture_video=False", "total_steps=260",
          "algo.learning_starts=200", "per_rank_sequence_length=16", "per_rank_batch_size=4", "algo.dense_units=256",
          "metric.log_every=100", "checkpoint.every=0", "root_dir=dv3prey", "run_name=g"])
    _check_ckpt("dv3prey", "g", DV3_KEYS, False)


def test_ppo_prey_gpu():
    """PPO on prey_d_1 (Discrete(100)) through the CLI on the GPU path."""
    _run(["exp=ppo", "env=prey", "mlp_keys.encoder=[state]", "env.num_envs=2", "env.sync_env=True",
          "env.capture_video=False", "total_steps=512", "algo.rollout_steps=128", "per_rank_batch_size=64",
          "metric.log_every=256", "checkpoint.every=0", "root_dir=ppoprey", "run_name=g"])
    _check_ckpt("ppoprey", "g", PPO_KEYS, False)
