"""Data-parallel equivalence of the GRAPHED multi-rank update (GPU): 2 ranks sharing one GPU over gloo
(RCCL refuses two ranks on one device; ``SRL_DIST_BACKEND=gloo`` keeps the GPU tensors) run the PPO
update as ``SegmentedPPOUpdate`` - per-minibatch hipGraph replays with the flat-slab gradient
all-reduce between them - on their halves of a rollout; the replicas must stay identical and equal a
single-process eager update over the whole rollout (the DDP guarantee of the reference,
``ppo/ppo.py:41-52``).  One minibatch per update makes the result independent of the row order."""
from __future__ import annotations

import os

import pytest
import torch

pytestmark = pytest.mark.gpu

N_PER_RANK = 64
UPDATES = 4  # two warm-up updates (eager), capture on the third, replay on the fourth


def _cfg(batch: int, graphs: bool):
    from sheeprl_prey_amd.config.compose import compose
    from sheeprl_prey_amd.utils.utils import dotdict

    cfg = dotdict(compose(["exp=ppo", "mlp_keys.encoder=[state]", "fabric.accelerator=cuda", f"fabric.cuda_graphs={graphs}",
                           "algo.update_epochs=1", f"per_rank_batch_size={batch}", "algo.normalize_advantages=False",
                           "algo.anneal_lr=False", "buffer.share_data=False"]))
    cfg.pop("hydra", None)
    return cfg


def _agent(cfg, device):
    from sheeprl_prey_amd.algos.ppo.agent import PPOAgent
    from sheeprl_prey_amd.envs import spaces

    torch.manual_seed(0)
    obs_space = spaces.Dict({"state": spaces.Box(-1.0, 1.0, (4,), "float32")})
    return PPOAgent([2], obs_space, cfg.algo.encoder, cfg.algo.actor, cfg.algo.critic, [], ["state"], 64, cfg.distribution,
                    False).to(device)


def _data(device):
    g = torch.Generator().manual_seed(11)
    n = 2 * N_PER_RANK
    d = {
        "state": torch.randn(UPDATES, n, 4, generator=g),
        "actions": torch.nn.functional.one_hot(torch.randint(0, 2, (UPDATES, n), generator=g), 2).float(),
        "logprobs": -torch.rand(UPDATES, n, 1, generator=g) - 0.3,
        "values": torch.randn(UPDATES, n, 1, generator=g),
        "returns": torch.randn(UPDATES, n, 1, generator=g),
        "advantages": torch.randn(UPDATES, n, 1, generator=g),
        "rewards": torch.ones(UPDATES, n, 1),
        "dones": torch.zeros(UPDATES, n, 1),
    }
    return {k: v.to(device) for k, v in d.items()}


def _run(runner, cfg, rows: slice):
    from sheeprl_prey_amd.algos.ppo.ppo import PPOTrainer
    from sheeprl_prey_amd.data.tensordict import TensorDict
    from sheeprl_prey_amd.parallel.flat_optim import build_optimizer

    dev = runner.device
    agent = _agent(cfg, dev)
    opt = build_optimizer(cfg.algo.optimizer, agent.parameters())
    data = _data(dev)
    n = rows.stop - rows.start
    tr = PPOTrainer(runner, agent, opt, cfg, n)
    for u in range(UPDATES):
        tr(TensorDict({k: v[u, rows].contiguous() for k, v in data.items()}, batch_size=[n]), None)
    torch.cuda.synchronize()
    return tr, opt.flat_param.detach().cpu().clone()


def _rank_fn(runner, out_dir: str) -> None:
    cfg = _cfg(N_PER_RANK, graphs=True)
    r = runner.global_rank
    tr, params = _run(runner, cfg, slice(r * N_PER_RANK, (r + 1) * N_PER_RANK))
    seg = tr.segmented
    torch.save({"params": params, "segmented": tr.mode == "segmented",
                "captured": seg is not None and seg.g_opt is not None and len(seg.g_fb) > 0},
               os.path.join(out_dir, f"rank{r}.pt"))


@pytest.mark.timeout(300)
def test_segmented_graph_ppo_update_two_ranks_equals_full_batch(tmp_path, monkeypatch):
    from sheeprl_prey_amd.parallel.runner import Runner

    monkeypatch.setenv("SRL_DIST_BACKEND", "gloo")
    Runner(devices=2, accelerator="cuda", cuda_graphs=True).launch(_rank_fn, str(tmp_path))
    r0 = torch.load(tmp_path / "rank0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "rank1.pt", weights_only=True)
    assert r0["segmented"] and r1["segmented"]
    assert r0["captured"] and r1["captured"], "the update must run as graph replays after warm-up"
    assert torch.equal(r0["params"], r1["params"]), "replicas diverged"

    monkeypatch.delenv("SRL_DIST_BACKEND")
    cfg = _cfg(2 * N_PER_RANK, graphs=False)
    cfg.algo.fused_update = False  # the eager per-minibatch reference, not the one-launch kernel
    runner = Runner(devices=1, accelerator="cuda", cuda_graphs=False)
    torch.cuda.set_device(runner.device)
    tr, full = _run(runner, cfg, slice(0, 2 * N_PER_RANK))
    assert tr.mode == "eager"
    torch.testing.assert_close(r0["params"], full, rtol=1e-4, atol=1e-5)
