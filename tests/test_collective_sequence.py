"""Every rank issues the same collectives in the same order (CPU, gloo, 2 and 3 ranks).

A data-parallel DreamerV3 step has three kinds of collectives: the gradient buckets of the three flat
slabs (world model / actor / critic; from the second step on they launch from post-accumulate-grad
hooks while the backward runs), the lambda all-gather of ``Moments`` (reference
``dreamer_v3/utils.py:35``) and - on the graphed single-step path - an actor all-reduce left in flight
across the critic phase.  If two ranks issued them in different orders or sizes the RCCL step would
deadlock.  ``CollectiveLog`` records ``(phase, op, numel, dtype)`` of every call on every rank over
three steps; the test asserts the sequences are identical across ranks, that every phase issued what
it must, and that the replicas stay bit-identical (reference DDP semantics,
``dreamer_v3/agent.py:1054-1063``)."""
from __future__ import annotations

import json
import os

import pytest
import torch

from sheeprl_prey_amd.parallel.runner import Runner

STEPS = 3
T, B = 6, 2


def _dv3_rank_fn(runner: Runner, args) -> None:
    out_dir, continuous = args
    import torch.distributed as dist

    from sheeprl_prey_amd.algos.dreamer_v3.agent import build_models
    from sheeprl_prey_amd.algos.dreamer_v3.dreamer_v3 import DreamerV3Trainer
    from sheeprl_prey_amd.algos.dreamer_v3.utils import Moments
    from sheeprl_prey_amd.config.compose import compose
    from sheeprl_prey_amd.envs import spaces
    from sheeprl_prey_amd.parallel.collectives import CollectiveLog
    from sheeprl_prey_amd.parallel.flat_optim import build_optimizer
    from sheeprl_prey_amd.utils.utils import dotdict

    rank = runner.global_rank
    cfg = dotdict(compose([
        "exp=dreamer_v3", "env=dummy", "mlp_keys.encoder=[state]", "mlp_keys.decoder=[state]", "algo.dense_units=16",
        "algo.mlp_layers=1", "algo.world_model.recurrent_model.recurrent_state_size=16",
        "algo.world_model.representation_model.hidden_size=16", "algo.world_model.transition_model.hidden_size=16",
        "algo.world_model.stochastic_size=4", "algo.world_model.discrete_size=4", "algo.horizon=3",
        # tiny buckets: each slab's all-reduce is cut into several hook-launched collectives
        "fabric.bucket_mb=0.01",
    ]))
    obs_space = spaces.Dict({"state": spaces.Box(-1, 1, (5,), "float32")})
    actions_dim = [2] if continuous else [3]
    torch.manual_seed(0)
    wm, actor, critic, target = build_models(runner, actions_dim, continuous, cfg, obs_space)
    wopt = build_optimizer(cfg.algo.world_model.optimizer, wm.parameters())
    aopt = build_optimizer(cfg.algo.actor.optimizer, actor.parameters())
    copt = build_optimizer(cfg.algo.critic.optimizer, critic.parameters())
    moments = Moments(runner)
    trainer = DreamerV3Trainer(runner, cfg, wm, actor, critic, target, wopt, aopt, copt, moments, continuous,
                               actions_dim)
    g = torch.Generator().manual_seed(100 + rank)  # every rank trains on its own data
    with CollectiveLog() as log:
        for _ in range(STEPS):
            if continuous:
                act = torch.rand(T, B, 2, generator=g) * 2 - 1
            else:
                act = torch.nn.functional.one_hot(torch.randint(0, 3, (T, B), generator=g), 3).float()
            data = {"state": torch.randn(T, B, 5, generator=g), "actions": act,
                    "rewards": torch.randn(T, B, 1, generator=g), "dones": torch.zeros(T, B, 1),
                    "is_first": torch.zeros(T, B, 1)}
            trainer.update_target(0.02)
            trainer.train_step(data)
    seqs = [None] * runner.world_size
    dist.all_gather_object(seqs, log.records)
    params = torch.cat([o.flat_param for o in (wopt, aopt, copt)])
    torch.save({"params": params}, os.path.join(out_dir, f"rank{rank}.pt"))
    with open(os.path.join(out_dir, f"seqs{rank}.json"), "w") as f:
        json.dump(seqs, f)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("continuous", [False, True])
def test_dv3_collective_sequence_identical_across_ranks(tmp_path, world, continuous):
    Runner(devices=world, accelerator="cpu", bucket_mb=0.01).launch(_dv3_rank_fn, (str(tmp_path), continuous))
    ranks = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(world)]
    seqs = [[tuple(x) for x in rs] for rs in json.loads((tmp_path / "seqs0.json").read_text())]
    assert len(seqs) == world
    for r in range(1, world):
        assert seqs[r] == seqs[0], f"rank {r} issued a different collective sequence than rank 0"
    per_step = {}
    for step, phase, op, numel, _ in seqs[0]:
        per_step.setdefault(step, []).append((phase, op, numel))
    assert sorted(per_step) == list(range(1, STEPS + 1))
    order = {"wm": 0, "coll_wm": 0, "imagine": 1, "coll_lambda": 1, "actor": 2, "coll_actor": 2, "critic": 3,
             "coll_critic": 3, "final": 4}
    for step, recs in per_step.items():
        groups = [order[p] for p, _, _ in recs]
        # world-model buckets, then the lambda all-gather, then the actor's, then the critic's buckets
        assert groups == sorted(groups), recs
        assert set(groups) == {0, 1, 2, 3}, recs
        assert [op for p, op, _ in recs if order[p] == 1] == ["all_gather"], recs
        assert sum(1 for p, op, _ in recs if order[p] == 0 and op == "all_reduce") >= 2, recs
    # from the second step on the world-model buckets launch inside the backward (hooks), not after it
    assert any(p == "wm" and op == "all_reduce" for p, op, _ in per_step[2]), per_step[2]
    # data parallelism keeps the replicas bit-identical
    for r in range(1, world):
        assert torch.equal(ranks[r]["params"], ranks[0]["params"])
