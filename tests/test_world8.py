"""Rehearsal at the node's real width: 8 gloo ranks on the CPU (the driver's SCALE run uses 8 GPUs).

The reference's data-parallel DreamerV3 (``sheeprl/algos/dreamer_v3/dreamer_v3.py:394`` per-rank buffer
size ``buffer.size // (num_envs * world_size)``, ``:514`` env seeds ``seed + rank * num_envs + i``, ``:540``
DDP gradient all-reduce) is exercised here at world 8 with tiny dims:

* the collective sequence of three DV3 steps is identical on all 8 ranks and the replicas stay bit-identical
  (``tests/test_collective_sequence.py`` at 2-3 ranks, same rank function);
* every rank seeds its envs ``seed + rank * num_envs + i`` (distinct across the 8 x num_envs envs);
* the 8-rank DV3 CLI run checkpoints one replay buffer per rank, each ``size // (num_envs * 8)`` long.
"""
from __future__ import annotations

import json
import os

import pytest
import torch

from sheeprl_prey_amd.parallel.runner import Runner
from tests.test_collective_sequence import STEPS, _dv3_rank_fn

WORLD = 8


@pytest.mark.timeout(600)
def test_dv3_collective_sequence_world8(tmp_path):
    Runner(devices=WORLD, accelerator="cpu", bucket_mb=0.01).launch(_dv3_rank_fn, (str(tmp_path), False))
    seqs = [[tuple(x) for x in rs] for rs in json.loads((tmp_path / "seqs0.json").read_text())]
    assert len(seqs) == WORLD
    for r in range(1, WORLD):
        assert seqs[r] == seqs[0], f"rank {r} issued a different collective sequence than rank 0"
    steps = {s for s, *_ in seqs[0]}
    assert steps == set(range(1, STEPS + 1))
    ranks = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(WORLD)]
    for r in range(1, WORLD):
        assert torch.equal(ranks[r]["params"], ranks[0]["params"]), f"replica {r} diverged"


def _seed_rank_fn(runner: Runner, args) -> None:
    out_dir, num_envs = args
    import torch.distributed as dist

    from sheeprl_prey_amd.algos import common
    from sheeprl_prey_amd.config.compose import compose
    from sheeprl_prey_amd.utils.utils import dotdict

    cfg = dotdict(compose(["exp=dreamer_v3", "env=dummy", "env.id=discrete_dummy", f"env.num_envs={num_envs}",
                           "env.sync_env=True", "env.capture_video=False", "seed=42"]))
    seen = []
    orig = common.make_env

    def spy(cfg_, seed, *a, **k):
        seen.append(int(seed))
        return orig(cfg_, seed, *a, **k)

    common.make_env = spy
    try:
        envs = common.build_envs(runner, cfg, None)
        envs.close()
    finally:
        common.make_env = orig
    allseen = [None] * runner.world_size
    dist.all_gather_object(allseen, seen)
    if runner.global_rank == 0:
        with open(os.path.join(out_dir, "seeds.json"), "w") as f:
            json.dump(allseen, f)


@pytest.mark.timeout(300)
def test_env_seeds_world8(tmp_path):
    num_envs = 2
    Runner(devices=WORLD, accelerator="cpu").launch(_seed_rank_fn, (str(tmp_path), num_envs))
    seeds = json.loads((tmp_path / "seeds.json").read_text())
    assert seeds == [[42 + r * num_envs + i for i in range(num_envs)] for r in range(WORLD)]
    flat = [s for rs in seeds for s in rs]
    assert len(set(flat)) == WORLD * num_envs


@pytest.mark.timeout(600)
def test_dreamer_v3_cli_world8_buffers(tmp_path, monkeypatch):
    from tests.test_algos import DV3_KEYS, STD, TINY_DREAMER, _check_ckpt, _run

    monkeypatch.chdir(tmp_path)
    size = 16
    _run(STD + ["exp=dreamer_v3", "env=dummy", "env.id=discrete_dummy", f"buffer.size={size}", "root_dir=dv3w8",
                "run_name=w8", "buffer.checkpoint=True"] + TINY_DREAMER, WORLD)
    st = _check_ckpt("dv3w8", "w8", DV3_KEYS, True)
    assert isinstance(st["rb"], list) and len(st["rb"]) == WORLD
    for r, sd in enumerate(st["rb"]):
        assert sd["buffer_size"] == size // (1 * WORLD), (r, sd["buffer_size"])
    assert st["update"] % WORLD == 0
