"""Data-parallel equivalence on CPU (2 gloo ranks): a step over per-rank halves of a batch with the
flat-slab gradient all-reduce must equal one single-process step over the whole batch - for Adam
(bucketed all-reduce: the slab is split into several collectives) and for the DreamerV3 ``Moments``
percentile EMA (all-gathered returns).  This is what DDP guarantees in the reference
(``dreamer_v3/agent.py:1054-1063`` setup_module, ``dreamer_v3/utils.py:35`` Moments all_gather);
here it pins ``FlatOptimizer.all_reduce_grads`` and ``Runner.all_gather``, the collectives the
multi-GPU bench relies on."""
from __future__ import annotations

import os

import pytest
import torch

from sheeprl_prey_amd.parallel.flat_optim import FlatAdam
from sheeprl_prey_amd.parallel.runner import Runner

STEPS = 3
BATCH = 8


def _model():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(6, 32), torch.nn.Tanh(), torch.nn.Linear(32, 32), torch.nn.Tanh(),
                               torch.nn.Linear(32, 3))


def _data():
    g = torch.Generator().manual_seed(1)
    return torch.randn(STEPS, BATCH, 6, generator=g), torch.randn(STEPS, BATCH, 3, generator=g)


def _train(model, x, y, reduce=None):
    opt = FlatAdam(model.parameters(), lr=1e-2)
    for s in range(STEPS):
        opt.zero_grad()
        torch.nn.functional.mse_loss(model(x[s]), y[s]).backward()
        if reduce is not None:
            reduce(opt)
        opt.step()
    return torch.cat([p.detach().reshape(-1) for p in model.parameters()])


def _rank_fn(runner: Runner, out_dir: str) -> None:
    from sheeprl_prey_amd.algos.dreamer_v3.utils import Moments

    rank, ws = runner.global_rank, runner.world_size
    x, y = _data()
    half = BATCH // ws
    sl = slice(rank * half, (rank + 1) * half)
    # ~1.4k parameters, 0.001 MiB buckets (262 floats): the all-reduce is split into 6 collectives
    params = _train(_model(), x[:, sl], y[:, sl],
                    reduce=lambda opt: opt.all_reduce_grads(world_size=ws, bucket_mb=0.001))
    lam = torch.linspace(-3.0, 5.0, 64).reshape(16, 4)[:, rank::ws].contiguous()
    moments = Moments(runner)
    low, invscale = moments(lam)
    low2, invscale2 = moments(lam * 2.0)
    torch.save({"params": params, "moments": torch.stack([low, invscale, low2, invscale2])},
               os.path.join(out_dir, f"rank{rank}.pt"))


@pytest.mark.timeout(300)
def test_two_rank_step_equals_full_batch_step(tmp_path):
    Runner(devices=2, accelerator="cpu").launch(_rank_fn, str(tmp_path))
    r0 = torch.load(tmp_path / "rank0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "rank1.pt", weights_only=True)
    # replicas stay bit-identical (same reduced gradient, same optimiser math)
    assert torch.equal(r0["params"], r1["params"])
    assert torch.equal(r0["moments"], r1["moments"])

    x, y = _data()
    full = _train(_model(), x, y)
    torch.testing.assert_close(r0["params"], full, rtol=1e-5, atol=1e-6)

    from sheeprl_prey_amd.algos.dreamer_v3.utils import Moments

    lam = torch.linspace(-3.0, 5.0, 64).reshape(16, 4)
    m = Moments(None)
    low, invscale = m(lam)
    low2, invscale2 = m(lam * 2.0)
    torch.testing.assert_close(r0["moments"], torch.stack([low, invscale, low2, invscale2]))


class _WithUnused(torch.nn.Module):
    def __init__(self):
        super().__init__()
        # never in the loss: head of the slab = the last bucket, completed by the sync itself
        self.unused = torch.nn.Linear(5, 5)
        self.body = _model()

    def forward(self, x):
        return self.body(x)


def _overlap_rank_fn(runner: Runner, out_dir: str) -> None:
    overlap = runner.overlap_grad_sync
    rank, ws = runner.global_rank, runner.world_size
    x, y = _data()
    half = BATCH // ws
    sl = slice(rank * half, (rank + 1) * half)
    torch.manual_seed(0)
    model = _WithUnused()
    opt = FlatAdam(model.parameters(), lr=1e-2)
    launched_in_backward = []
    for s in range(STEPS):
        opt.zero_grad()
        torch.nn.functional.mse_loss(model(x[s, sl]), y[s, sl]).backward()
        ov = getattr(opt, "_ov", None)
        launched_in_backward.append(ov["next"] if ov is not None and ov["armed"] else 0)
        runner.sync_gradients(opt)
        opt.step()
    params = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    torch.save({"params": params, "launched": torch.tensor(launched_in_backward),
                "buckets": torch.tensor(len(opt._ov["buckets"]) if getattr(opt, "_ov", None) else 0)},
               os.path.join(out_dir, f"{'ov' if overlap else 'plain'}{rank}.pt"))


@pytest.mark.timeout(300)
def test_overlapped_bucket_all_reduce_matches_plain(tmp_path):
    """Bucketed all-reduce launched from post-accumulate-grad hooks during the backward
    (``FlatOptimizer.enable_overlap``) gives the same replicas as the all-reduce after the backward,
    including a parameter that never receives a gradient."""
    for overlap in (False, True):
        Runner(devices=2, accelerator="cpu", bucket_mb=0.0002, overlap_grad_sync=overlap).launch(
            _overlap_rank_fn, str(tmp_path))
    plain = [torch.load(tmp_path / f"plain{r}.pt", weights_only=True) for r in range(2)]
    ov = [torch.load(tmp_path / f"ov{r}.pt", weights_only=True) for r in range(2)]
    assert torch.equal(ov[0]["params"], ov[1]["params"])
    assert torch.equal(ov[0]["params"], plain[0]["params"])
    # step 0 syncs on the plain path and enables the hooks; later steps launch buckets mid-backward
    # 52-float buckets: 4 of them, the 3 of the used layers launched before the backward returned
    assert int(ov[0]["buckets"]) == 4
    assert ov[0]["launched"].tolist() == [0] + [3] * (STEPS - 1)
    assert int(plain[0]["buckets"]) == 0
