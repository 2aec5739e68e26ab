"""RCCL on the real device (one rank: the multi-GPU runs are the driver's).  The framework's gradient
collectives - the bucketed flat-slab all-reduce (``FlatOptimizer.all_reduce_grads``), the
overlapped per-bucket all-reduce launched from post-accumulate-grad hooks (``enable_overlap``) - and
the all-gather the DreamerV3 lambda / Moments path uses, issued over a 1-rank ``nccl`` (= RCCL) group
with ReduceOp.AVG: every result must equal the local value exactly.  ``world_size=2`` is passed to the
optimiser so its multi-rank code paths run (AVG over the one real rank leaves the values unchanged)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.nn as nn

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture
def rccl_group():
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        yield None
    finally:
        dist.destroy_process_group()


def _model_and_batch():
    torch.manual_seed(0)
    m = nn.Sequential(nn.Linear(64, 256), nn.ReLU(), nn.Linear(256, 256), nn.ReLU(), nn.Linear(256, 8)).cuda()
    x = torch.randn(32, 64, device="cuda")
    return m, x


def test_rccl_flat_slab_all_reduce_and_overlap(rccl_group):
    from sheeprl_prey_amd.parallel.flat_optim import FlatAdam

    assert dist.get_backend() == "nccl"
    m, x = _model_and_batch()
    opt = FlatAdam(m.parameters(), lr=1e-3)
    opt.zero_grad()
    m(x).square().mean().backward()
    opt._gather()
    expected = opt.flat_grad.clone()
    # 1) bucketed async all-reduce over slab slices (bucket of ~1 k floats: many buckets)
    opt.zero_grad()
    m(x).square().mean().backward()
    opt.all_reduce_grads(None, world_size=2, bucket_mb=0.004)
    torch.cuda.synchronize()
    assert torch.equal(opt.flat_grad, expected)
    # 2) overlapped buckets launched from the backward hooks, finished by the sync
    assert opt.enable_overlap(None, world_size=2, bucket_mb=0.004)
    assert len(opt._ov["buckets"]) >= 2
    opt.zero_grad()
    m(x).square().mean().backward()
    assert len(opt._ov["works"]) > 0, "no bucket all-reduce was launched during the backward"
    opt.all_reduce_grads(None, world_size=2)
    torch.cuda.synchronize()
    assert torch.equal(opt.flat_grad, expected)
    opt.step()  # the slab stays usable by the fused Adam after the collectives


def test_rccl_all_gather_into_tensor(rccl_group):
    lam = torch.randn(15, 1024, 1, device="cuda")
    buf = torch.empty((1,) + tuple(lam.shape), device="cuda")
    dist.all_gather_into_tensor(buf, lam)
    torch.cuda.synchronize()
    assert torch.equal(buf[0], lam)
