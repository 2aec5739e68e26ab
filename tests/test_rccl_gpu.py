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


def test_rccl_collectives_captured_in_hipgraph(rccl_group):
    """The single-graph multi-rank mode: the flat-slab all-reduce - deferred (``wait=False``, joined by
    ``step``) and launched from the backward hooks during the capture (``in_capture``) - recorded in a
    hipGraph together with the backward, then replayed on new inputs: every replay's averaged slab must
    equal the local gradient of that replay's input."""
    from sheeprl_prey_amd.parallel.flat_optim import FlatAdam

    m, x = _model_and_batch()
    opt = FlatAdam(m.parameters(), lr=0.0)  # lr 0: the weights stay fixed, so gradients are comparable
    static_x = x.clone()

    def expected_for(inp):  # plain eager gradients of the same model (fresh tensors, the slab untouched)
        for p in m.parameters():
            p.grad = None
        m(inp).square().mean().backward()
        return torch.cat([p.grad.reshape(-1) for p in m.parameters()])

    # warm-up eagerly on a side stream (communicator, allocator), enabling the hook overlap in capture
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            opt.zero_grad()
            m(static_x).square().mean().backward()
            opt.all_reduce_grads(None, world_size=2, bucket_mb=0.004)
        assert opt.enable_overlap(None, world_size=2, bucket_mb=0.004, in_capture=True)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()

    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):  # the RCCL watchdog polls from its own thread
        opt.zero_grad()
        m(static_x).square().mean().backward()
        launched = len(opt._ov["works"])
        opt.all_reduce_grads(None, world_size=2, wait=False)
        opt.wait_grads()
        captured = opt.flat_grad.clone()
    assert launched > 0, "no bucket all-reduce was captured from the backward hooks"
    for seed in range(3):
        torch.manual_seed(100 + seed)
        new_x = torch.randn_like(static_x)
        static_x.copy_(new_x)
        g.replay()
        torch.cuda.synchronize()
        got = torch.cat([captured[o:o + p.numel()] for p, o in zip(opt.params, opt.offsets)])
        exp = expected_for(new_x)
        torch.testing.assert_close(got, exp, rtol=1e-6, atol=1e-7)


def test_dv3_step_graph_with_captured_collectives(rccl_group, monkeypatch):
    """DreamerV3's multi-rank single-graph mode (``graph_mode == 'single+rccl'``) on the real RCCL
    group: the runner reports 2 ranks, so every collective of the step (bucketed world-model all-reduce
    from the backward hooks, the lambda all-gather, the actor all-reduce left in flight across the
    critic phase, the critic all-reduce) is issued and CAPTURED in the step's hipGraph; AVG over the one
    real rank is the identity, so the step must reproduce the plain 1-rank graph step."""
    from sheeprl_prey_amd.parallel.runner import Runner
    from tests.test_dreamer_gpu import _build, _data

    ref = _build(graphs=True, seed=5)
    monkeypatch.setattr(Runner, "world_size", property(lambda self: 2))
    real_gather = dist.all_gather_into_tensor

    def gather_2(out, inp, group=None, async_op=False):  # the 2nd "rank" holds the same values
        real_gather(out[:1], inp, group=group)
        out[1:].copy_(out[:1].expand_as(out[1:]))

    monkeypatch.setattr(dist, "all_gather_into_tensor", gather_2)
    tr = _build(graphs=True, seed=5, extra=("fabric.graph_collectives=True",))  # opt-in mode (default: segmented)
    assert tr.graph_mode == "single+rccl", tr.graph_mode
    data = _data(seed=9)
    la, lb = [], []
    for i in range(5):
        torch.manual_seed(100 + i)
        la.append(float(ref.train_step(data)["Loss/world_model_loss"]))
        torch.manual_seed(100 + i)
        out = tr.train_step(data)
        lb.append(float(out["Loss/world_model_loss"]))
    assert tr.graphed.graph is not None
    assert tr.world_optimizer._ov is not None and tr.world_optimizer._ov["in_capture"]
    assert abs(la[1] - lb[1]) / abs(la[1]) < 1e-3, (la, lb)
    assert lb[-1] < lb[0], lb
    for k in ("Loss/policy_loss", "Loss/value_loss", "Grads/actor", "Grads/critic"):
        assert torch.isfinite(out[k]).all(), k
