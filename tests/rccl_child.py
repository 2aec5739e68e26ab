"""RCCL cases run in a CHILD process each (``tests/test_rccl_gpu.py`` launches ``python tests/rccl_child.py
<case>``): a process-group abort (SIGABRT from a C++ watchdog / runtime assertion) then fails one test
instead of taking the whole GPU suite down with it.  Each case opens a 1-rank ``nccl`` (= RCCL) group on
cuda:0; the optimiser / trainer is told there are 2 ranks so the multi-rank code paths run (ReduceOp.AVG
over the one real rank is the identity).  Exit status 0 = pass; ``faulthandler`` dumps every thread on a
fatal signal."""
import faulthandler
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.nn as nn  # noqa: E402


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _model_and_batch():
    torch.manual_seed(0)
    m = nn.Sequential(nn.Linear(64, 256), nn.ReLU(), nn.Linear(256, 256), nn.ReLU(), nn.Linear(256, 8)).cuda()
    x = torch.randn(32, 64, device="cuda")
    return m, x


class _CollectiveLog:
    """Wraps the torch.distributed collectives: records, per call, whether a hipGraph capture was open on
    the calling thread's stream (the invariant: never - no collective is captured)."""

    NAMES = ("all_reduce", "all_gather_into_tensor", "all_gather", "broadcast", "reduce_scatter_tensor")

    def __init__(self):
        self.calls = []
        self._orig = {}

    def __enter__(self):
        for n in self.NAMES:
            f = getattr(dist, n)
            self._orig[n] = f

            def wrap(*a, _f=f, _n=n, **k):
                self.calls.append((_n, torch.cuda.is_current_stream_capturing()))
                return _f(*a, **k)

            setattr(dist, n, wrap)
        return self

    def __exit__(self, *exc):
        for n, f in self._orig.items():
            setattr(dist, n, f)


def case_flat_slab_all_reduce_and_overlap():
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


def case_all_gather_into_tensor():
    lam = torch.randn(15, 1024, 1, device="cuda")
    buf = torch.empty((1,) + tuple(lam.shape), device="cuda")
    dist.all_gather_into_tensor(buf, lam)
    torch.cuda.synchronize()
    assert torch.equal(buf[0], lam)


def case_hooks_silent_inside_capture():
    """The overlap hooks launch nothing while a hipGraph is being captured (round 5's captured-collective
    mode aborted the process there): the captured backward records no collective, the eager sync after
    the replay averages the whole slab."""
    from sheeprl_prey_amd.parallel.flat_optim import FlatAdam

    m, x = _model_and_batch()
    ref = torch.cat([g.reshape(-1) for g in torch.autograd.grad(m(x).square().mean(), list(m.parameters()))])
    opt = FlatAdam(m.parameters(), lr=0.0)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            opt.zero_grad()
            m(x).square().mean().backward()
            opt.all_reduce_grads(None, world_size=2, bucket_mb=0.004)
        assert opt.enable_overlap(None, world_size=2, bucket_mb=0.004)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    from sheeprl_prey_amd.parallel.graphs import capture_error_mode, quiesce_for_capture

    quiesce_for_capture()
    g = torch.cuda.CUDAGraph()
    with _CollectiveLog() as log, torch.cuda.graph(g, capture_error_mode=capture_error_mode()):
        opt.zero_grad()
        m(x).square().mean().backward()
        launched = len(opt._ov["works"])
    assert launched == 0 and not log.calls, (launched, log.calls)
    g.replay()
    opt.all_reduce_grads(None, world_size=2)
    torch.cuda.synchronize()
    got = torch.cat([opt.flat_grad[o:o + p.numel()] for p, o in zip(opt.params, opt.offsets)])
    torch.testing.assert_close(got, ref, rtol=1e-6, atol=1e-7)


def case_dv3_segmented_step():
    """DreamerV3's multi-rank graph mode (``segmented``: one hipGraph per phase, the RCCL collectives eagerly
    between replays - what an N-GPU run executes) on the real RCCL group, the runner reporting 2 ranks.  No
    collective may be issued inside a capture, and the step must reproduce the plain 1-rank graph step."""
    from sheeprl_prey_amd.parallel.runner import Runner
    from tests.test_dreamer_gpu import _build, _data

    fake = {"ws": 1}  # what Runner.world_size reports: 1 while the reference trainer runs, 2 for the segmented one
    Runner.world_size = property(lambda self: fake["ws"])
    ref = _build(graphs=True, seed=5)
    real_gather = dist.all_gather_into_tensor

    def gather_2(out, inp, group=None, async_op=False):  # the 2nd "rank" holds the same values
        real_gather(out[:1], inp, group=group)
        out[1:].copy_(out[:1].expand_as(out[1:]))

    dist.all_gather_into_tensor = gather_2
    fake["ws"] = 2
    tr = _build(graphs=True, seed=5)
    assert tr.graph_mode == "segmented" and ref.graph_mode == "single", (tr.graph_mode, ref.graph_mode)
    data = _data(seed=9)
    la, lb = [], []
    log = _CollectiveLog()
    for i in range(5):
        fake["ws"] = 1
        torch.manual_seed(100 + i)
        la.append(float(ref.train_step(data)["Loss/world_model_loss"]))
        fake["ws"] = 2
        torch.manual_seed(100 + i)
        with log:
            out = tr.train_step(data)
        lb.append(float(out["Loss/world_model_loss"]))
    assert tr.seg.graphs is not None
    assert log.calls and not any(cap for _, cap in log.calls), log.calls
    assert abs(la[1] - lb[1]) / abs(la[1]) < 1e-3, (la, lb)
    assert lb[-1] < lb[0], lb
    for k in ("Loss/policy_loss", "Loss/value_loss", "Grads/actor", "Grads/critic"):
        assert torch.isfinite(out[k]).all(), k


CASES = {k[5:]: v for k, v in dict(globals()).items() if k.startswith("case_")}


def main(name: str) -> int:
    faulthandler.enable(all_threads=True)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        CASES[name]()
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()
    print(f"__RCCL_CASE_OK__ {name}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
