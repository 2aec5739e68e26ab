"""hipGraph execution modes (parallel/graphs.py) with the flat optimisers' deferred gradient gather:
in the multi-rank (segmented) mode the collective between two phase graphs must see the gradients of
the phase before it.  A fake collective (zeroing the slab) stands in for the RCCL all-reduce, so one
GPU checks the ordering."""
import pytest
import torch

from sheeprl_prey_amd.parallel.flat_optim import build_optimizer
from sheeprl_prey_amd.parallel.graphs import SegmentedGraph

pytestmark = pytest.mark.gpu


def test_segmented_graph_collective_sees_phase_gradients():
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.Tanh(), torch.nn.Linear(16, 4)).cuda()
    opt = build_optimizer({"_target_": "torch.optim.SGD", "lr": 0.1}, net.parameters())
    seen = []

    def fwd_bwd(data):
        opt.zero_grad(set_to_none=True)
        net(data["x"]).square().sum().backward()

    def coll(dry: bool = False):
        if not dry:
            opt.all_reduce_grads(None, 1)  # rebuilds the slab if needed (eager path)
            seen.append(float(opt.flat_grad.abs().sum()))
            opt.flat_grad.zero_()  # "collective" result: every rank's gradient cancels

    def apply(data):
        opt.step()
        return {"p": opt.flat_param}

    seg = SegmentedGraph([fwd_bwd, apply], [coll], warmup=2)
    before = opt.flat_param.clone()
    x = torch.randn(32, 8, device="cuda")
    for _ in range(6):
        seg({"x": x})
    torch.cuda.synchronize()
    assert seg.graphs is not None
    # the collective saw real gradients every step (they were in the slab before it ran) ...
    assert len(seen) == 6 and all(s > 0 for s in seen), seen
    # ... and its result (zeros) is what the optimiser applied: no update at all
    torch.testing.assert_close(opt.flat_param, before)


def test_gemm_tuning_use_loads_results():
    import torch.cuda.tunable as tun

    from sheeprl_prey_amd.parallel import gemm_tuning

    try:
        assert gemm_tuning.configure("use") is True
        assert tun.is_enabled() and not tun.tuning_is_enabled()
        a, b = torch.randn(1024, 512, device="cuda"), torch.randn(512, 1536, device="cuda")
        torch.testing.assert_close(a @ b, (a.double() @ b.double()).float(), rtol=1e-4, atol=1e-3)
    finally:
        tun.enable(False)
