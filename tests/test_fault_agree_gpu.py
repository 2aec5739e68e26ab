"""The device-side update skip is a COLLECTIVE decision (two gloo ranks sharing the one GPU).

A kernel fault (persistent-scan hand-off timeout, out-of-range replay index) sets word 0 / 1 of the device
fault block (``ops.fault_block``) and the flat optimisers' norm / advance kernels then skip the update.  If only
the faulted rank skipped, its replica would silently diverge from the others after the gradient all-reduce.
``Runner.agree_faults`` (called by the world-model ``sync_gradients(..., faults=True)`` of DV1/DV2/DV3/P2E)
all-reduces those words, so here rank 1 alone trips the guard and BOTH ranks must skip the step, count it, and
keep bit-identical parameters; a following clean step must update both."""
import os
import socket
import types

import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank: int, port: int, out_dir: str) -> None:
    import torch.distributed as dist

    from sheeprl_prey_amd import ops
    from sheeprl_prey_amd.parallel.flat_optim import FlatAdam
    from sheeprl_prey_amd.parallel.runner import Runner

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    try:
        dev = torch.device("cuda", 0)
        torch.manual_seed(0)
        m = torch.nn.Linear(32, 16).to(dev)
        opt = FlatAdam(m.parameters(), lr=1e-2)
        fb = ops.fault_block(dev)
        fb.zero_()
        shim = types.SimpleNamespace(world_size=2, group=None)
        res = {}
        for step in range(2):
            opt.zero_grad()
            x = torch.randn(8, 32, device=dev, generator=torch.Generator(device=dev).manual_seed(7))
            m(x).square().mean().backward()
            opt._gather()
            if step == 0 and rank == 1:
                fb[1] = 1  # a replay-gather fault on rank 1 only
            Runner.agree_faults(shim, dev)
            opt.clip_grad_norm_(1.0)
            opt.step()
            torch.cuda.synchronize()
            res[step] = (fb.cpu().clone(), opt.flat_param.detach().cpu().clone())
            fb[:2] = 0  # the host health check's reset
        torch.save(res, os.path.join(out_dir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_fault_skip_is_collective(tmp_path):
    import torch.multiprocessing as mp

    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    mp.spawn(_rank, args=(_free_port(), str(tmp_path)), nprocs=2, join=True)
    r0 = torch.load(tmp_path / "r0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "r1.pt", weights_only=True)
    fb0, p0 = r0[0]
    fb1, p1 = r1[0]
    assert int(fb0[1]) == 1 and int(fb1[1]) == 1, (fb0, fb1)   # both ranks saw the fault
    assert int(fb0[2]) == 1 and int(fb1[2]) == 1, (fb0, fb1)   # both skipped that update
    assert torch.equal(p0, p1)
    # the clean second step updates both replicas identically
    (_, q0), (_, q1) = r0[1], r1[1]
    assert torch.equal(q0, q1) and not torch.equal(q0, p0)
