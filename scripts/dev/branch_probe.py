"""Graph-branch dispatch probe: main branch = one long spin kernel, side branch = N short kernels.
Prints when the side kernels run relative to the spin (rocprofv3 kernel trace of this script)."""
import sys
import torch

mode = sys.argv[1] if len(sys.argv) > 1 else "graph"
dev = torch.device("cuda")
a = torch.randn(4096, 256, device=dev)
outs = [torch.empty(4096, 256, device=dev) for _ in range(10)]
side = torch.cuda.Stream()
main = torch.cuda.current_stream()


def step():
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream())
    torch.cuda._sleep(1_000_000)  # ~0.4 ms spin on the main branch
    side.wait_event(ev)
    with torch.cuda.stream(side):
        for o in outs:
            torch.mul(a, 2.0, out=o)
    torch.cuda.current_stream().wait_stream(side)


if mode == "graph":
    s = torch.cuda.Stream()
    s.wait_stream(main)
    with torch.cuda.stream(s):
        step()
    main.wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    torch.cuda.synchronize()
    torch.cuda._sleep(100)
    torch.cuda.synchronize()
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
else:
    torch.cuda._sleep(100)
    torch.cuda.synchronize()
    for _ in range(3):
        step()
        torch.cuda.synchronize()
torch.cuda.synchronize()
print("done", mode)
