"""Side work (ops/sidestream.py deferral) beside the persistent scan BACKWARD, in isolation: a tap on the scan
outputs queues 20 short side kernels in the backward; the scan backward forks them.  eager vs graph."""
import sys
import torch

from sheeprl_prey_amd.algos.dreamer_v3.agent import RSSM, RecurrentModel, init_weights
from sheeprl_prey_amd.models.models import MLP
from sheeprl_prey_amd.ops import sidestream as ss

mode = sys.argv[1] if len(sys.argv) > 1 else "graph"
nside = int(sys.argv[2]) if len(sys.argv) > 2 else 20
torch.manual_seed(0)
H = D = hid = 512
B, T, S, A, E = 16, 64, 1024, 6, 4096
rec = RecurrentModel(S + A, H, D)
rep = MLP(H + E, S, [hid], activation=torch.nn.SiLU, norm_layer=[torch.nn.LayerNorm], norm_args=[{"normalized_shape": hid}])
tr = MLP(H, S, [hid], activation=torch.nn.SiLU, norm_layer=[torch.nn.LayerNorm], norm_args=[{"normalized_shape": hid}])
rssm = RSSM(rec.apply(init_weights), rep.apply(init_weights), tr.apply(init_weights), {"validate_args": False}).cuda()
rssm.scan_impl = "persist"
emb = torch.randn(T, B, E, device="cuda", requires_grad=True)
act = torch.nn.functional.one_hot(torch.randint(0, A, (T, B), device="cuda"), A).float()
first = torch.zeros(T, B, 1, device="cuda")
first[0] = 1
a = torch.randn(4096, 256, device="cuda")
import os
DIRECT = os.environ.get("PROBE_DIRECT") == "1"
side = torch.cuda.Stream()
outs = [torch.empty(4096, 256, device="cuda") for _ in range(nside)]
dummy = [torch.nn.Parameter(torch.zeros(4096, 256, device="cuda")) for _ in range(nside)]


class Tap(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        if DIRECT:
            # no sidestream module: fork a plain side stream here (before the scan backward is enqueued)
            cur = torch.cuda.current_stream()
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                torch.cuda._sleep(100000)  # hold the branch ~ until the scan has started
                for o in outs:
                    torch.mul(a, 2.0, out=o)
            torch.autograd.Variable._execution_engine.queue_callback(lambda: cur.wait_stream(side))
            return g
        if os.environ.get("PROBE_NOALLOC") == "1":
            for p, o in zip(dummy, outs):
                ss.param_grads(g.device, lambda o=o: (torch.mul(a, 2.0, out=o),), [p], a)
            return g
        for p in dummy:
            ss.param_grads(g.device, lambda: (torch.mul(a, 2.0),), [p], a)
        return g


def step():
    for p in dummy:
        p.grad = None
    hs = rssm.scan_dynamic(emb, act, first)[0]
    with ss.scope():
        Tap.apply(hs).square().sum().backward()


for _ in range(3):
    step()
torch.cuda.synchronize()
if mode == "graph":
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    torch.cuda.synchronize()
    torch.cuda._sleep(100)
    torch.cuda.synchronize()
    for _ in range(2):
        g.replay()
        torch.cuda.synchronize()
else:
    torch.cuda._sleep(100)
    torch.cuda.synchronize()
    for _ in range(2):
        step()
        torch.cuda.synchronize()
print("done", mode)
