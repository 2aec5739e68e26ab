"""Does a side-stream branch run beside the persistent RSSM scan?  main: the fused posterior scan forward
(persistent kernel, Atari dims); side: 20 short elementwise kernels forked before it.  eager vs graph."""
import sys
import torch

from sheeprl_prey_amd.algos.dreamer_v3.agent import RSSM, RecurrentModel, init_weights
from sheeprl_prey_amd.models.models import MLP

mode = sys.argv[1] if len(sys.argv) > 1 else "graph"
torch.manual_seed(0)
H = D = hid = 512
B, T, S, A, E = 16, 64, 1024, 6, 4096
rec = RecurrentModel(S + A, H, D)
rep = MLP(H + E, S, [hid], activation=torch.nn.SiLU, norm_layer=[torch.nn.LayerNorm], norm_args=[{"normalized_shape": hid}])
tr = MLP(H, S, [hid], activation=torch.nn.SiLU, norm_layer=[torch.nn.LayerNorm], norm_args=[{"normalized_shape": hid}])
rssm = RSSM(rec.apply(init_weights), rep.apply(init_weights), tr.apply(init_weights), {"validate_args": False}).cuda()
rssm.scan_impl = "persist"
emb = torch.randn(T, B, E, device="cuda")
act = torch.nn.functional.one_hot(torch.randint(0, A, (T, B), device="cuda"), A).float()
first = torch.zeros(T, B, 1, device="cuda")
first[0] = 1
a = torch.randn(4096, 256, device="cuda")
outs = [torch.empty(4096, 256, device="cuda") for _ in range(20)]
side = torch.cuda.Stream()


def step():
    cur = torch.cuda.current_stream()
    ev = torch.cuda.Event()
    ev.record(cur)
    with torch.no_grad():
        rssm.scan_dynamic(emb, act, first)
    side.wait_event(ev)
    with torch.cuda.stream(side):
        for o in outs:
            torch.mul(a, 2.0, out=o)
    cur.wait_stream(side)


for _ in range(2):
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
