"""DreamerV3-XL RSSM scan (deter 4096, dense 1024, hidden 1024, B 16, T 64): fwd and fwd+bwd time
of the fused scan (SRL_SKINNY=0: library GEMMs) vs the weight bytes it must stream per step (the scan is weight-bandwidth bound)."""
import time

import torch

from sheeprl_prey_amd.algos.dreamer_v3.agent import RSSM, RecurrentModel, init_weights
from sheeprl_prey_amd.models.models import MLP

H, D, hid, B, T, S, A, E = 4096, 1024, 1024, 16, 64, 1024, 17, 4096 + 1024
torch.manual_seed(0)
rec = RecurrentModel(S + A, H, D)
rep = MLP(H + E, S, [hid], activation=torch.nn.SiLU, norm_layer=[torch.nn.LayerNorm], norm_args=[{"normalized_shape": hid}])
tr = MLP(H, S, [hid], activation=torch.nn.SiLU, norm_layer=[torch.nn.LayerNorm], norm_args=[{"normalized_shape": hid}])
rssm = RSSM(rec.apply(init_weights), rep.apply(init_weights), tr.apply(init_weights), {"validate_args": False}).cuda()
emb = torch.randn(T, B, E, device="cuda", requires_grad=True)
act = torch.nn.functional.one_hot(torch.randint(0, A, (T, B), device="cuda"), A).float()
first = torch.zeros(T, B, 1, device="cuda")
first[0] = 1
uni = torch.rand(T, 2 * B * 32, device="cuda")
wbytes = 4 * (3 * H * (H + D) + H * hid + hid * S + D * S)
for it in range(6):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = rssm.scan_dynamic(emb, act, first, uniform=uni)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    sum(o.float().sum() for o in out).backward()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    if it >= 3:
        print(f"XL scan T={T} B={B}: fwd {1e3 * (t1 - t0):.2f} ms ({1e6 * (t1 - t0) / T:.1f} us/step), "
              f"bwd {1e3 * (t2 - t1):.2f} ms; recurrent weights {wbytes / 2**20:.0f} MiB/step -> "
              f"fwd {wbytes * T / (t1 - t0) / 1e12:.2f} TB/s effective", flush=True)
print("grad_fn", type(out[0].grad_fn).__name__)
