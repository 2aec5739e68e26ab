"""Per-phase cycle counts of the 4-launch RSSM scan kernels (block 0, last recorded step).

    python scripts/scan4_phases.py            # DreamerV3 Atari-100k shapes: B16 T64 H512 D512 hid512 S1024
    python scripts/scan4_phases.py 256 1024 256 100   # the prey preset: deter 256, dense 1024, hidden 256, 100 actions
"""
import sys

import torch

from sheeprl_prey_amd import ops
from sheeprl_prey_amd.algos.dreamer_v3.agent import RSSM, RecurrentModel, init_weights
from sheeprl_prey_amd.models.models import MLP


def main(H=512, D=512, hid=512, B=16, T=64, E=4096, A=9):
    torch.manual_seed(0)
    S = 32 * 32
    rec = RecurrentModel(S + A, H, D)
    rep = MLP(H + E, S, [hid], activation=torch.nn.SiLU, norm_layer=[torch.nn.LayerNorm], norm_args=[{"normalized_shape": hid}])
    tr = MLP(H, S, [hid], activation=torch.nn.SiLU, norm_layer=[torch.nn.LayerNorm], norm_args=[{"normalized_shape": hid}])
    rssm = RSSM(rec.apply(init_weights), rep.apply(init_weights), tr.apply(init_weights), {"validate_args": False}).cuda()
    rssm.scan_impl = "scan4"
    emb = torch.randn(T, B, E, device="cuda", requires_grad=True)
    act = torch.nn.functional.one_hot(torch.randint(0, A, (T, B), device="cuda"), A).float()
    first = (torch.rand(T, B, 1, device="cuda") < 0.05).float()
    prof = torch.zeros(128, dtype=torch.int64, device="cuda")
    C = ops._ext()
    for it in range(3):
        if it == 2:
            C.set_scan4_prof(prof)
        out = rssm.scan_dynamic(emb, act, first)
        sum(o.float().sum() for o in out).backward()
        torch.cuda.synchronize()
    C.set_scan4_prof(None)
    p = prof.cpu().tolist()
    for k, name in enumerate(["f1", "f2", "f3", "f4", "g1", "g2", "g3", "g4"]):
        st = [v for v in p[k * 16:(k + 1) * 16]]
        n = max(i for i, v in enumerate(st) if v) + 1 if any(st) else 0
        d = [st[i + 1] - st[i] for i in range(n - 1)]
        tot = st[n - 1] - st[0] if n else 0
        print(f"{name}: total {tot:7d} cyc ({tot / 2400:.1f} us @2.4GHz) phases " + " ".join(f"{x}" for x in d))


if __name__ == "__main__":
    a = [int(x) for x in sys.argv[1:]]
    main(*a[:3], A=a[3]) if len(a) >= 4 else main(*a)
