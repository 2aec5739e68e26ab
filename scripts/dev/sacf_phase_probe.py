"""Phase timestamps inside the fused SAC target / update kernels (workgroup 0, s_memrealtime at 100 MHz) at the
bench shape (walker: obs 24, action 6, hidden 256, 2 critics, batch 256).  Prints us per phase (median of 20)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from sheeprl_prey_amd import ops  # noqa: E402
from sheeprl_prey_amd.algos.sac.agent import SACActor, SACCriticEnsemble  # noqa: E402


def main():
    C = ops._ext()
    torch.manual_seed(0)
    OD, A, H, n, M = 24, 6, 256, 2, 256
    a = SACActor(OD, A, hidden_size=H).cuda()
    crit = SACCriticEnsemble(OD + A, n=n, hidden_size=H).cuda()
    m = a.model.model
    aw = [m[0].weight, m[0].bias, m[2].weight, m[2].bias, a.fc_mean.weight, a.fc_mean.bias, a.fc_logstd.weight,
          a.fc_logstd.bias, a.action_scale, a.action_bias]
    e = crit.model
    cw = [e.layers[0].weight, e.layers[0].bias, e.layers[1].weight, e.layers[1].bias, e.head.weight, e.head.bias]
    obs = torch.randn(M, OD, device="cuda")
    rew, done = torch.randn(M, device="cuda"), torch.zeros(M, device="cuda")
    la = torch.tensor([-0.5], device="cuda")
    te = torch.tensor([-6.0], device="cuda")
    ctr = torch.zeros(2, dtype=torch.int64, device="cuda")
    y = torch.empty(M, device="cuda")
    zp, nb = C.sac_fused_zp(A), C.sac_fused_blocks(M)
    ws = [torch.empty(M, 32, device="cuda"), *[torch.empty(M, H, device="cuda") for _ in range(2)],
          torch.empty(M, zp, device="cuda"), *[torch.empty(M, H, device="cuda") for _ in range(2)],
          torch.empty(n, M, device="cuda"), torch.empty(n, M, A, device="cuda"), torch.empty(nb, 2, device="cuda")]
    cnt = torch.zeros(nb, dtype=torch.int32, device="cuda")
    grads = [torch.empty_like(p) for p in aw[:8]] + [torch.empty(1, device="cuda")]
    losses = torch.empty(2, device="cuda")
    tt = torch.zeros(16, dtype=torch.int64, device="cuda")
    tu = torch.zeros(16, dtype=torch.int64, device="cuda")
    rt, ru = [], []
    for i in range(25):
        tt.zero_()
        tu.zero_()
        C.sac_fused_target(obs, rew, done, la, aw, -5.0, 2.0, cw, ctr, 7, 0.99, y, None, None, None, tt)
        C.sac_fused_actor(obs, la, te, aw, -5.0, 2.0, cw, ctr, 7, True, ws, cnt, grads, None, losses, None, None, None,
                          None, None, tu)
        torch.cuda.synchronize()
        if i >= 5:
            rt.append(tt.cpu().numpy().astype(np.float64))
            ru.append(tu.cpu().numpy().astype(np.float64))
    for name, r, labels in (("tgt_kernel", rt, ["load", "actor fwd", "sample", "c0 l1", "c0 l2+q", "c1 l1", "c1 l2+q",
                                                   "y"]),
                            ("upd_kernel", ru, ["load", "actor fwd", "sample+c l1", "c l2+q", "dq/da bwd", "ticket",
                                                "(last wg) ->", "reduce+squash bwd", "DZ+dh2a", "dh1a+loss"])):
        d = np.median(np.diff(np.stack(r), axis=1), axis=0) * 10 / 1000  # 100 MHz ticks -> us
        print(name)
        for k, lab in enumerate(labels):
            print(f"  {k}->{k + 1} {lab:22s} {d[k]:7.2f} us")
        print(f"  total {np.median(np.stack(r)[:, len(labels)] - np.stack(r)[:, 0]) / 100:7.2f} us")


if __name__ == "__main__":
    main()
