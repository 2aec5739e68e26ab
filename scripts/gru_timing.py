"""Event-timed LN-GRU kernels (gru.hip) at the shapes the presets run: the XL scan (16 rows x deter 4096) and
imagination (1024 rows), the Atari-100k imagination (1024 x 512).  Prints effective HBM bandwidth per call.

    python scripts/gru_timing.py
"""
import json

import torch

from sheeprl_prey_amd import ops


def _time(fn, iters=50):
    for _ in range(3):
        fn()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(iters):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) * 1e3 / iters


def main():
    C = ops._ext()
    out = {}
    for M, H in ((16, 4096), (1024, 4096), (16, 512), (1024, 512), (1024, 2048)):
        g = torch.Generator(device="cuda").manual_seed(0)
        x = torch.randn(M, 3 * H, device="cuda", generator=g)
        h = torch.randn(M, H, device="cuda", generator=g)
        gam = 1 + 0.1 * torch.randn(3 * H, device="cuda", generator=g)
        bet = 0.1 * torch.randn(3 * H, device="cuda", generator=g)
        hn = torch.empty(M, H, device="cuda")
        mean, rstd = torch.empty(M, device="cuda"), torch.empty(M, device="cuda")
        C.set_gru_vec(False)
        fwd_s = _time(lambda: C.ln_gru_into(x, h, gam, bet, 1e-3, hn, mean, rstd))
        C.set_gru_vec(True)
        fwd = _time(lambda: C.ln_gru_into(x, h, gam, bet, 1e-3, hn, mean, rstd))
        grid = C.ln_gru_bwd_grid(M)
        dhn = torch.randn(M, H, device="cuda", generator=g)
        dx, dh = torch.empty_like(x), torch.empty_like(h)
        pdg, pdb = torch.empty(grid, 3 * H, device="cuda"), torch.empty(grid, 3 * H, device="cuda")
        dg, db = torch.empty(3 * H, device="cuda"), torch.empty(3 * H, device="cuda")
        bwd = _time(lambda: C.ln_gru_bwd_into(x, h, H, gam, bet, mean, rstd, dhn, dx, dh, pdg, pdb, dg, db, M, H))
        fb = 4 * (M * 3 * H + 2 * M * H)  # x, h in; hn out
        bb = 4 * (2 * M * 3 * H + 3 * M * H + 2 * grid * 3 * H)  # x, dx; h, dhn, dh; partials
        out[f"{M}x{H}"] = {"fwd_us": round(fwd, 1), "fwd_scalar_us": round(fwd_s, 1), "fwd_GBps": round(fb / fwd / 1e3, 0),
                           "bwd_us": round(bwd, 1),
                           "bwd_GBps": round(bb / bwd / 1e3, 0)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
