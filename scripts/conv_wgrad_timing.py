"""Per-call timing of the conv weight-gradient kernel (conv.hip wgrad_kernel + split reduce) at the DreamerV3
encoder / decoder layer shapes (N = B*T = 1024 frames): the Atari-100k model (channel multiplier 32) and the XL
model (multiplier 96).  Every k4 s2 p1 layer's weight gradient is one call C.conv_wgrad(P, Q, Cb) with P the
small-grid NHWC operand and Q the large-grid one (encoder: dZ and the input; decoder: the input and dZ).

    python scripts/conv_wgrad_timing.py          (A/B switches are environment variables read at load:
                                                  SRL_WGRAD_REMAP=0, SRL_WGRAD_PLAN=0)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sheeprl_prey_amd import ops  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    C = ops._ext()
    N = 1024
    tag = " ".join(f"{k}={os.environ[k]}" for k in ("SRL_WGRAD_REMAP", "SRL_WGRAD_PLAN") if k in os.environ) or "default"
    tot_us = {}
    for name, mult in (("atari", 32), ("xl", 96)):
        # (small grid side, Ca = channels on the small grid, Cb = channels on the large grid)
        shapes = [(32, mult, 3), (16, 2 * mult, mult), (8, 4 * mult, 2 * mult), (4, 8 * mult, 4 * mult)]
        tot = 0.0
        for (s, ca, cb) in shapes:
            cbp = 4 if cb < 4 else cb
            P = torch.randn(N, s, s, ca, device="cuda")
            Q = torch.randn(N, 2 * s, 2 * s, cbp, device="cuda")
            if cb < cbp:
                Q[..., cb:] = 0
            us = timeit(lambda: C.conv_wgrad(P, Q, cb))
            fl = 2.0 * N * s * s * ca * 16 * cb
            tot += us * (2 if s < 32 else 1)  # the three inner shapes occur twice (encoder + decoder)
            print(f"[{tag}] {name} wgrad P={N}x{s}x{s}x{ca} Q={N}x{2 * s}x{2 * s}x{cbp}: {us:8.1f} us "
                  f"({fl / us / 1e6:6.1f} TF/s)", flush=True)
            del P, Q
        tot_us[name] = tot
        print(f"[{tag}] {name}: weight gradients per train step (E1 + 2 x inner) {tot / 1e3:.3f} ms", flush=True)
    # numerics spot check against the fp64 reference of one XL shape
    P = torch.randn(64, 8, 8, 384, device="cuda")
    Q = torch.randn(64, 16, 16, 192, device="cuda")
    dw = C.conv_wgrad(P, Q, 192)
    ref = torch.nn.grad.conv2d_weight(Q.permute(0, 3, 1, 2).double(), (384, 192, 4, 4), P.permute(0, 3, 1, 2).double(),
                                      stride=2, padding=1)
    err = ((dw.double() - ref).abs().max() / ref.abs().max()).item()
    print(f"[{tag}] max rel err vs fp64 (64 frames, 384x192): {err:.2e}", flush=True)
    assert err < 1e-5


if __name__ == "__main__":
    main()
