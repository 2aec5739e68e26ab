"""Conv weight-gradient kernels (csrc/conv.hip wgrad_kernel + reduce) at the Atari-100k layer shapes (B*T = 1024 frames):
us per call and TF/s for each main-loop variant (set_wgrad_variant: 0 default, 1 = 64 pixels per LDS stage,
2 = double-buffered LDS, 3 = both), plus the max abs error vs the default variant."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from sheeprl_prey_amd import ops  # noqa: E402

SHAPES = [  # (P small grid [N, SH, SW, Ca], Q large grid channels Cb)
    (1024, 16, 16, 64, 32),
    (1024, 8, 8, 128, 64),
    (1024, 4, 4, 256, 128),
    (1024, 32, 32, 32, 4),
]


def main():
    C = ops._ext()
    torch.manual_seed(0)
    for N, SH, SW, Ca, Cb in SHAPES:
        P = torch.randn(N, SH, SW, Ca, device="cuda")
        Q = torch.randn(N, 2 * SH, 2 * SW, Cb, device="cuda")
        flop = 2.0 * N * SH * SW * Ca * Cb * 16
        ref = None
        for v in ((0, 1, 2, 3) if hasattr(C, "set_wgrad_variant") else (0,)):  # the variants were not kept
            if v:
                C.set_wgrad_variant(v)
            for _ in range(3):
                dw = C.conv_wgrad(P, Q, Cb)
            torch.cuda.synchronize()
            ts = []
            for _ in range(20):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                dw = C.conv_wgrad(P, Q, Cb)
                b.record()
                torch.cuda.synchronize()
                ts.append(a.elapsed_time(b) * 1e3)
            us = float(np.median(ts))
            if ref is None:
                ref = dw.clone()
            err = float((dw - ref).abs().max() / ref.abs().max())
            print(f"P {N}x{SH}x{SW}x{Ca} Cb {Cb} var {v}: {us:8.1f} us  {flop / us / 1e6:6.1f} TF/s  rel err {err:.2e}", flush=True)
        if hasattr(C, "set_wgrad_variant"):
            C.set_wgrad_variant(0)


if __name__ == "__main__":
    main()
