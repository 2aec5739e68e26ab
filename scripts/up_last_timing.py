"""A/B of the decoder's final ConvTranspose2d (Ca -> CO image channels, k4 s2 p1): the input-centric MFMA kernel
(``up_last_mfma_kernel``) vs the VALU form (``up_small2_kernel``), event-timed, checked against
``F.conv_transpose2d``.  Default shape: Atari-100k (1024 frames, 32 -> 3 channels, 32x32 -> 64x64).

    python scripts/up_last_timing.py [N] [Ca] [CO] [SH]
"""
import json
import sys

import torch
import torch.nn.functional as F

from sheeprl_prey_amd import ops


def main(N=1024, Ca=32, CO=3, SH=32, iters=50):
    C = ops._ext()
    torch.manual_seed(0)
    x = torch.randn(N, Ca, SH, SH, device="cuda")
    w = torch.randn(Ca, CO, 4, 4, device="cuda") * 0.1
    b = torch.randn(CO, device="cuda")
    p = x.permute(0, 2, 3, 1).contiguous()
    ref = F.conv_transpose2d(x, w, b, stride=2, padding=1) + 0.5
    res = {"shape": [N, Ca, CO, SH]}
    for form, name in ((0, "mfma"), (1, "valu")):
        C.set_up_last_form(form)
        out = C.conv_up_small(p, w, b, 0.5)
        err = float((out - ref).abs().max())
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for _ in range(3):
            C.conv_up_small(p, w, b, 0.5)
        ev[0].record()
        for _ in range(iters):
            C.conv_up_small(p, w, b, 0.5)
        ev[1].record()
        torch.cuda.synchronize()
        res[name] = {"us": round(ev[0].elapsed_time(ev[1]) * 1e3 / iters, 1), "max_abs_err": err}
    C.set_up_last_form(0)
    print(json.dumps(res))


if __name__ == "__main__":
    a = [int(v) for v in sys.argv[1:]]
    main(*a)
