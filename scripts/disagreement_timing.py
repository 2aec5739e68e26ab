"""P2E-DV2 intrinsic-reward shape (10 members, 16 x 1024 imagined rows, hidden 400, 1024 posterior
features): fused head + member variance kernel vs the eager bmm + var + mean."""
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from sheeprl_prey_amd import ops  # noqa: E402

n, M, H, O = 10, 16384, 400, 1024
X = torch.randn(n, M, H, device="cuda")
W = torch.randn(n, O, H, device="cuda") / 20
b = torch.randn(n, O, device="cuda")


def eager():
    return torch.baddbmm(b.unsqueeze(1), X, W.transpose(1, 2)).var(0).mean(-1)


def fused():
    return ops.ensemble_disagreement(X, W, b)


for name, fn in (("eager bmm+var+mean", eager), ("fused kernel", fused)):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(f"{name:22s} {ms * 1e3:9.1f} us   ({2 * n * M * O * H / ms / 1e9:6.1f} TFLOP/s on the head GEMMs)")
print("max |fused - eager| / mean:", float((fused() - eager()).abs().max() / eager().abs().mean()))
