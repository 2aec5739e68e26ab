"""Event-timed A/B of the imagination prior head at the Atari-100k shape (M = 1024 rows, K = 512, N = 32 x 32): the
one-launch ``prior_head.hip`` vs the three-launch form (LayerNorm + act kernel, hipBLASLt GEMM + bias, unimix
sampler).  Also times the library GEMM alone (the floor the fused kernel's MFMA body competes with).

    python scripts/prior_head_timing.py [M] [K]
"""
import json
import sys

import torch

from sheeprl_prey_amd import ops


def _time(fn, iters=200):
    for _ in range(5):
        fn()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(iters):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return round(ev[0].elapsed_time(ev[1]) * 1e3 / iters, 2)


def main(M=1024, K=512, N=1024):
    C = ops._ext()
    torch.manual_seed(0)
    G = N // 32
    xs = torch.randn(M, 2560, device="cuda")
    x = xs[:, :K]
    gamma, beta = torch.ones(K, device="cuda"), torch.zeros(K, device="cuda")
    W = torch.randn(N, K, device="cuda") / K ** 0.5
    b = torch.zeros(N, device="cuda")
    u = torch.rand(M * G, device="cuda")
    out = torch.empty(M, N + 16, device="cuda")
    idx = torch.empty(M, G + 2, dtype=torch.int32, device="cuda")
    y = torch.empty(M, K, device="cuda")
    mean, rstd = torch.empty(M, device="cuda"), torch.empty(M, device="cuda")
    logits = torch.empty(M, N, device="cuda")
    act = ops._act_code("silu")

    def fused():
        C.prior_head(x, gamma, beta, 1e-5, act, W, b, u, 0.01, out[:, 16:], idx[:, 2:], 9)

    def three():
        C.ln_act_fwd_into(x, xs.stride(0), y, K, gamma, beta, mean, rstd, M, K, 1, 1e-5, act)
        torch.addmm(b, y, W.t(), out=logits)
        C.unimix_sample_into(logits, u, 32, 0.01, out[:, 16:], idx[:, 2:], 9)

    def gemm():
        torch.addmm(b, y, W.t(), out=logits)

    print(json.dumps({"shape": [M, K, N], "prior_head_us": _time(fused), "three_launch_us": _time(three),
                      "gemm_alone_us": _time(gemm)}))


if __name__ == "__main__":
    main(*[int(v) for v in sys.argv[1:]])
