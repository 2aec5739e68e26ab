"""Timing of the one-hot gather first layer (ops/csrc/onehot.hip) at the rollout-wide shapes of the DV3 actor /
critic phase (M = 16 x 1024 rows, N = 512, 32 categoricals of 32 over K = 1024 table rows, dense part Y given).

    python scripts/dev/onehot_gather_bench.py [M] [N]      (run under rocprofv3 --kernel-trace --stats)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from sheeprl_prey_amd import ops  # noqa: E402


def main(M=16384, N=512, G=32, C=32):
    ext = ops._ext()
    torch.manual_seed(0)
    K = G * C
    idx = (torch.randint(0, C, (M, G), device="cuda") + torch.arange(G, device="cuda") * C).int()
    T = torch.randn(K, N, device="cuda")
    Y = torch.randn(M, N, device="cuda")
    bias, g, b = torch.randn(N, device="cuda"), torch.rand(N, device="cuda") + 0.5, torch.randn(N, device="cuda")
    z, y = torch.empty(M, N, device="cuda"), torch.empty(M, N, device="cuda")
    mean, rstd = torch.empty(M, device="cuda"), torch.empty(M, device="cuda")
    err = torch.zeros(1, dtype=torch.int32, device="cuda")
    act = ops._act_code("silu")

    def run():
        assert ext.onehot_gather_ln(Y, idx, G, 0, T, bias, g, b, 1e-3, act, True, z, y, mean, rstd, err)

    for _ in range(5):
        run()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(50):
        run()
    ev[1].record()
    torch.cuda.synchronize()
    # fp64 check of a few rows
    rows = torch.arange(0, M, max(1, M // 64), device="cuda")
    zr = Y[rows].double() + bias.double() + T.double()[idx[rows].long()].sum(1)
    ln = torch.nn.functional.layer_norm(zr, (N,), g.double(), b.double(), 1e-3)
    ref = torch.nn.functional.silu(ln)
    print(json.dumps({"M": M, "N": N, "us": round(ev[0].elapsed_time(ev[1]) * 1e3 / 50, 2),
                      "max_err": float((y[rows].double() - ref).abs().max()), "err_word": int(err.item())}))


if __name__ == "__main__":
    main(*[int(v) for v in sys.argv[1:]])
