"""Probe fp32 GEMM rates at the XL head shapes: torch.mm layouts vs ops.wgrad (diagnostic)."""
import torch
from sheeprl_prey_amd import ops
from scripts.wgrad_timing import timeit

M = 16384
for (K, N) in [(1024, 1024), (4096, 1024), (1024, 255)]:
    a = torch.randn(M, K, device="cuda")
    w = torch.randn(N, K, device="cuda")
    fl = 2.0 * M * N * K
    t1 = timeit(lambda: a.mm(w.t()))
    g = torch.randn(M, N, device="cuda")
    t2 = timeit(lambda: g.mm(w))
    t3 = timeit(lambda: g.t().mm(a))
    t4 = timeit(lambda: ops.wgrad(g, a, bias=True))
    print(f"M={M} K={K} N={N}: fwd x W^T {t1:7.1f} us ({fl/t1/1e6:5.1f} TF/s)  dX {t2:7.1f} ({fl/t2/1e6:5.1f})  "
          f"dW lib {t3:7.1f} ({fl/t3/1e6:5.1f})  dW wgrad {t4:7.1f} ({fl/t4/1e6:5.1f})", flush=True)
