"""Event-timed skinny GEMM vs torch.mm on the XL recurrent shapes (env SRL_SKINNY_WGS / SRL_SKINNY_NT
are read once per process: run one process per setting)."""
import os

import torch

from sheeprl_prey_amd import ops

shapes = [(16, 12288, 5120, "Wg fwd"), (16, 5120, 12288, "Wg bwd"), (16, 2048, 4096, "W1 fwd"), (16, 4096, 2048, "W1 bwd"),
          (16, 1024, 1024, "Wz")]
res = []
for M, N, K, name in shapes:
    A = torch.randn(M, K, device="cuda")
    W = torch.randn(N, K, device="cuda")
    out = torch.empty(M, N, device="cuda")
    row = [name]
    for impl in ("skinny", "torch"):
        f = (lambda: ops.skinny_nt(A, W, out)) if impl == "skinny" else (lambda: torch.mm(A, W.t(), out=out))
        for _ in range(5):
            f()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            f()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 50 * 1e3
        row.append(f"{impl} {us:6.1f} us ({N * K * 4 / us / 1e6:5.2f} TB/s)")
    res.append("  ".join(row))
print(f"WGS={os.environ.get('SRL_SKINNY_WGS', 'default')} FUSED={os.environ.get('SRL_SKINNY_FUSED', '1')}:\n  " +
      "\n  ".join(res), flush=True)
