"""Kernel-level timing of the DV3 wgrad shapes (run under rocprofv3 per knob setting)."""
import torch
from sheeprl_prey_amd import ops
from scripts.wgrad_timing import timeit

M, N, K = 16384, 512, 512
dz = torch.randn(M, N, device="cuda")
x = torch.randn(M, K, device="cuda")
k = torch.randint(0, 32, (M, 32), device="cuda")
idx = (k + torch.arange(32, device="cuda") * 32).int()
for _ in range(3):
    timeit(lambda: ops.wgrad(dz, x, bias=True))
    timeit(lambda: ops.wgrad(dz, None, onehot=(idx, 32, 0, 1024)))
