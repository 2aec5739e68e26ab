import os, torch
from sheeprl_prey_amd import ops
from scripts.wgrad_timing import timeit
M, N, G, Cc = 16384, 512, 32, 32
k = torch.randint(0, Cc, (M, G), device="cuda")
idx = (k + torch.arange(G, device="cuda") * Cc).int()
dz = torch.randn(M, N, device="cuda")
print(os.environ.get("SRL_WGRAD_OH_MODE"), timeit(lambda: ops.wgrad(dz, None, onehot=(idx, G, 0, G * Cc))))
