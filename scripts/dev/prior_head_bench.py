"""prior_head.hip forms at the imagination shapes: us per launch (events, median of 50) and sample agreement."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from sheeprl_prey_amd import ops  # noqa: E402


def main():
    C = ops._ext()
    torch.manual_seed(0)
    for M, K, N in ((1024, 512, 1024), (1024, 1024, 1024), (1024, 256, 1024)):
        G = N // 32
        xs = torch.randn(M, K + 2560, device="cuda")
        x = xs[:, :K]
        gamma, beta = 1 + 0.1 * torch.randn(K, device="cuda"), 0.1 * torch.randn(K, device="cuda")
        W, b = torch.randn(N, K, device="cuda") / K ** 0.5, 0.1 * torch.randn(N, device="cuda")
        u = torch.rand(M * G, device="cuda")
        outs = []
        for form in ((0, 1) if hasattr(C, "set_prior_head_form") else (0,)):  # the 32-row form was not kept
            if form:
                C.set_prior_head_form(form)
        
            out = torch.empty(M, N, device="cuda")
            idx = torch.empty(M, G, dtype=torch.int32, device="cuda")
            for _ in range(5):
                C.prior_head(x, gamma, beta, 1e-3, ops._act_code("silu"), W, b, u, 0.01, out, idx, 0)
            torch.cuda.synchronize()
            ts = []
            for _ in range(50):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                C.prior_head(x, gamma, beta, 1e-3, ops._act_code("silu"), W, b, u, 0.01, out, idx, 0)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            outs.append(out.clone())
            print(f"M {M} K {K} N {N} form {form}: {np.median(ts):6.1f} us", flush=True)
        if len(outs) > 1:
            C.set_prior_head_form(0)
            print(f"  samples identical: {torch.equal(outs[0], outs[1])}", flush=True)


if __name__ == "__main__":
    main()
