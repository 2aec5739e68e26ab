"""A/B the DreamerV3 Atari-100k CNN encoder + decoder (fwd + bwd, N = B*T = 1024 frames of 3x64x64,
mult 32) in NCHW vs channels-last (NHWC) storage, each replayed from a hipGraph.

    python scripts/conv_bench.py [N]
"""
import sys
import time

import os
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sheeprl_prey_amd.algos.dreamer_v3.agent import CNNDecoder, CNNEncoder
from sheeprl_prey_amd.ops import conv as conv_ops


def run(layout: str, N: int, iters: int = 20):
    torch.manual_seed(0)
    enc = CNNEncoder(["rgb"], [3], (64, 64), 32).cuda()
    dec = CNNDecoder(["rgb"], [3], 32, 1536, enc.output_dim, (64, 64)).cuda()
    cl = layout == "nhwc"
    conv_ops.ENABLED = layout == "fused"
    if cl:
        enc = enc.to(memory_format=torch.channels_last)
        dec = dec.to(memory_format=torch.channels_last)
        enc.channels_last = True
        dec.channels_last = True
    x = torch.rand(N, 3, 64, 64, device="cuda")
    lat = torch.randn(N, 1536, device="cuda", requires_grad=True)
    params = list(enc.parameters()) + list(dec.parameters())

    def step():
        xi = x.contiguous(memory_format=torch.channels_last) if cl else x
        e = enc({"rgb": xi})
        r = dec(lat)["rgb"]
        loss = e.square().mean() + (r - x).square().mean()
        loss.backward()
        return loss

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            for p in params:
                p.grad = None
            step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    for p in params:
        p.grad = None
    with torch.cuda.graph(g):
        step()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        g.replay()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iters * 1e3
    print(f"{layout}: encoder+decoder fwd+bwd N={N}: {dt:.3f} ms", flush=True)
    return dt


if __name__ == "__main__":
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    bm = os.environ.get("CONV_BENCHMARK", "0") == "1"
    torch.backends.cudnn.benchmark = bm
    print("cudnn.benchmark =", bm)
    layouts = os.environ.get("CONV_LAYOUTS", "nchw,fused,nchw,fused").split(",")
    for layout in layouts:
        run(layout, N)
