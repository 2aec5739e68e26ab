"""Player encoder (1 frame, raw uint8, Atari-100k stack): small-batch HIP stack vs the per-layer modules."""
import torch

from sheeprl_prey_amd.algos.dreamer_v3.agent import CNNEncoder
from sheeprl_prey_amd.ops import conv as conv_ops

enc = CNNEncoder(["rgb"], [3], (64, 64), 32, stages=4).cuda()
x = torch.randint(0, 256, (1, 3, 64, 64), device="cuda", dtype=torch.int64).to(torch.uint8)


def timeit(n=200):
    with torch.no_grad():
        for _ in range(20):
            enc({"rgb": x})
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(n):
            enc({"rgb": x})
        e.record()
        torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


for flag in (True, False, True, False):
    conv_ops.SMALL_ENABLED = flag
    print(f"player encoder 1 frame, small stack {'on ' if flag else 'off'}: {timeit():7.1f} us/call (eager, stream-timed)")
