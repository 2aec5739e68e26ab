"""Per-call timing of the tall-layer weight-gradient kernels (ops.wgrad) vs the library GEMM (+ colsum) and of
the LayerNorm backward, at the DreamerV3 imagination-head shapes.  usage: python scripts/wgrad_timing.py"""
import torch

from sheeprl_prey_amd import ops


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    C = ops._ext()
    dev = "cuda"
    for (M, N, K) in [(16384, 512, 512), (15360, 255, 512), (16384, 9, 512), (16384, 512, 1536)]:
        dz = torch.randn(M, N, device=dev)
        xb = torch.randn(M, K + 9, device=dev)
        x = xb[:, 9:]
        lib = timeit(lambda: (dz.t().mm(x), C.colsum(dz)))
        ours = timeit(lambda: ops.wgrad(dz, x, bias=True))
        fl = 2.0 * M * N * K
        print(f"dense  M={M} N={N} K={K}: library+colsum {lib:7.1f} us ({fl / lib / 1e6:6.1f} TF/s)   "
              f"wgrad {ours:7.1f} us ({fl / ours / 1e6:6.1f} TF/s)")
    M, N, G, Cc, Kd = 16384, 512, 32, 32, 512
    k = torch.randint(0, Cc, (M, G), device=dev)
    z = torch.nn.functional.one_hot(k, Cc).float().view(M, G * Cc)
    h = torch.randn(M, Kd, device=dev)
    x = torch.cat((z, h), 1)
    idx = (k + torch.arange(G, device=dev) * Cc).int()
    dz = torch.randn(M, N, device=dev)
    lib = timeit(lambda: (dz.t().mm(x), C.colsum(dz)))
    ours = timeit(lambda: ops.wgrad(dz, h, onehot=(idx, G, 0, G * Cc), bias=True))
    oh_only = timeit(lambda: ops.wgrad(dz, None, onehot=(idx, G, 0, G * Cc)))
    print(f"onehot M={M} N={N} [1024 one-hot | 512]: library dense+colsum {lib:7.1f} us   wgrad {ours:7.1f} us "
          f"(one-hot part alone {oh_only:6.1f} us)")
    for (M, N) in [(16384, 512), (15360, 512), (1024, 512)]:
        xx = torch.randn(M, N, device=dev)
        w = torch.randn(N, device=dev)
        b = torch.randn(N, device=dev)
        y, mean, rstd = C.ln_act_fwd(xx, w, b, 1e-3, ops._act_code("silu"))
        dy = torch.randn(M, N, device=dev)
        t = timeit(lambda: C.ln_act_bwd(xx, dy, w, b, mean, rstd, ops._act_code("silu")))
        print(f"ln_act_bwd M={M} N={N}: {t:6.1f} us (incl. dgamma/dbeta reduction)")


if __name__ == "__main__":
    main()
