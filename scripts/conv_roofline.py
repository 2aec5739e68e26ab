"""Per-launch roofline of the DreamerV3 Atari-100k CNN stack (encoder + decoder, forward + backward, N = 1024
frames of 3x64x64, channel multiplier 32), as the train step runs it: the fused stack (ops/conv.py) captured in a
hipGraph and replayed.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/convroof -o conv -- python scripts/conv_roofline.py
    python scripts/conv_roofline.py --csv <kernel_trace.csv> [--iters 10]

Run mode replays the graph ``--iters`` times after a marker kernel; report mode takes the launches after the marker,
splits them into iterations, and prints one row per launch (position-wise median over the iterations): kernel,
grid, microseconds, and - for the GEMM-shaped launches it can attribute - the layer, its FLOPs, TF/s and the
fraction of the fp32 MFMA peak (157.3 TF/s: 256 CUs x 256 FLOP/clk x 2.4 GHz)."""
import argparse
import collections
import csv
import os
import statistics
import sys

PEAK_TF = 157.3
N = 1024
MULT = 32  # --mult: the channel multiplier (32 = Atari-100k, 96 = XL)


def layer_flops():
    """FLOPs of every conv GEMM of the stack (k4 s2 p1; 2 * M * N * K)."""
    out = {}
    m = MULT
    enc = [(3, m, 32), (m, 2 * m, 16), (2 * m, 4 * m, 8), (4 * m, 8 * m, 4)]  # (cin, cout, output side)
    for i, (ci, co, s) in enumerate(enc):
        cip = max(ci, 4)
        out[f"E{i + 1} fwd"] = 2 * N * s * s * co * cip * 16
        out[f"E{i + 1} wgrad"] = out[f"E{i + 1} fwd"]
        if i > 0:
            out[f"E{i + 1} dgrad"] = 2 * N * s * s * co * ci * 16
    dec = [(8 * m, 4 * m, 8), (4 * m, 2 * m, 16), (2 * m, m, 32), (m, 3, 64)]
    for i, (ci, co, s) in enumerate(dec):
        out[f"D{i + 1} fwd"] = 2 * N * s * s * co * ci * 4  # UP: K = 4 taps x Ca per parity class
        out[f"D{i + 1} wgrad"] = out[f"D{i + 1} fwd"]
        out[f"D{i + 1} dgrad"] = out[f"D{i + 1} fwd"]
    return out


def run(iters: int) -> None:
    import torch

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from sheeprl_prey_amd.algos.dreamer_v3.agent import CNNDecoder, CNNEncoder

    torch.manual_seed(0)
    enc = CNNEncoder(["rgb"], [3], (64, 64), MULT).cuda()
    dec = CNNDecoder(["rgb"], [3], MULT, 1536, enc.output_dim, (64, 64)).cuda()
    x = torch.randint(0, 255, (N, 3, 64, 64), dtype=torch.uint8, device="cuda")
    lat = torch.randn(N, 1536, device="cuda", requires_grad=True)
    g_e = torch.randn(N, enc.output_dim, device="cuda")
    g_d = torch.randn(N, 3, 64, 64, device="cuda")
    params = list(enc.parameters()) + list(dec.parameters())

    def step():
        e = enc({"rgb": x})
        r = dec(lat)["rgb"]
        ((e * g_e).sum() + (r * g_d).sum()).backward()

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
    torch.cuda._sleep(1000)  # marker
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(iters):
        g.replay()
        torch.cuda.synchronize()
    ev[1].record()
    torch.cuda.synchronize()
    print(f"stack fwd+bwd replay: {ev[0].elapsed_time(ev[1]) / iters:.3f} ms/iter (synced per iter)", flush=True)


def short(name: str) -> str:
    name = name.replace("srl::conv::", "").replace("(anonymous namespace)::", "")
    return name[:90]


def report(path: str, iters: int) -> None:
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = max(i for i, r in enumerate(rows) if "sleep" in r["Kernel_Name"].lower() or "spin" in r["Kernel_Name"].lower())
    win = rows[idx + 1:]
    per = len(win) // iters
    gkey = next((k for k in ("Grid_Size", "Grid_Size_X", "grid_size") if k in win[0]), None)
    its = [win[i * per:(i + 1) * per] for i in range(iters)]
    print(f"{per} launches per iteration, {iters} iterations\n")
    print("| # | kernel | grid | us (median) |\n|---:|---|---:|---:|")
    tot = 0.0
    by = collections.defaultdict(float)
    for j in range(per):
        ds = [(int(it[j]["End_Timestamp"]) - int(it[j]["Start_Timestamp"])) / 1e3 for it in its]
        d = statistics.median(ds)
        tot += d
        nm = its[0][j]["Kernel_Name"]
        by[short(nm).split("(")[0].split("<")[0]] += d
        print(f"| {j} | `{short(nm)}` | {its[0][j].get(gkey, '')} | {d:.1f} |")
    print(f"\nsum of launches: {tot / 1e3:.3f} ms per fwd+bwd\n")
    print("| kernel family | us |\n|---|---:|")
    for k, v in sorted(by.items(), key=lambda kv: -kv[1]):
        print(f"| `{k}` | {v:.1f} |")
    fl = layer_flops()
    print(f"\nlayer FLOPs (GF): " + ", ".join(f"{k} {v / 1e9:.1f}" for k, v in fl.items()))
    print(f"total {sum(fl.values()) / 1e9:.1f} GF; at {tot / 1e3:.3f} ms = {sum(fl.values()) / tot / 1e6:.1f} TF/s "
          f"({100 * sum(fl.values()) / tot / 1e6 / PEAK_TF:.0f} % of the fp32 MFMA peak)")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--csv", default=None)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--mult", type=int, default=32)
    a = ap.parse_args()
    MULT = a.mult
    if a.csv:
        report(a.csv, a.iters)
    else:
        run(a.iters)
