"""Aggregate a rocprofv3 kernel-trace CSV over the timed window only (after the last marker
kernel launched by ``bench.py --profile-steps``), dropping MIOpen find/tuning noise from warm-up.

usage: python scripts/trace_window.py <kernel_trace.csv> <timed_steps> [top]"""
import collections
import csv
import sys


CATS = [
    ("rssm scan (persistent)", ["scanp::"]),
    ("conv (srl igemm/wgrad)", ["srl::conv::"]),
    ("library GEMM (hipBLASLt/rocBLAS)", ["Cijk_", "gemm"]),
    ("layernorm / LN-GRU", ["ln_wave", "ln_gru", "layer_norm"]),
    ("ATen elementwise / reduce / copy", ["at::native", "__amd_rocclr", "zero2_kernel"]),
    ("srl other", ["srl::"]),
]


def main(path, steps, top=40):
    rows = list(csv.DictReader(open(path)))
    key_s, key_e = "Start_Timestamp", "End_Timestamp"
    rows.sort(key=lambda r: int(r[key_s]))
    idx = max(i for i, r in enumerate(rows) if "sleep" in r["Kernel_Name"].lower() or "spin" in r["Kernel_Name"].lower())
    win = rows[idx + 1 :]
    t0, t1 = int(win[0][key_s]), int(win[-1][key_e])
    agg = collections.defaultdict(lambda: [0, 0])
    for r in win:
        d = int(r[key_e]) - int(r[key_s])
        a = agg[r["Kernel_Name"]]
        a[0] += d
        a[1] += 1
    busy = sum(a[0] for a in agg.values())
    n = sum(a[1] for a in agg.values())
    # union of the kernel intervals: wall - union = time with NO kernel running (launch gaps, host waits)
    iv = sorted((int(r[key_s]), int(r[key_e])) for r in win)
    union, cs, ce = 0, iv[0][0], iv[0][1]
    for s_, e_ in iv[1:]:
        if s_ > ce:
            union += ce - cs
            cs, ce = s_, e_
        else:
            ce = max(ce, e_)
    union += ce - cs
    print(f"timed window: {steps} steps, wall {(t1 - t0) / 1e6:.2f} ms ({(t1 - t0) / 1e6 / steps:.2f} ms/step), "
          f"kernel busy {busy / 1e6:.2f} ms ({busy / 1e6 / steps:.2f} ms/step), {n / steps:.0f} dispatches/step, "
          f"GPU occupied (union) {union / 1e6 / steps:.2f} ms/step, idle {(t1 - t0 - union) / 1e6 / steps:.2f} ms/step\n")
    cats = collections.defaultdict(lambda: [0, 0])
    for name, (d, c) in agg.items():
        cat = next((k for k, pat in CATS if any(p in name for p in pat)), "other")
        cats[cat][0] += d
        cats[cat][1] += c
    print("| category | ms/step | calls/step |\n|---|---:|---:|")
    for k, (d, c) in sorted(cats.items(), key=lambda kv: -kv[1][0]):
        print(f"| {k} | {d / 1e6 / steps:.3f} | {c / steps:.1f} |")
    print()
    print("| ms/step | calls/step | avg us | % busy | kernel |\n|---:|---:|---:|---:|---|")
    for name, (d, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
        print(f"| {d / 1e6 / steps:.3f} | {c / steps:.1f} | {d / c / 1e3:.1f} | {100 * d / busy:.1f} | `{_short(name)}` |")
    import os

    for pat in filter(None, os.environ.get("TRACE_BY_GRID", "").split(",")):
        by_grid(win, steps, pat)


def by_grid(win, steps, pat):
    """Per (kernel, grid size) breakdown of the kernels whose name contains ``pat`` (TRACE_BY_GRID=pat)."""
    import collections

    gkey = next((k for k in ("Grid_Size", "Grid_Size_X", "grid_size") if k in win[0]), None)
    if gkey is None:
        return
    agg = collections.defaultdict(lambda: [0, 0])
    for r in win:
        if pat in r["Kernel_Name"]:
            a = agg[(r["Kernel_Name"], r[gkey], r.get("Workgroup_Size", r.get("Workgroup_Size_X", "")))]
            a[0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            a[1] += 1
    print(f"\n| ms/step | calls/step | avg us | grid | wg | kernel (by grid: {pat}) |\n|---:|---:|---:|---:|---:|---|")
    for (name, g, w), (d, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:40]:
        print(f"| {d / 1e6 / steps:.3f} | {c / steps:.1f} | {d / c / 1e3:.1f} | {g} | {w} | `{_short(name)}` |")


def _short(name: str) -> str:
    """First 95 characters; ATen kernels also name their functor / op (templated names share the prefix)."""
    if "at::native" not in name or len(name) <= 95:
        return name[:95]
    import re

    ops = []
    for m in re.findall(r"(\w*(?:Functor|functor|_kernel_cuda|_kernel_impl|copy_kernel|Op)\w*)", name):
        if m not in ops and not m.startswith("gpu_kernel"):
            ops.append(m)
    return name[:60] + " .. " + ",".join(ops[:3])


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]) if len(sys.argv) > 3 else 40)
