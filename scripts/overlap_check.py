"""How much of the decoder weight-gradient work overlaps the persistent scan backward in a rocprofv3
kernel trace (timed window of bench.py --profile-steps): per scan-bwd launch, the wgrad kernel time
inside its [start, end] interval.

usage: python scripts/overlap_check.py <kernel_trace.csv>"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
scans = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if "scanp::bwd_kernel" in r["Kernel_Name"]]
wg = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]) for r in rows
      if "wgrad" in r["Kernel_Name"] and "srl::conv" in r["Kernel_Name"]]
tot_in = tot = 0
for s0, s1 in scans[-10:]:
    near = [(a, b, n) for a, b, n in wg if a < s1 + 3_000_000 and b > s0 - 3_000_000]
    inside = sum(max(0, min(b, s1) - max(a, s0)) for a, b, _ in near)
    allt = sum(b - a for a, b, _ in near)
    tot_in += inside
    tot += allt
    first = min((a for a, _, _ in near), default=0)
    print(f"scan bwd {(s1 - s0) / 1e3:8.1f} us | wgrad near {allt / 1e3:8.1f} us, inside the scan {inside / 1e3:8.1f} us"
          f" | first wgrad starts {(first - s0) / 1e3:+8.1f} us after the scan start")
print(f"overlapped fraction of wgrad time: {tot_in / max(tot, 1):.2f}")
