#!/bin/bash
# DreamerV3 prey preset train step (exp=dreamer_v3_prey: dense 1024, deter 256, vector obs, Discrete(100)): time + kernel stats
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out/prey_prof
timeout -k 10 300 python -u scripts/dv3_step_bench.py exp=dreamer_v3_prey --vector 14 --actions 100 --steps 20 > gpurun_out/prey_step.log 2>&1 && tail -1 gpurun_out/prey_step.log || { tail -20 gpurun_out/prey_step.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prey_prof -o run -- python3 scripts/dv3_step_bench.py exp=dreamer_v3_prey --vector 14 --actions 100 --steps 20 > gpurun_out/prey_prof.log 2>&1 || { tail -20 gpurun_out/prey_prof.log; exit 1; }
f=$(find gpurun_out/prey_prof -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY' > gpurun_out/prey_kernel_stats.md
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot/1e6:.1f} ms over the run (24 train steps + capture)\n")
print("| % | calls | avg us | kernel |\n|---:|---:|---:|---|")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:45]:
    print(f"| {100*float(r['TotalDurationNs'])/tot:.1f} | {r['Calls']} | {float(r['AverageNs'])/1e3:.1f} | `{r['Name'][:100]}` |")
PY
find gpurun_out/prey_prof -name '*.csv' ! -name '*kernel_stats.csv' -delete
head -30 gpurun_out/prey_kernel_stats.md
