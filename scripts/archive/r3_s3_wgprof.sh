#!/bin/bash
# Kernel-level stats of the wgrad timing script (rocprofv3 kernel trace).
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
rm -rf gpurun_out/wgprof
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wgprof -o wg -- python3 scripts/wgrad_timing.py > gpurun_out/wgprof.log 2>&1 || { tail -20 gpurun_out/wgprof.log; exit 1; }
grep -v amdgpu.ids gpurun_out/wgprof.log
f=$(find gpurun_out/wgprof -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print(f'{float(r["AverageNs"])/1e3:9.1f} us avg  {int(r["Calls"]):5d} calls  {r["Name"][:110]}')
PY
find gpurun_out/wgprof -name '*kernel_trace.csv' -delete
