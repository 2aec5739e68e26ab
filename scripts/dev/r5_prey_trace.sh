#!/bin/bash
# kernel trace of the prey train step (B16 x T64, captured)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ptrace
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ptrace -o prey -- python3 scripts/dv3_step_bench.py exp=dreamer_v3_prey --vector 14 --actions 100 --steps 10 --marker > gpurun_out/ptrace/prey.log 2>&1 || { tail -20 gpurun_out/ptrace/prey.log; exit 1; }
tail -1 gpurun_out/ptrace/prey.log
f=$(find gpurun_out/ptrace -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_window.py "$f" 10 45 > gpurun_out/ptrace/summary.md
rm -f gpurun_out/ptrace/*kernel_trace.csv
head -50 gpurun_out/ptrace/summary.md
