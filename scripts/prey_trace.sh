#!/bin/bash
# Kernel trace of the prey preset's captured train step (exp=dreamer_v3_prey, vector 14, Discrete(100)):
# rocprofv3 --kernel-trace over scripts/dv3_step_bench.py --marker, summarised by scripts/trace_window.py
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
STEPS=${STEPS:-10}
mkdir -p gpurun_out/preytrace
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/preytrace -o prey -- python3 scripts/dv3_step_bench.py exp=dreamer_v3_prey --vector 14 --actions 100 --steps $STEPS --marker > gpurun_out/prey_trace.log 2>&1 || { tail -20 gpurun_out/prey_trace.log; exit 1; }
f=$(find gpurun_out/preytrace -name '*kernel_trace.csv' | head -1)
python3 scripts/trace_window.py "$f" $STEPS ${TOP:-50} > gpurun_out/prey_trace_summary.md
rm -f "$f"
tail -1 gpurun_out/prey_trace.log; head -14 gpurun_out/prey_trace_summary.md
