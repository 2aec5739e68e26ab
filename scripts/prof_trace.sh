#!/bin/bash
# Kernel trace of the timed bench window: rocprofv3 --kernel-trace, then aggregate the dispatches
# after bench.py's marker kernel (scripts/trace_window.py).  Usage: STEPS=10 bash scripts/prof_trace.sh [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/trace
STEPS=${STEPS:-10}
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace -o run -- \
  python3 bench.py --steps $STEPS --warmup 4 --profile-steps $STEPS "$@" > gpurun_out/trace_bench.log 2>&1 || exit $?
f=$(find gpurun_out/trace -name '*kernel_trace.csv' | head -1)
python3 scripts/trace_window.py "$f" $STEPS ${TOP:-60} > gpurun_out/trace_summary.md
rm -f "$f"
head -70 gpurun_out/trace_summary.md
