#!/bin/bash
# Kernel trace of the timed bench window only; leaves a markdown summary in gpurun_out/trace_summary.md
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
STEPS=${STEPS:-20}
mkdir -p gpurun_out/trace
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace -o dv3 -- python bench.py --steps $STEPS --warmup 6 --prefill 100 --profile-steps $STEPS $@ > gpurun_out/trace.log 2>&1
rc=$?
tail -1 gpurun_out/trace.log
f=$(find gpurun_out/trace -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python scripts/trace_window.py "$f" $STEPS ${TOP:-45} > gpurun_out/trace_summary.md
[ -n "$f" ] && [ -n "${STEPDUMP:-}" ] && python scripts/trace_step.py "$f" $STEPS > "$STEPDUMP"
rm -f gpurun_out/trace/*kernel_trace.csv
head -3 gpurun_out/trace_summary.md
exit $rc
