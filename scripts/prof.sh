#!/bin/bash
# Parameterised kernel trace of a bench variant's timed window (replaces the per-session one-off scripts
# under scripts/archive/).  usage: bash scripts/prof.sh NAME STEPS [bench.py args...]
# -> gpurun_out/NAME_summary.md (per-category + top-kernel table, scripts/trace_window.py) and NAME.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=$PWD
NAME=$1; STEPS=$2; shift 2
mkdir -p gpurun_out/tr_$NAME
timeout -k 10 ${TLIM:-600} rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr_$NAME -o run -- \
  python3 bench.py --steps $STEPS --warmup ${WARM:-4} --profile-steps $STEPS "$@" > gpurun_out/$NAME.log 2>&1
rc=$?
tail -1 gpurun_out/$NAME.log | cut -c1-400
f=$(find gpurun_out/tr_$NAME -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python3 scripts/trace_window.py "$f" $STEPS ${TOP:-120} > gpurun_out/${NAME}_summary.md
rm -rf gpurun_out/tr_$NAME
[ -f gpurun_out/${NAME}_summary.md ] && head -12 gpurun_out/${NAME}_summary.md
exit $rc
