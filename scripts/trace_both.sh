#!/bin/bash
# Kernel trace of the DV3 bench: per-kernel summary of the timed window + the kernel sequence of one step.
export TMPDIR=/tmp
mkdir -p gpurun_out/tr2
STEPS=${STEPS:-10}
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr2 -o run -- \
  python3 bench.py --steps $STEPS --warmup 4 --prefill 100 --profile-steps $STEPS > gpurun_out/tr2_bench.log 2>&1 || exit $?
f=$(find gpurun_out/tr2 -name '*kernel_trace.csv' | head -1)
python3 scripts/trace_window.py "$f" $STEPS ${TOP:-70} > gpurun_out/tr2_summary.md
python3 scripts/trace_step.py "$f" $STEPS > gpurun_out/tr2_step.tsv
rm -f "$f"
head -16 gpurun_out/tr2_summary.md
