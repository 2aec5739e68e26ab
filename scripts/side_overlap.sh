#!/bin/bash
# Kernel trace of the DV3 bench with side-stream decoder weight gradients; overlap with the scan bwd.
export TMPDIR=/tmp
mkdir -p gpurun_out/ovl
SRL_SIDE_WGRAD=${SIDE:-1} timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ovl -o dv3 -- python bench.py --steps 10 --warmup 6 --prefill 100 --profile-steps 10 > gpurun_out/ovl.log 2>&1
rc=$?
f=$(find gpurun_out/ovl -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python scripts/overlap_check.py "$f" > gpurun_out/overlap.txt
rm -f gpurun_out/ovl/*kernel_trace.csv
cat gpurun_out/overlap.txt
exit $rc
