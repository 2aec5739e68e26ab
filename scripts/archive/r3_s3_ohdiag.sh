#!/bin/bash
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
for m in 0 1 2; do SRL_WGRAD_OH_MODE=$m timeout -k 10 60 python scripts/wg_oh_diag.py 2>&1 | grep -v amdgpu.ids || exit 1; done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/ohprof -o oh -- python3 scripts/wg_oh_diag.py > gpurun_out/ohprof.log 2>&1 || exit 1
f=$(find gpurun_out/ohprof -name '*kernel_stats.csv' | head -1); cut -d, -f1-8 "$f" | head -8
find gpurun_out/ohprof -name '*kernel_trace.csv' -delete
