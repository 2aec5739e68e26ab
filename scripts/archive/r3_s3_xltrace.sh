#!/bin/bash
# Kernel trace of the XL DV3 bench (timed window: categories + top kernels).
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out/trxl
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trxl -o run -- \
  python3 bench.py --xl --steps 4 --warmup 3 --prefill 100 --profile-steps 4 > gpurun_out/trxl_bench.log 2>&1 || { tail -5 gpurun_out/trxl_bench.log; exit 1; }
f=$(find gpurun_out/trxl -name '*kernel_trace.csv' | head -1)
python3 scripts/trace_window.py "$f" 4 45 > gpurun_out/trxl_summary.md
rm -f "$f"
head -60 gpurun_out/trxl_summary.md | cut -c1-160
