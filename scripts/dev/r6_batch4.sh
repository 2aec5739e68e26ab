#!/bin/bash
# Round-6 batch 4: XL conv roofline, XL bench, XL kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONPATH=. TMPDIR=/tmp
mkdir -p gpurun_out
MULT=96 bash scripts/conv_roofline.sh > gpurun_out/b4_roof.txt 2>&1; cp gpurun_out/conv_roofline.md gpurun_out/b4_conv_roofline_xl.md; tail -3 gpurun_out/b4_roof.txt
timeout -k 10 600 python -u bench.py --xl --steps 10 --warmup 4 > gpurun_out/b4_xl.log 2>&1 && tail -1 gpurun_out/b4_xl.log | cut -c1-150 || exit 1
STEPS=5 bash scripts/gpu_trace.sh --xl > /dev/null 2>&1 && cp gpurun_out/trace_summary.md gpurun_out/b4_xl_trace.md && head -14 gpurun_out/b4_xl_trace.md
