#!/bin/bash
# wgrad kernels: numerics tests + per-call timing only.
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_wgrad_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/wg_t.log 2>&1 || { tail -30 gpurun_out/wg_t.log; exit 1; }
tail -2 gpurun_out/wg_t.log
timeout -k 10 120 python -u scripts/wgrad_timing.py > gpurun_out/wg_timing.txt 2>&1 || { tail -20 gpurun_out/wg_timing.txt; exit 1; }
cat gpurun_out/wg_timing.txt
