#!/bin/bash
# wgrad kernels: numerics tests, per-call timing, DV3-path GPU tests, DV3 bench x2.
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_wgrad_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/wg_t.log 2>&1 || { tail -30 gpurun_out/wg_t.log; exit 1; }
tail -2 gpurun_out/wg_t.log
timeout -k 10 120 python -u scripts/wgrad_timing.py > gpurun_out/wg_timing.txt 2>&1 || { tail -20 gpurun_out/wg_timing.txt; exit 1; }
cat gpurun_out/wg_timing.txt
timeout -k 10 400 python -u -m pytest tests/test_onehot_gpu.py tests/test_dreamer_gpu.py tests/test_ops_gpu.py -x -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > gpurun_out/wg_t2.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/wg_t2.log | head -20; tail -5 gpurun_out/wg_t2.log; exit 1; }
tail -2 gpurun_out/wg_t2.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/wg_dv3_$i.log 2>&1 && tail -1 gpurun_out/wg_dv3_$i.log | cut -c1-140 || { tail -20 gpurun_out/wg_dv3_$i.log; exit 1; }
done
