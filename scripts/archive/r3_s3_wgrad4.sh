#!/bin/bash
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_wgrad_gpu.py tests/test_onehot_gpu.py tests/test_dreamer_gpu.py tests/test_ops_gpu.py tests/test_graphs_gpu.py -x -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > gpurun_out/wg_t2.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/wg_t2.log | head -20; tail -5 gpurun_out/wg_t2.log; exit 1; }
tail -2 gpurun_out/wg_t2.log
bash scripts/r3_s3_wgprof.sh 2>&1 | grep -E "^ +[0-9.]+ us avg" | head -8
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/wg_dv3_$i.log 2>&1 && tail -1 gpurun_out/wg_dv3_$i.log | cut -c1-140 || { tail -20 gpurun_out/wg_dv3_$i.log; exit 1; }
done
SRL_WGRAD_MIN_ROWS=0 timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/wg_dv3_off.log 2>&1 && tail -1 gpurun_out/wg_dv3_off.log | cut -c1-140 || exit 1
TOP=90 bash scripts/trace_both.sh > gpurun_out/s3_trace.log 2>&1 || { tail -20 gpurun_out/s3_trace.log; exit 1; }
head -12 gpurun_out/tr2_summary.md
