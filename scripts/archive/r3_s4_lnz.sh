#!/bin/bash
# LN backward zeroing its dgamma/dbeta targets in-kernel (no zero2 launch): LN / ops / dreamer tests, bench, trace
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_wgrad_gpu.py tests/test_ops_gpu.py tests/test_dreamer_gpu.py tests/test_graphs_gpu.py \
  tests/test_onehot_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/lnz_t.log 2>&1 \
  || { grep -E "FAILED|Error|error|assert" gpurun_out/lnz_t.log | head -20; tail -5 gpurun_out/lnz_t.log; exit 1; }
tail -1 gpurun_out/lnz_t.log
for i in 1 2; do
  timeout -k 10 300 python bench.py > gpurun_out/lnz_dv3_$i.log 2>&1 && tail -1 gpurun_out/lnz_dv3_$i.log | cut -c1-140 || { tail -20 gpurun_out/lnz_dv3_$i.log; exit 1; }
done
TOP=90 bash scripts/trace_both.sh > gpurun_out/lnz_trace.log 2>&1 || { tail -20 gpurun_out/lnz_trace.log; exit 1; }
head -3 gpurun_out/tr2_summary.md
grep -E "zero2|colsum2" gpurun_out/tr2_summary.md | cut -c1-120
