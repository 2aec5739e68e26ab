#!/bin/bash
# batched weight transposes + one LN-partial column sum in the scan backward: tests, bench A/B vs HEAD~ numbers, trace
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_transpose_gpu.py tests/test_dreamer_gpu.py tests/test_onehot_gpu.py tests/test_graphs_gpu.py \
  tests/test_imagine_cont_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/tr_t.log 2>&1 \
  || { grep -E "FAILED|Error|error|assert" gpurun_out/tr_t.log | head -20; tail -5 gpurun_out/tr_t.log; exit 1; }
tail -1 gpurun_out/tr_t.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/tr_dv3_$i.log 2>&1 && tail -1 gpurun_out/tr_dv3_$i.log | cut -c1-140 || { tail -20 gpurun_out/tr_dv3_$i.log; exit 1; }
done
TOP=90 bash scripts/trace_both.sh > gpurun_out/tr_trace.log 2>&1 || { tail -20 gpurun_out/tr_trace.log; exit 1; }
head -12 gpurun_out/tr2_summary.md
grep -E "transpose|manual_unroll|reduce_kernel|copyBuffer" gpurun_out/tr2_summary.md | cut -c1-150 | head -12
