#!/bin/bash
# autograd Functions without materialized zero grads: GPU tests of every touched op family, bench, trace
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_dreamer_gpu.py tests/test_ops_gpu.py tests/test_graphs_gpu.py tests/test_sac_gpu.py \
  tests/test_lstm_gpu.py tests/test_dv3_loss_kernels_gpu.py tests/test_algos_gpu.py tests/test_imagine_cont_gpu.py -x -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > gpurun_out/mat_t.log 2>&1 \
  || { grep -E "FAILED|Error|error|assert" gpurun_out/mat_t.log | head -20; tail -5 gpurun_out/mat_t.log; exit 1; }
tail -1 gpurun_out/mat_t.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/mat_dv3_$i.log 2>&1 && tail -1 gpurun_out/mat_dv3_$i.log | cut -c1-140 || { tail -20 gpurun_out/mat_dv3_$i.log; exit 1; }
done
TOP=90 bash scripts/trace_both.sh > gpurun_out/mat_trace.log 2>&1 || { tail -20 gpurun_out/mat_trace.log; exit 1; }
head -12 gpurun_out/tr2_summary.md
grep -E "Fill" gpurun_out/tr2_summary.md | cut -c1-150 | head -5
