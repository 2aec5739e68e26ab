#!/bin/bash
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_buffers_gpu.py tests/test_dreamer_gpu.py tests/test_algos_gpu.py -x -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > gpurun_out/sm_t.log 2>&1 || { grep -E "^FAILED|^E  " gpurun_out/sm_t.log | head -20; tail -5 gpurun_out/sm_t.log; exit 1; }
tail -1 gpurun_out/sm_t.log
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/sm_on.log 2>&1 && echo "fused sample on  $(tail -1 gpurun_out/sm_on.log | cut -c60-130)" || { tail -20 gpurun_out/sm_on.log; exit 1; }
  SRL_FUSED_SAMPLE=0 timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/sm_off.log 2>&1 && echo "fused sample off $(tail -1 gpurun_out/sm_off.log | cut -c60-130)" || exit 1
done
TOP=90 bash scripts/trace_both.sh > gpurun_out/s3_trace.log 2>&1 || { tail -20 gpurun_out/s3_trace.log; exit 1; }
head -3 gpurun_out/tr2_summary.md
awk -F'\t' '$4 ~ /to_nhwc4_kernel<unsigned/ {print "encoder start at", $2, "us; kernel index", $1}' gpurun_out/tr2_step.tsv
