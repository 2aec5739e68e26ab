#!/bin/bash
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_dreamer_gpu.py tests/test_graphs_gpu.py tests/test_algos_gpu.py -x -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > gpurun_out/pl_t.log 2>&1 || { grep -E "^FAILED|^E  " gpurun_out/pl_t.log | head -20; tail -5 gpurun_out/pl_t.log; exit 1; }
tail -1 gpurun_out/pl_t.log
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/pl_on.log 2>&1 && echo "bench $(tail -1 gpurun_out/pl_on.log | cut -c60-130)" || { tail -20 gpurun_out/pl_on.log; exit 1; }
done
TOP=90 bash scripts/trace_both.sh > gpurun_out/s3_trace.log 2>&1 || { tail -20 gpurun_out/s3_trace.log; exit 1; }
head -3 gpurun_out/tr2_summary.md
awk -F'\t' '$4 ~ /to_nhwc4_kernel<unsigned/ {print "encoder start at", $2, "us; kernel index", $1}' gpurun_out/tr2_step.tsv
