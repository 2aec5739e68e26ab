#!/bin/bash
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  > gpurun_out/up_t.log 2>&1 || { grep -E "^FAILED|^E  " gpurun_out/up_t.log | head -20; tail -5 gpurun_out/up_t.log; exit 1; }
tail -1 gpurun_out/up_t.log
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/up_on.log 2>&1 && echo "up2 $(tail -1 gpurun_out/up_on.log | cut -c60-130)" || { tail -20 gpurun_out/up_on.log; exit 1; }
  SRL_UP_SMALL1=1 timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/up_off.log 2>&1 && echo "up1 $(tail -1 gpurun_out/up_off.log | cut -c60-130)" || exit 1
done
TOP=90 bash scripts/trace_both.sh > gpurun_out/s3_trace.log 2>&1 || { tail -20 gpurun_out/s3_trace.log; exit 1; }
head -12 gpurun_out/tr2_summary.md
grep "up_small" gpurun_out/tr2_summary.md | cut -c1-120
