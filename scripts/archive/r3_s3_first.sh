#!/bin/bash
# Session 3 baseline at HEAD: GPU suite, DV3 bench x2, step trace (categories + top kernels).
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/s3_suite.log 2>&1; rc=$?
tail -3 gpurun_out/s3_suite.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR" gpurun_out/s3_suite.log | head -20; exit $rc; fi
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/s3_dv3_$i.log 2>&1 && tail -1 gpurun_out/s3_dv3_$i.log | cut -c1-160 || exit 1
done
TOP=90 bash scripts/trace_both.sh > gpurun_out/s3_trace.log 2>&1 || { tail -20 gpurun_out/s3_trace.log; exit 1; }
head -12 gpurun_out/tr2_summary.md
