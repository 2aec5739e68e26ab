#!/bin/bash
# GPU validation as the driver runs it at round end: the whole GPU suite, smoke(), the default bench twice.
# Usage: bash scripts/gpu_validate.sh [tag]   (logs under gpurun_out/<tag>_*)
set -u
tag=${1:-val}
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/${tag}_gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/${tag}_gpu_tests.log
[ $rc -ne 0 ] && { grep -E "^FAILED|^ERROR" gpurun_out/${tag}_gpu_tests.log | head; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${tag}_smoke.log 2>&1 && tail -1 gpurun_out/${tag}_smoke.log || { tail -20 gpurun_out/${tag}_smoke.log; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python bench.py > gpurun_out/${tag}_bench_$i.log 2>&1 && tail -1 gpurun_out/${tag}_bench_$i.log | cut -c1-200 || { tail -20 gpurun_out/${tag}_bench_$i.log; exit 1; }
done
