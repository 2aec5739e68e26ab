#!/bin/bash
# one-launch ticket column sums: the ticket test, the whole GPU suite + smoke + bench, a headline trace (dispatches)
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "colsum" > gpurun_out/r4_colsum_test.log 2>&1 && tail -1 gpurun_out/r4_colsum_test.log || { tail -30 gpurun_out/r4_colsum_test.log; exit 1; }
bash scripts/gpu_validate.sh || exit 1
TOP=40 bash scripts/prof.sh r4_colsum_dv3 10 || exit 1
