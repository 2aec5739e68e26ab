#!/bin/bash
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_wgrad_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/wg_t.log 2>&1 || { tail -30 gpurun_out/wg_t.log; exit 1; }
tail -1 gpurun_out/wg_t.log
bash scripts/r3_sites.sh > gpurun_out/r3p_sites.txt 2>&1 || { tail -20 gpurun_out/r3p_sites.txt; exit 1; }
grep -c SITE gpurun_out/r3p_sites.txt
