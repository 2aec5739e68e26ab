#!/bin/bash
# 4-launch scan: posterior rows gathered by FX instead of F4's atomics - scan tests, prey step, kernel stats
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dreamer_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "fused_rssm_scan or vector_obs" > gpurun_out/r4_fx_tests.log 2>&1 && tail -1 gpurun_out/r4_fx_tests.log || { tail -30 gpurun_out/r4_fx_tests.log; exit 1; }
bash scripts/archive/r4/r4_prey_step.sh || exit 1
