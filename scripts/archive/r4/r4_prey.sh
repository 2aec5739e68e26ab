#!/bin/bash
# wide-categorical unimix kernels (prey_d_1's Discrete(100) actor): tests, then DV3 on prey_d_1 through the CLI
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_dreamer_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "unimix or vector_obs" > gpurun_out/r4_wide_tests.log 2>&1 && tail -2 gpurun_out/r4_wide_tests.log || { tail -30 gpurun_out/r4_wide_tests.log; exit 1; }
timeout -k 10 1000 python -u scripts/dv3_atari_curve.py gpurun_out/r4_dv3_prey_curve.md ${PREY_STEPS:-250000} --prey
