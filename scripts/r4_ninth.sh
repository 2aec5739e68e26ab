#!/bin/bash
# Round-4: player env-count fix + vector-observation DV3 tests, then the CartPole learning curve.
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_dreamer_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k "player or vector" > gpurun_out/r49_tests.log 2>&1 && tail -1 gpurun_out/r49_tests.log || { tail -20 gpurun_out/r49_tests.log; exit 1; }
bash scripts/r4_second.sh
