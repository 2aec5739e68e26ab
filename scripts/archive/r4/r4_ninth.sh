#!/bin/bash
# Round-4: player env-count fix + vector-observation DV3 + LN kernel tests, the CartPole learning curve, XL bench.
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_dreamer_gpu.py tests/test_ops_gpu.py -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread -k "player or vector or ln" > gpurun_out/r49_tests.log 2>&1 && tail -1 gpurun_out/r49_tests.log || { tail -20 gpurun_out/r49_tests.log; exit 1; }
bash scripts/r4_second.sh || exit 1
timeout -k 10 500 python bench.py --xl --steps 12 --warmup 4 --prefill 100 > gpurun_out/r49_xl.log 2>&1 \
  && echo "xl $(grep '"metric"' gpurun_out/r49_xl.log | tail -1 | cut -c1-160)" || { tail -20 gpurun_out/r49_xl.log; exit 1; }
