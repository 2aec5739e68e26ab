#!/bin/bash
# Side-stream decoder weight gradients beside the persistent scan backward (ops/sidework.py):
# DV3 + conv GPU tests, then the DV3 bench with the deferral off / on.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  ${SIDE_TESTS:-tests/test_dreamer_gpu.py tests/test_conv_gpu.py} > gpurun_out/side_tests.log 2>&1 || { tail -30 gpurun_out/side_tests.log; exit 1; }
tail -2 gpurun_out/side_tests.log
for v in 0 1; do
  SRL_SIDE_WGRAD=$v timeout -k 10 300 python -u bench.py --steps 100 --warmup 20 > gpurun_out/bench_side$v.log 2>&1 || { tail -20 gpurun_out/bench_side$v.log; exit 1; }
  echo "side=$v $(tail -1 gpurun_out/bench_side$v.log | cut -c1-200)"
done
