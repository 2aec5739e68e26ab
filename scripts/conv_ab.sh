#!/bin/bash
# conv numerics tests, then the fused conv stack timing and the DV3 bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/conv_tests.log 2>&1 || { tail -30 gpurun_out/conv_tests.log; exit 1; }
tail -1 gpurun_out/conv_tests.log
CONV_LAYOUTS=fused,fused timeout -k 10 200 python -u scripts/conv_bench.py > gpurun_out/conv_bench.log 2>&1 || { tail -20 gpurun_out/conv_bench.log; exit 1; }
cat gpurun_out/conv_bench.log
timeout -k 10 300 python -u bench.py --steps 40 --warmup 8 > gpurun_out/bench_dv3.log 2>&1 || { tail -20 gpurun_out/bench_dv3.log; exit 1; }
tail -1 gpurun_out/bench_dv3.log | cut -c1-200
