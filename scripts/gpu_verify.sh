#!/bin/bash
# GPU verification: full gpu test suite, smoke, DV3 + PPO bench lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 120 python -u __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py --steps 40 --warmup 8 > gpurun_out/bench_dv3.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench_dv3.log; exit 1; }
tail -1 gpurun_out/bench_dv3.log
