#!/bin/bash
# continuous DV3: kernel test, bench, trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_actor_loss_cont_gpu.py tests/test_imagine_cont_gpu.py > gpurun_out/cont_tests.log 2>&1 || { tail -30 gpurun_out/cont_tests.log; exit 1; }
tail -1 gpurun_out/cont_tests.log
timeout -k 10 400 python bench.py --continuous --steps 20 --warmup 6 > gpurun_out/r5_bench_cont.json 2> gpurun_out/r5_bench_cont.err || { tail -20 gpurun_out/r5_bench_cont.err; exit 1; }
tail -1 gpurun_out/r5_bench_cont.json | cut -c1-220
STEPS=10 TOP=40 bash scripts/gpu_trace.sh --continuous
