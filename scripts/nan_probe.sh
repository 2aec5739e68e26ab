#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ppo_fused_gpu.py tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_sub.log 2>&1 || { tail -20 gpurun_out/gpu_tests_sub.log; exit 1; }
tail -1 gpurun_out/gpu_tests_sub.log
for i in 1 2; do
timeout -k 10 200 python -u bench.py --steps 2 --warmup 0 --check-finite 90 > gpurun_out/nan_graph_$i.log 2>&1; echo "rc=$?"
grep -A12 "non-finite=\[.G\|non-finite=\[.L" gpurun_out/nan_graph_$i.log | cut -c1-400
grep "check step 89" gpurun_out/nan_graph_$i.log | cut -c1-200
done
