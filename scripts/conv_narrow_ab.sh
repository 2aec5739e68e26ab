#!/bin/bash
set -o pipefail
for v in 0 1 2 3; do
SRL_CONV_NARROW=$v CONV_LAYOUTS=fused,fused timeout -k 10 200 python -u scripts/conv_bench.py > gpurun_out/conv_narrow_$v.log 2>&1 || { tail -20 gpurun_out/conv_narrow_$v.log; exit 1; }
echo "narrow=$v $(grep fused: gpurun_out/conv_narrow_$v.log | tail -1)"
done
SRL_CONV_NARROW=3 timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | tail -1
