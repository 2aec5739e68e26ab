#!/bin/bash
# Round-4: rounds-aware conv weight-gradient plan (numerics, XL + Atari A/B), then the SAC / fleet / op-site items.
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/r410_tests.log 2>&1 && tail -1 gpurun_out/r410_tests.log || { tail -20 gpurun_out/r410_tests.log; exit 1; }
for v in 1 0; do
  SRL_WGRAD_PLAN=$v timeout -k 10 500 python bench.py --xl --steps 12 --warmup 4 --prefill 100 > gpurun_out/r410_xl_$v.log 2>&1 \
    && echo "xl plan=$v $(grep '"metric"' gpurun_out/r410_xl_$v.log | tail -1 | cut -c1-160)" || { tail -20 gpurun_out/r410_xl_$v.log; exit 1; }
done
for v in 1 0; do
  SRL_WGRAD_PLAN=$v timeout -k 10 300 python bench.py --steps 200 > gpurun_out/r410_b_$v.log 2>&1 \
    && echo "atari plan=$v $(tail -1 gpurun_out/r410_b_$v.log | cut -c1-140)" || { tail -20 gpurun_out/r410_b_$v.log; exit 1; }
done
bash scripts/r4_sixth.sh
