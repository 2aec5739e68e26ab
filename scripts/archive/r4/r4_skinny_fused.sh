#!/bin/bash
# skinny GEMM in-launch split combine (SRL_SKINNY_FUSED): tests, per-shape A/B, XL scan A/B, XL bench A/B
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_skinny_gpu.py tests/test_dreamer_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "skinny or xl_shape" > gpurun_out/r4_sk_tests.log 2>&1 && tail -2 gpurun_out/r4_sk_tests.log || { tail -30 gpurun_out/r4_sk_tests.log; exit 1; }
timeout -k 10 200 python -u scripts/skinny_sweep.py > gpurun_out/r4_sk_sweep1.log 2>&1 && cat gpurun_out/r4_sk_sweep1.log || { tail -20 gpurun_out/r4_sk_sweep1.log; exit 1; }
SRL_SKINNY_FUSED=0 timeout -k 10 200 python -u scripts/skinny_sweep.py > gpurun_out/r4_sk_sweep0.log 2>&1 && cat gpurun_out/r4_sk_sweep0.log || { tail -20 gpurun_out/r4_sk_sweep0.log; exit 1; }
timeout -k 10 300 python -u scripts/xl_scan_timing.py > gpurun_out/r4_sk_scan1.log 2>&1 && tail -2 gpurun_out/r4_sk_scan1.log || { tail -20 gpurun_out/r4_sk_scan1.log; exit 1; }
SRL_SKINNY_FUSED=0 timeout -k 10 300 python -u scripts/xl_scan_timing.py > gpurun_out/r4_sk_scan0.log 2>&1 && tail -2 gpurun_out/r4_sk_scan0.log || { tail -20 gpurun_out/r4_sk_scan0.log; exit 1; }
timeout -k 10 400 python bench.py --xl > gpurun_out/r4_xl_sk1.log 2>&1 && tail -1 gpurun_out/r4_xl_sk1.log | cut -c1-200 || { tail -20 gpurun_out/r4_xl_sk1.log; exit 1; }
SRL_SKINNY_FUSED=0 timeout -k 10 400 python bench.py --xl > gpurun_out/r4_xl_sk0.log 2>&1 && tail -1 gpurun_out/r4_xl_sk0.log | cut -c1-200 || { tail -20 gpurun_out/r4_xl_sk0.log; exit 1; }
