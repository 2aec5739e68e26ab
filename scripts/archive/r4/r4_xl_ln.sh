#!/bin/bash
# grouped LayerNorm on the 16-byte kernels (XL scan prior/posterior hidden layers): tests, scan A/B, bench, trace
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "ln_" > gpurun_out/r4_ln_tests.log 2>&1 && tail -2 gpurun_out/r4_ln_tests.log || { tail -30 gpurun_out/r4_ln_tests.log; exit 1; }
timeout -k 10 300 python -u scripts/xl_scan_timing.py > gpurun_out/r4_xlscan_vec.log 2>&1 && tail -2 gpurun_out/r4_xlscan_vec.log || { tail -20 gpurun_out/r4_xlscan_vec.log; exit 1; }
SRL_LN_VEC_GROUPS=0 timeout -k 10 300 python -u scripts/xl_scan_timing.py > gpurun_out/r4_xlscan_scalar.log 2>&1 && tail -2 gpurun_out/r4_xlscan_scalar.log || { tail -20 gpurun_out/r4_xlscan_scalar.log; exit 1; }
timeout -k 10 400 python bench.py --xl > gpurun_out/r4_xl_lnvec.log 2>&1 && tail -1 gpurun_out/r4_xl_lnvec.log | cut -c1-200 || { tail -20 gpurun_out/r4_xl_lnvec.log; exit 1; }
TLIM=500 TOP=60 bash scripts/prof.sh r4_xl_head 6 --xl --prefill 100 || exit 1
