#!/bin/bash
# merged imagination GEMM only for recurrent states <= 1024 (auto): imagination tests, Atari / XL / continuous benches
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_dreamer_gpu.py tests/test_imagine_cont_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4_mp_tests.log 2>&1 && tail -1 gpurun_out/r4_mp_tests.log || { tail -30 gpurun_out/r4_mp_tests.log; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/r4_mp_atari.log 2>&1 && echo "atari $(tail -1 gpurun_out/r4_mp_atari.log | cut -c60-100)" || exit 1
timeout -k 10 400 python bench.py --xl > gpurun_out/r4_mp_xl.log 2>&1 && echo "xl $(tail -1 gpurun_out/r4_mp_xl.log | cut -c60-100)" || exit 1
timeout -k 10 300 python bench.py --continuous > gpurun_out/r4_mp_cont.log 2>&1 && echo "cont $(tail -1 gpurun_out/r4_mp_cont.log | cut -c70-130)" || exit 1
