#!/bin/bash
# Round-4 fourth GPU call: the merged imagination GEMM + one-launch prior head now active (transition bias in the
# GEMM epilogue): numerics, A/B benches (discrete + continuous), trace.
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_prior_head_gpu.py tests/test_onehot_gpu.py tests/test_dreamer_gpu.py tests/test_imagine_cont_gpu.py \
  tests/test_dv3_step_oracle_gpu.py -x -q -s -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4f_tests.log 2>&1; rc=$?
grep ORACLE gpurun_out/r4f_tests.log | cut -c1-160; tail -3 gpurun_out/r4f_tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^ERROR|Error" gpurun_out/r4f_tests.log | head; exit 1; }
for v in "1 1 a" "0 1 b" "1 0 c" "1 1 d"; do
  set -- $v
  SRL_IMAG_MERGE=$1 SRL_PRIOR_HEAD=$2 timeout -k 10 300 python bench.py > gpurun_out/r4f_bench_$1$2$3.log 2>&1 \
    && echo "merge=$1 phead=$2 $(tail -1 gpurun_out/r4f_bench_$1$2$3.log | cut -c1-140)" || { tail -20 gpurun_out/r4f_bench_$1$2$3.log; exit 1; }
done
for m in 1 0; do
  SRL_IMAG_MERGE=$m timeout -k 10 300 python bench.py --continuous > gpurun_out/r4f_cont_$m.log 2>&1 \
    && echo "cont merge=$m $(tail -1 gpurun_out/r4f_cont_$m.log | cut -c1-160)" || { tail -20 gpurun_out/r4f_cont_$m.log; exit 1; }
done
bash scripts/prof.sh r4f_dv3 10 || exit 1
bash scripts/prof.sh r4f_cont 10 --continuous --prefill 200 || exit 1
