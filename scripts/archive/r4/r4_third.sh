#!/bin/bash
# Round-4 third GPU call: one-launch prior head + side-stream decoder weight gradients (tests, A/B benches, trace).
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_prior_head_gpu.py tests/test_conv_gpu.py tests/test_dreamer_gpu.py tests/test_onehot_gpu.py \
  tests/test_dv3_step_oracle_gpu.py tests/test_rccl_gpu.py -x -q -s -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4t_tests.log 2>&1; rc=$?
grep ORACLE gpurun_out/r4t_tests.log | cut -c1-160; tail -3 gpurun_out/r4t_tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^ERROR|Error" gpurun_out/r4t_tests.log | head; exit 1; }
for v in "1 1 a" "0 1 b" "1 0 c" "1 1 d"; do
  set -- $v
  SRL_SIDE_WGRAD=$1 SRL_PRIOR_HEAD=$2 timeout -k 10 300 python bench.py > gpurun_out/r4t_bench_$1$2$3.log 2>&1 \
    && echo "side=$1 phead=$2 $(tail -1 gpurun_out/r4t_bench_$1$2$3.log | cut -c1-140)" || { tail -20 gpurun_out/r4t_bench_$1$2$3.log; exit 1; }
done
bash scripts/prof.sh r4t_dv3 10 || exit 1
STEPS=6000 bash scripts/dv3_cli.sh > gpurun_out/r4t_cli.log 2>&1 && tail -1 gpurun_out/r4t_cli.log | cut -c1-1500 || { tail -30 gpurun_out/r4t_cli.log; exit 1; }
