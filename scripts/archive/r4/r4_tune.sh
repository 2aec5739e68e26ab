#!/bin/bash
# Round-4 TunableOp pass for the shapes the round-4 paths introduced (merged imagination GEMM, continuous rollout,
# XL), then A/B benches with the extended results file.  The merged file is left in gpurun_out/tunableop.csv.
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
cp sheeprl_prey_amd/configs/tunableop/mi355x_gemm_results.csv gpurun_out/tunableop.csv
timeout -k 10 200 python -u -m pytest tests/test_prior_head_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4u_ph_tests.log 2>&1 \
  && tail -1 gpurun_out/r4u_ph_tests.log || { tail -20 gpurun_out/r4u_ph_tests.log; exit 1; }
timeout -k 10 120 python scripts/prior_head_timing.py > gpurun_out/r4u_ph_timing.log 2>&1 && tail -1 gpurun_out/r4u_ph_timing.log || exit 1
export SRL_TUNABLEOP_FILE=gpurun_out/tunableop.csv
for v in "1 " "1 --continuous" "0 --continuous"; do
  set -- $v
  m=$1; shift
  SRL_IMAG_MERGE=$m timeout -k 10 400 python -u bench.py --steps 4 --warmup 4 --prefill 200 --gemm-tuning tune "$@" > gpurun_out/r4u_tune_$m$#.log 2>&1 \
    && echo "tuned merge=$m $* -> $(wc -l < gpurun_out/tunableop.csv) lines" || { tail -20 gpurun_out/r4u_tune_$m$#.log; exit 1; }
done
for v in "1 a" "0 b" "1 c" "0 d"; do
  set -- $v
  SRL_IMAG_MERGE=$1 timeout -k 10 300 python bench.py > gpurun_out/r4u_bench_$1$2.log 2>&1 \
    && echo "merge=$1 $(tail -1 gpurun_out/r4u_bench_$1$2.log | cut -c1-140)" || { tail -20 gpurun_out/r4u_bench_$1$2.log; exit 1; }
done
for m in 1 0; do
  SRL_IMAG_MERGE=$m timeout -k 10 300 python bench.py --continuous > gpurun_out/r4u_cont_$m.log 2>&1 \
    && echo "cont merge=$m $(tail -1 gpurun_out/r4u_cont_$m.log | cut -c1-160)" || { tail -20 gpurun_out/r4u_cont_$m.log; exit 1; }
done
