#!/bin/bash
# One-time TunableOp tuning of the DV3 bench's library GEMMs; results -> gpurun_out/tunableop.csv
set -o pipefail
mkdir -p gpurun_out
export SRL_TUNABLEOP_FILE=gpurun_out/tunableop.csv
timeout -k 10 900 python -u bench.py --steps 4 --warmup 4 --prefill 100 --gemm-tuning tune > gpurun_out/gemm_tune.log 2>&1 || { tail -30 gpurun_out/gemm_tune.log; exit 1; }
tail -1 gpurun_out/gemm_tune.log | cut -c1-200
wc -l gpurun_out/tunableop.csv
unset SRL_TUNABLEOP_FILE
cp gpurun_out/tunableop.csv sheeprl_prey_amd/configs/tunableop/mi355x_gemm_results.csv
timeout -k 10 300 python -u bench.py --steps 40 --warmup 8 > gpurun_out/bench_tuned.log 2>&1 || { tail -30 gpurun_out/bench_tuned.log; exit 1; }
tail -1 gpurun_out/bench_tuned.log | cut -c1-300
timeout -k 10 300 python -u bench.py --steps 40 --warmup 8 --gemm-tuning off > gpurun_out/bench_untuned.log 2>&1 || { tail -30 gpurun_out/bench_untuned.log; exit 1; }
tail -1 gpurun_out/bench_untuned.log | cut -c1-300
