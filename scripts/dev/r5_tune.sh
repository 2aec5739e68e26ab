#!/bin/bash
# TunableOp: tune the library GEMM shapes not yet in the committed table (continuous + Atari presets), merge,
# then bench both with the merged table.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
cp sheeprl_prey_amd/configs/tunableop/mi355x_gemm_results.csv gpurun_out/tunableop.csv
export SRL_TUNABLEOP_FILE=gpurun_out/tunableop.csv
timeout -k 10 600 python -u bench.py --continuous --steps 2 --warmup 2 --gemm-tuning tune > gpurun_out/tune_cont.log 2>&1 || { tail -20 gpurun_out/tune_cont.log; exit 1; }
wc -l gpurun_out/tunableop.csv
timeout -k 10 600 python -u bench.py --steps 2 --warmup 2 --gemm-tuning tune > gpurun_out/tune_atari.log 2>&1 || { tail -20 gpurun_out/tune_atari.log; exit 1; }
wc -l gpurun_out/tunableop.csv
unset SRL_TUNABLEOP_FILE
cp gpurun_out/tunableop.csv sheeprl_prey_amd/configs/tunableop/mi355x_gemm_results.csv
timeout -k 10 300 python -u bench.py --continuous --steps 20 --warmup 6 > gpurun_out/tuned_cont.json 2>/dev/null || exit 1
tail -1 gpurun_out/tuned_cont.json | cut -c1-160
timeout -k 10 300 python -u bench.py --steps 60 --warmup 8 > gpurun_out/tuned_atari.json 2>/dev/null || exit 1
tail -1 gpurun_out/tuned_atari.json | cut -c1-160
