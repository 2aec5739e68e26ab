#!/bin/bash
# Incremental TunableOp tuning: seed with the committed results, tune only shapes they lack (bench
# shapes after a code change), then bench committed vs retuned on the same box.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cp sheeprl_prey_amd/configs/tunableop/mi355x_gemm_results.csv gpurun_out/tunableop_new.csv
SRL_TUNABLEOP_FILE=gpurun_out/tunableop_new.csv timeout -k 10 900 python -u bench.py --steps 4 --warmup 4 --prefill 100 \
  --gemm-tuning tune > gpurun_out/gemm_retune.log 2>&1 || { tail -30 gpurun_out/gemm_retune.log; exit 1; }
wc -l gpurun_out/tunableop_new.csv
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 150 --warmup 30 > gpurun_out/bench_old.log 2>&1 || exit 1
  echo "committed rep$rep $(tail -1 gpurun_out/bench_old.log | cut -c60-140)"
  SRL_TUNABLEOP_FILE=gpurun_out/tunableop_new.csv timeout -k 10 300 python -u bench.py --steps 150 --warmup 30 > gpurun_out/bench_new.log 2>&1 || exit 1
  echo "retuned   rep$rep $(tail -1 gpurun_out/bench_new.log | cut -c60-140)"
done
