#!/bin/bash
# XL with the merged imagination GEMM: tune its new shapes (seeded with the committed results), then A/B merge on/off
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
cp sheeprl_prey_amd/configs/tunableop/mi355x_gemm_results.csv gpurun_out/tunableop_xl.csv
SRL_TUNABLEOP_FILE=gpurun_out/tunableop_xl.csv timeout -k 10 700 python -u bench.py --xl --steps 2 --warmup 3 --prefill 100 --gemm-tuning tune > gpurun_out/xl_tune.log 2>&1 || { tail -30 gpurun_out/xl_tune.log; exit 1; }
wc -l gpurun_out/tunableop_xl.csv
for rep in 1 2; do
  SRL_IMAG_MERGE=0 timeout -k 10 400 python bench.py --xl > gpurun_out/xl_m0.log 2>&1 && echo "merge=0 committed rep$rep $(tail -1 gpurun_out/xl_m0.log | cut -c60-100)" || exit 1
  SRL_TUNABLEOP_FILE=gpurun_out/tunableop_xl.csv timeout -k 10 400 python bench.py --xl > gpurun_out/xl_m1.log 2>&1 && echo "merge=1 retuned rep$rep $(tail -1 gpurun_out/xl_m1.log | cut -c60-100)" || exit 1
done
