#!/bin/bash
# TunableOp for the prey preset's library GEMM shapes (seeded with the committed results), then step A/B
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
cp sheeprl_prey_amd/configs/tunableop/mi355x_gemm_results.csv gpurun_out/tunableop_prey.csv
SRL_TUNABLEOP_FILE=gpurun_out/tunableop_prey.csv timeout -k 10 800 python -u scripts/dv3_step_bench.py exp=dreamer_v3_prey fabric.tunable_gemm=tune --vector 14 --actions 100 --steps 2 --warmup 3 > gpurun_out/prey_tune.log 2>&1 || { tail -30 gpurun_out/prey_tune.log; exit 1; }
wc -l gpurun_out/tunableop_prey.csv
for rep in 1 2; do
  timeout -k 10 300 python -u scripts/dv3_step_bench.py exp=dreamer_v3_prey --vector 14 --actions 100 --steps 30 > gpurun_out/prey_old.log 2>&1 || exit 1
  echo "committed rep$rep $(tail -1 gpurun_out/prey_old.log)"
  SRL_TUNABLEOP_FILE=gpurun_out/tunableop_prey.csv timeout -k 10 300 python -u scripts/dv3_step_bench.py exp=dreamer_v3_prey --vector 14 --actions 100 --steps 30 > gpurun_out/prey_new.log 2>&1 || exit 1
  echo "retuned   rep$rep $(tail -1 gpurun_out/prey_new.log)"
done
