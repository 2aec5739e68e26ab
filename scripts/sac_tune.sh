#!/bin/bash
# merge SAC Pendulum GEMM shapes into the committed TunableOp results, then re-measure SAC + DV3 phases
set -o pipefail
mkdir -p gpurun_out/sac
cp sheeprl_prey_amd/configs/tunableop/mi355x_gemm_results.csv gpurun_out/tunableop_merged.csv
SRL_TUNABLEOP_FILE=$PWD/gpurun_out/tunableop_merged.csv timeout -k 10 600 python -u sheeprl.py exp=sac env=gym env.id=Pendulum-v1 fabric=mi355x fabric.devices=1 \
  fabric.tunable_gemm=tune total_steps=1500 algo.learning_starts=1000 metric.log_every=5000 checkpoint.every=0 \
  root_dir=$PWD/gpurun_out/sac/tune > gpurun_out/sac/tune.log 2>&1 || { tail -30 gpurun_out/sac/tune.log; exit 1; }
wc -l gpurun_out/tunableop_merged.csv
cp gpurun_out/tunableop_merged.csv sheeprl_prey_amd/configs/tunableop/mi355x_gemm_results.csv
bash scripts/sac_pendulum.sh
timeout -k 10 200 python -u bench.py --steps 20 --warmup 6 --phase-times > gpurun_out/phase.log 2>&1 && grep "phase ms" gpurun_out/phase.log
