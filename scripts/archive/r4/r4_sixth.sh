#!/bin/bash
# Round-4 sixth GPU call: ATen op sites (discrete + continuous), SAC fused-critic A/B (interleaved, 2 rounds),
# actor-fleet rehearsal at weight lag 0 / 1, 2-rank gloo rehearsal of the DV3 step on one GPU.
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
bash scripts/r4_sites.sh || exit 1
for i in 1; do
  timeout -k 10 300 python bench.py --algo sac --steps 400 --warmup 50 > gpurun_out/r4_sac_fused_$i.log 2>&1 && echo "sac fused $(tail -1 gpurun_out/r4_sac_fused_$i.log | cut -c1-200)" || exit 1
  SRL_SAC_FUSED=0 timeout -k 10 300 python bench.py --algo sac --steps 400 --warmup 50 > gpurun_out/r4_sac_eager_$i.log 2>&1 && echo "sac eager $(tail -1 gpurun_out/r4_sac_eager_$i.log | cut -c1-200)" || exit 1
done
LAG=0 STEPS=20480 bash scripts/rehearse_fleet.sh > gpurun_out/r4_fleet_lag0.log 2>&1 && tail -1 gpurun_out/r4_fleet_lag0.log | cut -c1-1500 || { tail -30 gpurun_out/r4_fleet_lag0.log; exit 1; }
LAG=1 STEPS=20480 bash scripts/rehearse_fleet.sh > gpurun_out/r4_fleet_lag1.log 2>&1 && tail -1 gpurun_out/r4_fleet_lag1.log | cut -c1-1500 || { tail -30 gpurun_out/r4_fleet_lag1.log; exit 1; }
bash scripts/rehearse_2rank.sh > gpurun_out/r4_rehearse2.log 2>&1 && tail -1 gpurun_out/r4_rehearse2.log | cut -c1-1500 || { tail -30 gpurun_out/r4_rehearse2.log; exit 1; }
