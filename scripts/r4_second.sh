#!/bin/bash
# Round-4 second GPU call: DV3 CartPole learning curve (fused vs eager-ops world-model loss), the DV3 CLI loop at
# HEAD, the actor-fleet rehearsal at weight lag 0 / 1.
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 700 python -u scripts/dv3_return_curve.py gpurun_out/r4_dv3_cartpole_curve.md 40000 3000 > gpurun_out/r4_curve.log 2>&1 \
  && tail -1 gpurun_out/r4_curve.log || { tail -30 gpurun_out/r4_curve.log; exit 1; }
LAG=0 STEPS=20480 bash scripts/rehearse_fleet.sh > gpurun_out/r4_fleet_lag0.log 2>&1 && tail -1 gpurun_out/r4_fleet_lag0.log | cut -c1-1500 || { tail -30 gpurun_out/r4_fleet_lag0.log; exit 1; }
LAG=1 STEPS=20480 bash scripts/rehearse_fleet.sh > gpurun_out/r4_fleet_lag1.log 2>&1 && tail -1 gpurun_out/r4_fleet_lag1.log | cut -c1-1500 || { tail -30 gpurun_out/r4_fleet_lag1.log; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --algo sac --steps 400 --warmup 50 > gpurun_out/r4_sac_fused_$i.log 2>&1 && tail -1 gpurun_out/r4_sac_fused_$i.log | cut -c1-300 || exit 1
  SRL_SAC_FUSED=0 timeout -k 10 300 python bench.py --algo sac --steps 400 --warmup 50 > gpurun_out/r4_sac_eager_$i.log 2>&1 && tail -1 gpurun_out/r4_sac_eager_$i.log | cut -c1-300 || exit 1
done
bash scripts/rehearse_2rank.sh > gpurun_out/r4_rehearse2.log 2>&1 && tail -1 gpurun_out/r4_rehearse2.log | cut -c1-1500 || { tail -30 gpurun_out/r4_rehearse2.log; exit 1; }
