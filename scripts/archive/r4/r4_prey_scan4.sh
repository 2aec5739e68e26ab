#!/bin/bash
# 4-launch scan at the prey preset's dense 1024 (G4 reduction scratch on the dead dz tile): scan tests, step A/B
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dreamer_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "fused_rssm_scan_matches or vector_obs" > gpurun_out/r4_scan4_tests.log 2>&1 && tail -2 gpurun_out/r4_scan4_tests.log || { tail -30 gpurun_out/r4_scan4_tests.log; exit 1; }
timeout -k 10 300 python -u scripts/dv3_step_bench.py exp=dreamer_v3_prey --vector 14 --actions 100 --steps 20 > gpurun_out/prey_step_scan4.log 2>&1 && echo "scan4: $(tail -1 gpurun_out/prey_step_scan4.log)" || { tail -20 gpurun_out/prey_step_scan4.log; exit 1; }
SRL_SCAN_IMPL=scan9 timeout -k 10 300 python -u scripts/dv3_step_bench.py exp=dreamer_v3_prey --vector 14 --actions 100 --steps 20 > gpurun_out/prey_step_scan9.log 2>&1 && echo "scan9: $(tail -1 gpurun_out/prey_step_scan9.log)" || { tail -20 gpurun_out/prey_step_scan9.log; exit 1; }
