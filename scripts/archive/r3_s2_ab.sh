#!/bin/bash
# A/B: imagination rollout side-stream overlap (SRL_IMAG_OVERLAP) and the pipelined SAC critic kernels
# (SRL_SAC_FUSED), after the numerics tests of both paths.
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_sac_gpu.py tests/test_onehot_gpu.py tests/test_dreamer_gpu.py -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > gpurun_out/ab_t.log 2>&1; rc=$?
tail -2 gpurun_out/ab_t.log
if [ $rc -ne 0 ]; then grep -E "Error|assert |FAIL" gpurun_out/ab_t.log | head -20; fi
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u scripts/scanp_phases.py > gpurun_out/ab_scanp.txt 2>&1 || { tail -20 gpurun_out/ab_scanp.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_scanp.txt
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/ab_dv3_on$i.log 2>&1 && tail -1 gpurun_out/ab_dv3_on$i.log | cut -c1-200 &&
  SRL_IMAG_OVERLAP=0 timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/ab_dv3_off$i.log 2>&1 && tail -1 gpurun_out/ab_dv3_off$i.log | cut -c1-200 || exit 1
done
timeout -k 10 300 python bench.py --algo sac --steps 300 --warmup 20 > gpurun_out/ab_sac1.log 2>&1 && tail -1 gpurun_out/ab_sac1.log | cut -c1-200 &&
SRL_SAC_FUSED=0 timeout -k 10 300 python bench.py --algo sac --steps 300 --warmup 20 > gpurun_out/ab_sac0.log 2>&1 && tail -1 gpurun_out/ab_sac0.log | cut -c1-200
timeout -k 10 300 python bench.py --algo ppo --pixel --steps 10 --warmup 3 > gpurun_out/ab_ppo_pixel.log 2>&1 && tail -1 gpurun_out/ab_ppo_pixel.log | cut -c1-300 &&
timeout -k 10 300 python bench.py --algo ppo --steps 20 --warmup 3 > gpurun_out/ab_ppo_cart.log 2>&1 && tail -1 gpurun_out/ab_ppo_cart.log | cut -c1-300 &&
STEPS=20480 bash scripts/rehearse_fleet.sh > gpurun_out/ab_fleet.txt 2>&1; rc=$?; grep "actor fleet per update" gpurun_out/fleet/fleet.log | tail -3; tail -c 600 gpurun_out/ab_fleet.txt; exit $rc
