#!/bin/bash
# faster host envs (pixel PPO / SAC / continuous DV3 benches) + XCD-ordered conv weight gradients (A/B, tests)
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/conv_wgrad_timing.py > gpurun_out/r4_wg_remap1.log 2>&1 && cat gpurun_out/r4_wg_remap1.log || { tail -20 gpurun_out/r4_wg_remap1.log; exit 1; }
SRL_WGRAD_REMAP=0 timeout -k 10 300 python -u scripts/conv_wgrad_timing.py > gpurun_out/r4_wg_remap0.log 2>&1 && cat gpurun_out/r4_wg_remap0.log || { tail -20 gpurun_out/r4_wg_remap0.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_conv_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4_conv_tests.log 2>&1 && tail -2 gpurun_out/r4_conv_tests.log || { tail -30 gpurun_out/r4_conv_tests.log; exit 1; }
timeout -k 10 300 python bench.py --algo ppo --pixel --steps 20 --warmup 3 > gpurun_out/r4_pix1.log 2>&1 && tail -1 gpurun_out/r4_pix1.log || { tail -20 gpurun_out/r4_pix1.log; exit 1; }
timeout -k 10 300 python bench.py --algo sac > gpurun_out/r4_sac_env.log 2>&1 && tail -1 gpurun_out/r4_sac_env.log || { tail -20 gpurun_out/r4_sac_env.log; exit 1; }
timeout -k 10 400 python bench.py --xl > gpurun_out/r4_xl_remap1.log 2>&1 && tail -1 gpurun_out/r4_xl_remap1.log || { tail -20 gpurun_out/r4_xl_remap1.log; exit 1; }
SRL_WGRAD_REMAP=0 timeout -k 10 400 python bench.py --xl > gpurun_out/r4_xl_remap0.log 2>&1 && tail -1 gpurun_out/r4_xl_remap0.log || { tail -20 gpurun_out/r4_xl_remap0.log; exit 1; }
