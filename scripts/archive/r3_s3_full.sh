#!/bin/bash
# Whole GPU suite (one pytest process), then XL / continuous DV3, PPO pixel and SAC bench lines.
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/fs_t.log 2>&1; rc=$?
tail -2 gpurun_out/fs_t.log
grep -i -E "AccumulateGrad|stream does not match" gpurun_out/fs_t.log | head -3
if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR" gpurun_out/fs_t.log | head -20; exit $rc; fi
timeout -k 10 400 python bench.py --xl --steps 10 --warmup 3 --prefill 100 > gpurun_out/fs_xl.log 2>&1 && tail -1 gpurun_out/fs_xl.log | cut -c1-120 || { tail -5 gpurun_out/fs_xl.log; exit 1; }
timeout -k 10 300 python bench.py --continuous --steps 20 --warmup 4 > gpurun_out/fs_cont.log 2>&1 && tail -1 gpurun_out/fs_cont.log | cut -c1-120 || { tail -5 gpurun_out/fs_cont.log; exit 1; }
timeout -k 10 300 python bench.py --algo ppo --pixel --steps 6 --warmup 2 > gpurun_out/fs_pix.log 2>&1 && tail -1 gpurun_out/fs_pix.log | cut -c1-120 || { tail -5 gpurun_out/fs_pix.log; exit 1; }
timeout -k 10 300 python bench.py --algo sac --steps 200 --warmup 20 --prefill 300 > gpurun_out/fs_sac.log 2>&1 && tail -1 gpurun_out/fs_sac.log | cut -c1-120 || { tail -5 gpurun_out/fs_sac.log; exit 1; }
