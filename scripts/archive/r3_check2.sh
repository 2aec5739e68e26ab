#!/bin/bash
# One-hot gather layers: numerics tests, DV3 step tests, then benches (DV3 A/B SRL_ONEHOT, SAC, continuous DV3).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_onehot_gpu.py tests/test_dreamer_gpu.py tests/test_algos_gpu.py -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r3_t2.log 2>&1; rc=$?
tail -3 gpurun_out/r3_t2.log
if [ $rc -ne 0 ]; then grep -E "Error|assert |FAIL" gpurun_out/r3_t2.log | head -20; fi
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/r3_b2.log 2>&1 && tail -1 gpurun_out/r3_b2.log &&
SRL_ONEHOT=0 timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/r3_b2_dense.log 2>&1 && tail -1 gpurun_out/r3_b2_dense.log &&
timeout -k 10 300 python bench.py --algo sac --steps 200 --warmup 20 --prefill 300 > gpurun_out/r3_b2_sac.log 2>&1 && tail -1 gpurun_out/r3_b2_sac.log &&
timeout -k 10 400 python bench.py --continuous --steps 20 --warmup 6 > gpurun_out/r3_b2_cont.log 2>&1 && tail -1 gpurun_out/r3_b2_cont.log
