#!/bin/bash
# Continuous DV3 fused imagination: numerics vs the eager loop, DV3 step tests, benches fast vs eager.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_imagine_cont_gpu.py tests/test_dreamer_gpu.py -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r3_t3.log 2>&1; rc=$?
tail -3 gpurun_out/r3_t3.log
if [ $rc -ne 0 ]; then grep -E "Error|assert |FAIL|Mismatch" gpurun_out/r3_t3.log | head -30; fi
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --continuous --steps 20 --warmup 6 > gpurun_out/r3_b3_cont.log 2>&1 && tail -1 gpurun_out/r3_b3_cont.log &&
SRL_CONT_FAST=0 timeout -k 10 400 python bench.py --continuous --steps 20 --warmup 6 > gpurun_out/r3_b3_cont_eager.log 2>&1 && tail -1 gpurun_out/r3_b3_cont_eager.log
