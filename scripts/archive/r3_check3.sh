#!/bin/bash
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_onehot_gpu.py -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "dv3" > gpurun_out/r3_t3.log 2>&1; rc=$?
tail -3 gpurun_out/r3_t3.log
grep -E "Error|assert |FAIL" gpurun_out/r3_t3.log | head -30
exit $rc
