#!/bin/bash
# ATen op attribution of one eager DV3 step (framework call sites), for launch-count reduction.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
SRL_PROFILE_SITES=1 SRL_PROFILE_TOP=120 timeout -k 10 400 python bench.py --steps 2 --warmup 3 --prefill 100 --torch-profile 1 > gpurun_out/r3_sites.log 2>&1
rc=$?
grep SITE gpurun_out/r3_sites.log | head -130
exit $rc
