#!/bin/bash
# ATen call sites of one eager continuous DV3 train step (which small ops the 1037 dispatches/step come from)
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
SRL_PROFILE_SITES=1 SRL_PROFILE_TOP=90 timeout -k 10 400 python bench.py --continuous --torch-profile 1 --steps 3 --warmup 3 --prefill 200 > gpurun_out/r4_cont_sites.log 2>&1; rc=$?
grep "^SITE" gpurun_out/r4_cont_sites.log | head -90
tail -1 gpurun_out/r4_cont_sites.log | cut -c1-150
exit $rc
