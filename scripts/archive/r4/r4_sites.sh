#!/bin/bash
# ATen op call sites of one eager train step (bench.py --torch-profile + SRL_PROFILE_SITES): discrete and continuous.
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
SRL_PROFILE_SITES=1 SRL_PROFILE_TOP=90 timeout -k 10 300 python bench.py --steps 2 --warmup 3 --torch-profile 1 > gpurun_out/r4s_disc.log 2>&1 \
  && grep -c SITE gpurun_out/r4s_disc.log || { tail -20 gpurun_out/r4s_disc.log; exit 1; }
SRL_PROFILE_SITES=1 SRL_PROFILE_TOP=90 timeout -k 10 300 python bench.py --continuous --steps 2 --warmup 3 --torch-profile 1 > gpurun_out/r4s_cont.log 2>&1 \
  && grep -c SITE gpurun_out/r4s_cont.log || { tail -20 gpurun_out/r4s_cont.log; exit 1; }
