#!/bin/bash
# Round-4 fifth GPU call: reworked prior head (numerics + timing + merged-path bench A/B, 300 timed steps each),
# then traces of the continuous / SAC / XL presets.
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_prior_head_gpu.py tests/test_onehot_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r45_ph_tests.log 2>&1 \
  && tail -1 gpurun_out/r45_ph_tests.log || { tail -20 gpurun_out/r45_ph_tests.log; exit 1; }
timeout -k 10 120 python scripts/prior_head_timing.py > gpurun_out/r45_ph_timing.log 2>&1 && tail -1 gpurun_out/r45_ph_timing.log || exit 1
for v in "1 a" "0 b" "1 c" "0 d"; do
  set -- $v
  SRL_IMAG_MERGE=$1 timeout -k 10 300 python bench.py --steps 300 > gpurun_out/r45_bench_$1$2.log 2>&1 \
    && echo "merge=$1 $(tail -1 gpurun_out/r45_bench_$1$2.log | cut -c1-140)" || { tail -20 gpurun_out/r45_bench_$1$2.log; exit 1; }
done
bash scripts/r4_prof.sh
