#!/bin/bash
# Round-4 conv A/B: the double-buffered narrow-layer main loop (SRL_CONV_DB bits), the MFMA final ConvT (SRL_UP_LAST),
# numerics (conv GPU tests under each knob) and a bench per variant.
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
for db in 1 2 3; do
  SRL_CONV_DB=$db SRL_UP_LAST=mfma timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > gpurun_out/r4c_tests_db$db.log 2>&1 && tail -1 gpurun_out/r4c_tests_db$db.log || { tail -20 gpurun_out/r4c_tests_db$db.log; exit 1; }
done
for v in "0 valu" "1 mfma" "2 mfma" "3 mfma" "0 mfma"; do
  set -- $v
  SRL_CONV_DB=$1 SRL_UP_LAST=$2 timeout -k 10 300 python bench.py > gpurun_out/r4c_bench_$1_$2.log 2>&1 \
    && echo "db=$1 up=$2 $(tail -1 gpurun_out/r4c_bench_$1_$2.log | cut -c1-120)" || { tail -20 gpurun_out/r4c_bench_$1_$2.log; exit 1; }
done
TAG=base bash scripts/conv_pmc.sh > /dev/null 2>&1 || { echo pmc base failed; exit 1; }
SRL_CONV_DB=3 SRL_UP_LAST=mfma TAG=db3 bash scripts/conv_pmc.sh > /dev/null 2>&1 || { echo pmc db3 failed; exit 1; }
head -14 gpurun_out/pmc/base_summary.md | cut -c1-250; head -14 gpurun_out/pmc/db3_summary.md | cut -c1-250
