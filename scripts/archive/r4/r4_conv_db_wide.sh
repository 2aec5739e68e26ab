#!/bin/bash
# double-buffered conv main loop on the wide tiles (SRL_CONV_DB bits 2-6): conv tests, XL and Atari bench A/B
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
SRL_CONV_DB=124 timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4_db_tests.log 2>&1 && tail -2 gpurun_out/r4_db_tests.log || { tail -30 gpurun_out/r4_db_tests.log; exit 1; }
for db in 0 124 0 124; do
  SRL_CONV_DB=$db timeout -k 10 400 python bench.py --xl > gpurun_out/r4_xl_db$db.log 2>&1 && echo "xl db=$db $(tail -1 gpurun_out/r4_xl_db$db.log | cut -c1-160)" || { tail -20 gpurun_out/r4_xl_db$db.log; exit 1; }
done
for db in 0 40 0 40; do
  SRL_CONV_DB=$db timeout -k 10 300 python bench.py > gpurun_out/r4_at_db$db.log 2>&1 && echo "atari db=$db $(tail -1 gpurun_out/r4_at_db$db.log | cut -c1-160)" || { tail -20 gpurun_out/r4_at_db$db.log; exit 1; }
done
