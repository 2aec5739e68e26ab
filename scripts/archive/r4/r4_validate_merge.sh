#!/bin/bash
# merged imagination GEMM on by default (discrete): full GPU suite, smoke, bench; continuous merge A/B
set -u
export TMPDIR=/tmp PYTHONPATH=.
bash scripts/gpu_validate.sh || exit 1
for rep in 1 2; do
  for m in 0 1; do
    SRL_IMAG_MERGE_CONT=$m timeout -k 10 300 python bench.py --continuous > gpurun_out/r4_cmerge_$m.log 2>&1 && echo "cont merge=$m rep$rep $(tail -1 gpurun_out/r4_cmerge_$m.log | cut -c70-150)" || { tail -20 gpurun_out/r4_cmerge_$m.log; exit 1; }
  done
done
