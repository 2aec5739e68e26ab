#!/bin/bash
# merged imagination GEMM (SRL_IMAG_MERGE) A/B at HEAD, interleaved, 150 timed steps each
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
for rep in 1 2 3; do
  for m in 0 1; do
    SRL_IMAG_MERGE=$m timeout -k 10 300 python bench.py --steps 150 --warmup 30 > gpurun_out/r4_merge_$m.log 2>&1 && echo "merge=$m rep$rep $(tail -1 gpurun_out/r4_merge_$m.log | cut -c60-140)" || { tail -20 gpurun_out/r4_merge_$m.log; exit 1; }
  done
done
