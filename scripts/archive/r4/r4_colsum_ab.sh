#!/bin/bash
# one-launch ticket column sums vs the two-launch form, same box, interleaved, 150 timed steps
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
for rep in 1 2 3; do
  for t in 1 0; do
    SRL_COLSUM_TICKET=$t timeout -k 10 300 python bench.py --steps 150 --warmup 30 > gpurun_out/r4_ct_$t.log 2>&1 && echo "ticket=$t rep$rep $(tail -1 gpurun_out/r4_ct_$t.log | cut -c60-100)" || exit 1
  done
done
