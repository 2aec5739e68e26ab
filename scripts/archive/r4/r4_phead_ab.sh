#!/bin/bash
# one-launch prior head on the (now default) merged imagination path: A/B, interleaved, 150 timed steps
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
for rep in 1 2 3; do
  for ph in 1 0; do
    SRL_PRIOR_HEAD=$ph timeout -k 10 300 python bench.py --steps 150 --warmup 30 > gpurun_out/r4_ph_$ph.log 2>&1 && echo "prior_head=$ph rep$rep $(tail -1 gpurun_out/r4_ph_$ph.log | cut -c60-100)" || exit 1
  done
done
