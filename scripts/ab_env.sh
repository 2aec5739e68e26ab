#!/bin/bash
# A/B of one environment switch on the DV3 bench in one box: VAR=<name> bash scripts/ab_env.sh (0 then 1, twice)
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do for v in 0 1; do
  env $VAR=$v timeout -k 10 300 python -u bench.py --steps ${STEPS:-150} --warmup 30 > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
  echo "$VAR=$v rep$rep $(tail -1 gpurun_out/ab_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
