#!/bin/bash
# Round-6 batch 11: reference (serial) vs pipelined order of effects in the interaction step, 3 alternating pairs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONPATH=. TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3; do
  for so in True False; do
    timeout -k 10 300 python bench.py algo.interaction_serial_order=$so > gpurun_out/b11_${so}_$i.log 2>&1 || { tail -5 gpurun_out/b11_${so}_$i.log; exit 1; }
    echo "serial_order=$so: $(grep -o '"value": [0-9.]*' gpurun_out/b11_${so}_$i.log)"
  done
done
