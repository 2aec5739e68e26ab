#!/bin/bash
# Round-6 batch 10: wm-phase time (hipEvents, --phase-times) with the deferred weight-gradient branch enqueued after
# (default) vs before the persistent scan backward
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONPATH=. TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python bench.py --phase-times --steps 20 --warmup 6 > gpurun_out/b10_after_$i.log 2>&1 && echo "after:  $(grep -h 'phase ms' gpurun_out/b10_after_$i.log)" || exit 1
  SRL_SIDE_BEFORE_SCAN=1 SRL_SIDE_DELAY_US=150 timeout -k 10 300 python bench.py --phase-times --steps 20 --warmup 6 > gpurun_out/b10_before_$i.log 2>&1 && echo "before: $(grep -h 'phase ms' gpurun_out/b10_before_$i.log)" || exit 1
done
