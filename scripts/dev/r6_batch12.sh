#!/bin/bash
# Round-6 batch 12: one-launch prior head (default) vs LayerNorm + library GEMM + sampler (SRL_PRIOR_HEAD=0) in the
# imagination rollout: bench pairs + imagine-phase time
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONPATH=. TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  for ph in 1 0; do
    SRL_PRIOR_HEAD=$ph timeout -k 10 300 python bench.py > gpurun_out/b12_ph${ph}_$i.log 2>&1 || { tail -5 gpurun_out/b12_ph${ph}_$i.log; exit 1; }
    echo "prior_head=$ph: $(grep -o '"value": [0-9.]*' gpurun_out/b12_ph${ph}_$i.log)"
  done
done
for ph in 1 0; do
  SRL_PRIOR_HEAD=$ph timeout -k 10 300 python bench.py --phase-times --steps 20 --warmup 6 > gpurun_out/b12_phase_$ph.log 2>&1 && echo "prior_head=$ph: $(grep -h 'phase ms' gpurun_out/b12_phase_$ph.log)"
done
