#!/bin/bash
# Round-6 batch 13: the 512 x 512 head weight gradients over 16k imagined rows through the split-K kernel (tiles <= 32,
# default) vs the library GEMM + column sum (SRL_WGRAD_MAX_TILES=15): bench pairs + actor / critic phase times
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONPATH=. TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  for mt in 32 15; do
    SRL_WGRAD_MAX_TILES=$mt timeout -k 10 300 python bench.py > gpurun_out/b13_mt${mt}_$i.log 2>&1 || { tail -5 gpurun_out/b13_mt${mt}_$i.log; exit 1; }
    echo "max_tiles=$mt: $(grep -o '"value": [0-9.]*' gpurun_out/b13_mt${mt}_$i.log)"
  done
done
for mt in 32 15; do
  SRL_WGRAD_MAX_TILES=$mt timeout -k 10 300 python bench.py --phase-times --steps 20 --warmup 6 > gpurun_out/b13_phase_$mt.log 2>&1 && echo "max_tiles=$mt: $(grep -h 'phase ms' gpurun_out/b13_phase_$mt.log)"
done
