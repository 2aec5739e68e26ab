#!/bin/bash
# Round-4 DV3 CartPole learning curve on the GPU fast path (fused vs eager-ops world-model loss overlay).
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 700 python -u scripts/dv3_return_curve.py gpurun_out/r4_dv3_cartpole_curve.md 40000 3000 > gpurun_out/r4_curve.log 2>&1 \
  && tail -1 gpurun_out/r4_curve.log || { tail -30 gpurun_out/r4_curve.log; exit 1; }
