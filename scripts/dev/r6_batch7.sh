#!/bin/bash
# Round-6 batch 7: drain the gradient step before enqueuing the player (SRL_DRAIN_BEFORE_PLAYER=1, default) vs not (0):
# Atari and continuous benches alternating, then a one-step kernel dump of the continuous bench with the drain.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONPATH=. TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  for d in 1 0; do
    SRL_DRAIN_BEFORE_PLAYER=$d timeout -k 10 300 python bench.py > gpurun_out/b7_atari_d${d}_$i.log 2>&1 || { tail -5 gpurun_out/b7_atari_d${d}_$i.log; exit 1; }
    echo "atari drain=$d: $(tail -1 gpurun_out/b7_atari_d${d}_$i.log | cut -c70-140)"
    SRL_DRAIN_BEFORE_PLAYER=$d timeout -k 10 400 python bench.py --continuous --steps 20 --warmup 6 > gpurun_out/b7_cont_d${d}_$i.log 2>&1 || { tail -5 gpurun_out/b7_cont_d${d}_$i.log; exit 1; }
    echo "cont drain=$d: $(tail -1 gpurun_out/b7_cont_d${d}_$i.log | cut -c80-160)"
  done
done
STEPS=10 STEPDUMP=gpurun_out/b7_cont_stepdump.txt bash scripts/gpu_trace.sh --continuous > /dev/null 2>&1 && cp gpurun_out/trace_summary.md gpurun_out/b7_cont_trace.md && head -3 gpurun_out/b7_cont_trace.md
