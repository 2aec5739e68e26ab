#!/bin/bash
# Round-6 batch 6: host-side breakdown of the interaction step (SRL_HOST_TIMES) for the Atari and the continuous bench,
# serial (reference) vs pipelined effect order, and a one-step kernel dump of the continuous bench at HEAD.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONPATH=. TMPDIR=/tmp
mkdir -p gpurun_out
for so in True False; do
  SRL_HOST_TIMES=1 timeout -k 10 300 python bench.py algo.interaction_serial_order=$so > gpurun_out/b6_atari_$so.log 2>&1 || { tail -5 gpurun_out/b6_atari_$so.log; exit 1; }
  grep -h "host ms" gpurun_out/b6_atari_$so.log; tail -1 gpurun_out/b6_atari_$so.log | cut -c1-140
  SRL_HOST_TIMES=1 timeout -k 10 400 python bench.py --continuous --steps 20 --warmup 6 algo.interaction_serial_order=$so > gpurun_out/b6_cont_$so.log 2>&1 || { tail -5 gpurun_out/b6_cont_$so.log; exit 1; }
  grep -h "host ms" gpurun_out/b6_cont_$so.log; tail -1 gpurun_out/b6_cont_$so.log | cut -c1-140
done
STEPS=10 STEPDUMP=gpurun_out/b6_cont_stepdump.txt bash scripts/gpu_trace.sh --continuous > /dev/null 2>&1 && cp gpurun_out/trace_summary.md gpurun_out/b6_cont_trace.md && head -3 gpurun_out/b6_cont_trace.md
