#!/bin/bash
# Round-6 measurement batch 2: the player-gap probe, the continuous bench + kernel trace (with a one-step dump).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONPATH=. TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python scripts/player_after_train.py > gpurun_out/b2_player.log 2>&1; grep player gpurun_out/b2_player.log || tail -5 gpurun_out/b2_player.log
timeout -k 10 300 python -u -m pytest tests/test_imagine_cont_gpu.py tests/test_prior_head_gpu.py tests/test_actor_loss_cont_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/b2_tests.log 2>&1 || { tail -30 gpurun_out/b2_tests.log; exit 1; }
tail -1 gpurun_out/b2_tests.log
for i in 1 2; do
  timeout -k 10 400 python bench.py --continuous --steps 20 --warmup 6 > gpurun_out/b2_cont_$i.log 2>&1 && tail -1 gpurun_out/b2_cont_$i.log | cut -c1-160 || exit 1
  SRL_CONT_PHEAD=0 timeout -k 10 400 python bench.py --continuous --steps 20 --warmup 6 > gpurun_out/b2_cont_off_$i.log 2>&1 && tail -1 gpurun_out/b2_cont_off_$i.log | cut -c1-160 || exit 1
done
STEPS=10 STEPDUMP=gpurun_out/b2_cont_stepdump.txt bash scripts/gpu_trace.sh --continuous > /dev/null 2>&1 && cp gpurun_out/trace_summary.md gpurun_out/b2_cont_trace.md && head -14 gpurun_out/b2_cont_trace.md
