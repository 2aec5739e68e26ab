#!/bin/bash
# Round-6 measurement batch: kernel tests of the changed ops, prey step time, the default bench x2, the player-gap probe,
# the continuous bench + trace.  Every GPU step has its own time limit; a failed test step stops the batch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONPATH=. TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_onehot_gpu.py tests/test_conv_gpu.py tests/test_prior_head_gpu.py tests/test_dreamer_gpu.py tests/test_dv3_step_oracle_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/b1_tests.log 2>&1 || { tail -30 gpurun_out/b1_tests.log; exit 1; }
tail -1 gpurun_out/b1_tests.log
timeout -k 10 300 python scripts/dv3_step_bench.py exp=dreamer_v3_prey --vector 14 --actions 100 --steps 20 > gpurun_out/b1_prey.log 2>&1 && tail -1 gpurun_out/b1_prey.log || exit 1
for i in 1 2; do
  timeout -k 10 300 python bench.py > gpurun_out/b1_bench_$i.log 2>&1 && tail -1 gpurun_out/b1_bench_$i.log | cut -c1-160 || exit 1
  SRL_IMAG_LANES=1 timeout -k 10 300 python bench.py > gpurun_out/b1_bench_l1_$i.log 2>&1 && tail -1 gpurun_out/b1_bench_l1_$i.log | cut -c1-160 || exit 1
done
timeout -k 10 300 python bench.py --phase-times --steps 20 --warmup 6 > gpurun_out/b1_phases.log 2>&1 && grep -h "phase" gpurun_out/b1_phases.log | tail -1
SRL_IMAG_LANES=1 timeout -k 10 300 python bench.py --phase-times --steps 20 --warmup 6 > gpurun_out/b1_phases_l1.log 2>&1 && grep -h "phase" gpurun_out/b1_phases_l1.log | tail -1
timeout -k 10 300 python scripts/player_after_train.py > gpurun_out/b1_player.log 2>&1 && grep player gpurun_out/b1_player.log || exit 1
timeout -k 10 400 python bench.py --continuous --steps 20 --warmup 6 > gpurun_out/b1_cont.log 2>&1 && tail -1 gpurun_out/b1_cont.log | cut -c1-160 || exit 1
STEPS=10 bash scripts/gpu_trace.sh --continuous > /dev/null 2>&1 && cp gpurun_out/trace_summary.md gpurun_out/b1_cont_trace.md && head -12 gpurun_out/b1_cont_trace.md
