#!/bin/bash
# Round-6 batch 3: fused player draws (discrete tail / truncated-normal head) - tests, the benches, the player probe,
# and the ATen small-op call sites of one eager step (SRL_PROFILE_SITES).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONPATH=. TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_actor_tail_gpu.py tests/test_imagine_cont_gpu.py tests/test_dreamer_gpu.py tests/test_algos_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/b3_tests.log 2>&1 || { tail -30 gpurun_out/b3_tests.log; exit 1; }
tail -1 gpurun_out/b3_tests.log
timeout -k 10 300 python scripts/player_after_train.py > gpurun_out/b3_player.log 2>&1; grep player gpurun_out/b3_player.log
for i in 1 2; do
  timeout -k 10 300 python bench.py > gpurun_out/b3_bench_$i.log 2>&1 && tail -1 gpurun_out/b3_bench_$i.log | cut -c1-150 || exit 1
  timeout -k 10 400 python bench.py --continuous --steps 20 --warmup 6 > gpurun_out/b3_cont_$i.log 2>&1 && tail -1 gpurun_out/b3_cont_$i.log | cut -c1-150 || exit 1
done
SRL_PROFILE_SITES=1 SRL_PROFILE_TOP=80 timeout -k 10 300 python bench.py --torch-profile 1 --steps 2 --warmup 2 > gpurun_out/b3_sites.log 2>&1; grep -c SITE gpurun_out/b3_sites.log
