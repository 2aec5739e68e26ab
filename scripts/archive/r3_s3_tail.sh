#!/bin/bash
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_actor_tail_gpu.py tests/test_wgrad_gpu.py tests/test_dreamer_gpu.py tests/test_graphs_gpu.py -x -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > gpurun_out/at_t.log 2>&1 || { grep -E "^FAILED|^E  " gpurun_out/at_t.log | head -20; tail -5 gpurun_out/at_t.log; exit 1; }
tail -1 gpurun_out/at_t.log
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/at_on.log 2>&1 && echo "tail on  $(tail -1 gpurun_out/at_on.log | cut -c60-130)" || { tail -20 gpurun_out/at_on.log; exit 1; }
  SRL_ACTOR_TAIL=0 timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/at_off.log 2>&1 && echo "tail off $(tail -1 gpurun_out/at_off.log | cut -c60-130)" || exit 1
done
