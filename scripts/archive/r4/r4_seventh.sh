#!/bin/bash
# Round-4 seventh GPU call: wide-row LN-GRU forward (float4) numerics + timing, XL bench A/B.
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_imagine_cont_gpu.py tests/test_dreamer_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "ln_gru or cont or imagine or vector" > gpurun_out/r47_tests.log 2>&1 \
  && tail -1 gpurun_out/r47_tests.log || { tail -20 gpurun_out/r47_tests.log; exit 1; }
timeout -k 10 120 python scripts/gru_timing.py > gpurun_out/r47_gru_timing.log 2>&1 && tail -1 gpurun_out/r47_gru_timing.log || exit 1
for v in 1 0; do
  SRL_GRU_VEC=$v timeout -k 10 500 python bench.py --xl --steps 12 --warmup 4 --prefill 100 > gpurun_out/r47_xl_$v.log 2>&1 \
    && echo "xl vec=$v $(grep '"metric"' gpurun_out/r47_xl_$v.log | tail -1 | cut -c1-160)" || { tail -20 gpurun_out/r47_xl_$v.log; exit 1; }
done
TRACE_BY_GRID="ln_,skinny,gru" TLIM=600 bash scripts/prof.sh r47_xl 6 --xl --prefill 100 || exit 1
