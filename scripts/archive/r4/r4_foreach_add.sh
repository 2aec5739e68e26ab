#!/bin/bash
# replay add as one multi-tensor copy for device-resident rows: buffer / SAC / DV3 CLI tests, SAC + DV3 benches, dispatches
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_buffers_gpu.py tests/test_algos_gpu.py tests/test_sac_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r4_fe_tests.log 2>&1 && tail -1 gpurun_out/r4_fe_tests.log || { tail -30 gpurun_out/r4_fe_tests.log; exit 1; }
for i in 1 2; do timeout -k 10 200 python bench.py --algo sac --steps 200 --warmup 20 > gpurun_out/r4_fe_sac_$i.log 2>&1 && echo "sac $(tail -1 gpurun_out/r4_fe_sac_$i.log | cut -c60-100)" || exit 1; done
TOP=20 bash scripts/prof.sh r4_fe_dv3 10 || exit 1
