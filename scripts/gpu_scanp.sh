#!/bin/bash
# Persistent RSSM scan: numerics vs the python scan, phase timeline, then the DV3 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=.
timeout -k 10 400 python -u -m pytest tests/test_dreamer_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "persist" > gpurun_out/scanp_tests.log 2>&1
rc=$?
tail -8 gpurun_out/scanp_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/scanp_phases.py > gpurun_out/scanp_phases.txt 2>&1 || { tail -20 gpurun_out/scanp_phases.txt; exit 1; }
cat gpurun_out/scanp_phases.txt
timeout -k 10 300 python -u bench.py --steps 30 --warmup 6 > gpurun_out/bench_scanp.log 2>&1 || { tail -20 gpurun_out/bench_scanp.log; exit 1; }
tail -1 gpurun_out/bench_scanp.log
