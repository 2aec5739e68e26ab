#!/bin/bash
# GPU validation: kernel numerics + DV3 step tests, then the 1-GPU bench.
# Stops at the first step that ends abnormally (fault / abort / timeout), per pool rules.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-30}
WARMUP=${WARMUP:-6}
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest ended abnormally rc=$rc"; exit $rc; fi
timeout -k 10 600 python bench.py --steps $STEPS --warmup $WARMUP > gpurun_out/bench.log 2>&1
rc2=$?
tail -3 gpurun_out/bench.log
exit $(( rc != 0 ? rc : rc2 ))
