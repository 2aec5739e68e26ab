#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_algos_gpu.py tests/test_sac_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "sac or droq" > gpurun_out/sac_tests.log 2>&1 || { tail -30 gpurun_out/sac_tests.log; exit 1; }
tail -1 gpurun_out/sac_tests.log
bash scripts/sac_pendulum.sh
