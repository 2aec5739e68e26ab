set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5x
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dv3_step_oracle_gpu.py tests/test_dv3_overlap_gpu.py tests/test_dreamer_gpu.py tests/test_algos_gpu.py tests/test_fault_agree_gpu.py > gpurun_out/r5x/tests.log 2>&1; tail -2 gpurun_out/r5x/tests.log
grep -E "^FAILED|^ERROR" gpurun_out/r5x/tests.log | head -5
