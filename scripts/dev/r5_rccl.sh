set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5r
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_rccl_gpu.py tests/test_dv3_overlap_gpu.py > gpurun_out/r5r/tests.log 2>&1; tail -3 gpurun_out/r5r/tests.log
