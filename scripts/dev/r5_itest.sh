set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5i
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_interaction_stage_gpu.py > gpurun_out/r5i/tests.log 2>&1; tail -30 gpurun_out/r5i/tests.log
