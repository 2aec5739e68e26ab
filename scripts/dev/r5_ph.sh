set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5ph
timeout -k 10 200 python -u scripts/dev/prior_head_bench.py > gpurun_out/r5ph/bench.log 2>&1; grep -v amdgpu.ids gpurun_out/r5ph/bench.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_prior_head_gpu.py > gpurun_out/r5ph/tests.log 2>&1; tail -2 gpurun_out/r5ph/tests.log
