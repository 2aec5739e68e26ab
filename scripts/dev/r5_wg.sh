set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5w
timeout -k 10 200 python -u scripts/dev/wgrad_bench.py > gpurun_out/r5w/wg.log 2>&1; cat gpurun_out/r5w/wg.log | grep -v amdgpu.ids
