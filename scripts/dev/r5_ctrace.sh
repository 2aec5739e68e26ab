set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5ct
STEPS=10 TOP=60 STEPDUMP=gpurun_out/r5ct/step.txt timeout -k 10 500 bash scripts/gpu_trace.sh --continuous > gpurun_out/r5ct/trace.log 2>&1 && cp gpurun_out/trace_summary.md gpurun_out/r5ct/trace.md && head -12 gpurun_out/r5ct/trace.md
