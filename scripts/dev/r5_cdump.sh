set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5c3
STEPS=10 TOP=60 STEPDUMP=gpurun_out/r5c3/step.txt timeout -k 10 500 bash scripts/gpu_trace.sh --continuous > gpurun_out/r5c3/trace2.log 2>&1; head -1 gpurun_out/trace_summary.md
