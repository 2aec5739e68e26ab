set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5ac
STEPS=10 TOP=50 STEPDUMP=gpurun_out/r5ac/step_on.txt timeout -k 10 400 bash scripts/gpu_trace.sh > gpurun_out/r5ac/trace_on.log 2>&1 && cp gpurun_out/trace_summary.md gpurun_out/r5ac/trace_on.md &&
SRL_DV3_AC_OVERLAP=0 STEPS=10 TOP=50 STEPDUMP=gpurun_out/r5ac/step_off.txt timeout -k 10 400 bash scripts/gpu_trace.sh > gpurun_out/r5ac/trace_off.log 2>&1 && cp gpurun_out/trace_summary.md gpurun_out/r5ac/trace_off.md
