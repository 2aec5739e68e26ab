set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5h
for i in 0 1; do
SRL_HOST_TIMES=1 timeout -k 10 300 python -u bench.py --steps 60 --warmup 6 > gpurun_out/r5h/host_ps$i.log 2>&1 && tail -2 gpurun_out/r5h/host_ps$i.log | cut -c1-200 &&
SRL_PLAYER_STREAM=0 SRL_HOST_TIMES=1 timeout -k 10 300 python -u bench.py --steps 60 --warmup 6 > gpurun_out/r5h/host_main$i.log 2>&1 && tail -2 gpurun_out/r5h/host_main$i.log | cut -c1-200 || exit 1
done
STEPS=10 TOP=50 STEPDUMP=gpurun_out/r5h/step_ps.txt timeout -k 10 400 bash scripts/gpu_trace.sh > gpurun_out/r5h/trace_ps.log 2>&1
