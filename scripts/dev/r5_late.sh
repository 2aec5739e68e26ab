set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5l
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_interaction_stage_gpu.py > gpurun_out/r5l/tests.log 2>&1; tail -1 gpurun_out/r5l/tests.log
for i in 0 1; do
timeout -k 10 300 python -u bench.py --steps 60 --warmup 6 > gpurun_out/r5l/late$i.log 2>&1 && tail -1 gpurun_out/r5l/late$i.log | cut -c1-120 &&
SRL_LATE_ADD=0 timeout -k 10 300 python -u bench.py --steps 60 --warmup 6 > gpurun_out/r5l/early$i.log 2>&1 && tail -1 gpurun_out/r5l/early$i.log | cut -c1-120 || exit 1
done
STEPS=10 TOP=50 STEPDUMP=gpurun_out/r5l/step.txt timeout -k 10 400 bash scripts/gpu_trace.sh > gpurun_out/r5l/trace.log 2>&1; head -1 gpurun_out/trace_summary.md
