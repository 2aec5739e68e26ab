set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5c3
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_imagine_cont_gpu.py tests/test_actor_loss_cont_gpu.py > gpurun_out/r5c3/tests.log 2>&1; tail -2 gpurun_out/r5c3/tests.log
timeout -k 10 400 python -u bench.py --continuous --steps 20 --warmup 6 > gpurun_out/r5c3/c0.log 2>&1 && tail -1 gpurun_out/r5c3/c0.log | cut -c1-140 &&
STEPS=10 TOP=60 STEPDUMP=gpurun_out/r5c3/step.txt timeout -k 10 500 bash scripts/gpu_trace.sh --continuous > gpurun_out/r5c3/trace.log 2>&1 && cp gpurun_out/trace_summary.md gpurun_out/r5c3/trace.md && head -1 gpurun_out/r5c3/trace.md &&
timeout -k 10 400 python -u bench.py --continuous --steps 20 --warmup 6 > gpurun_out/r5c3/c1.log 2>&1 && tail -1 gpurun_out/r5c3/c1.log | cut -c1-140
