set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u bench.py --steps 30 --warmup 6 > gpurun_out/r5/bench0.log 2>&1 && tail -1 gpurun_out/r5/bench0.log &&
timeout -k 10 300 python -u bench.py --steps 30 --warmup 6 --phase-times > gpurun_out/r5/phase.log 2>&1 && tail -3 gpurun_out/r5/phase.log &&
timeout -k 10 300 python -u bench.py --steps 30 --warmup 6 algo.interaction_serial_order=True > gpurun_out/r5/bench_serial.log 2>&1 && tail -1 gpurun_out/r5/bench_serial.log &&
timeout -k 10 300 python -u bench.py --steps 30 --warmup 6 > gpurun_out/r5/bench1.log 2>&1 && tail -1 gpurun_out/r5/bench1.log &&
STEPS=10 TOP=60 STEPDUMP=gpurun_out/r5/step_seq.txt timeout -k 10 400 bash scripts/gpu_trace.sh > gpurun_out/r5/trace_run.log 2>&1; cp gpurun_out/trace_summary.md gpurun_out/r5/trace_summary.md
