set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
T="timeout -k 10"
$T 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_defer_wgrad_gpu.py tests/test_conv_gpu.py tests/test_fault_agree_gpu.py tests/test_dv3_step_oracle_gpu.py "tests/test_algos_gpu.py::test_dreamer_v3_gpu" -s > gpurun_out/r5/tests_s1.log 2>&1; rc=$?
grep -E "passed|failed|ORACLE|Error" gpurun_out/r5/tests_s1.log | tail -40
[ $rc -ne 0 ] && exit $rc
$T 300 python -u bench.py --steps 30 --warmup 6 > gpurun_out/r5/bench_defer1.log 2>&1 && tail -1 gpurun_out/r5/bench_defer1.log | cut -c1-200 &&
SRL_DEFER_WGRAD=0 $T 300 python -u bench.py --steps 30 --warmup 6 > gpurun_out/r5/bench_defer0.log 2>&1 && tail -1 gpurun_out/r5/bench_defer0.log | cut -c1-200 &&
$T 300 python -u bench.py --steps 30 --warmup 6 algo.interaction_serial_order=True > gpurun_out/r5/bench_serial.log 2>&1 && tail -1 gpurun_out/r5/bench_serial.log | cut -c1-200 &&
$T 300 python -u bench.py --steps 30 --warmup 6 --phase-times > gpurun_out/r5/phase.log 2>&1 && grep -i "phase" gpurun_out/r5/phase.log | tail -3 &&
STEPS=10 TOP=60 STEPDUMP=gpurun_out/r5/step_seq.txt $T 400 bash scripts/gpu_trace.sh > gpurun_out/r5/trace_run.log 2>&1; cp gpurun_out/trace_summary.md gpurun_out/r5/trace_summary.md; head -12 gpurun_out/r5/trace_summary.md
