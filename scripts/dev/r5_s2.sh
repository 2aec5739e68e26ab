set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_defer_wgrad_gpu.py tests/test_skinny_gpu.py tests/test_dreamer_gpu.py tests/test_conv_gpu.py tests/test_ops_gpu.py tests/test_prior_head_gpu.py > gpurun_out/r5/t_s2.log 2>&1; rc=$?; tail -3 gpurun_out/r5/t_s2.log; [ $rc -ne 0 ] && exit $rc
STEPS=10 TOP=50 STEPDUMP=gpurun_out/r5/step_seq_on.txt $T 400 bash scripts/gpu_trace.sh > gpurun_out/r5/trace_on.log 2>&1 && cp gpurun_out/trace_summary.md gpurun_out/r5/trace_summary_on.md && head -12 gpurun_out/r5/trace_summary_on.md &&
for v in "SRL_DEFER_WGRAD=1" "SRL_DEFER_WGRAD=0" "SRL_SIDE_DELAY_US=0" "SRL_SIDE_DELAY_US=30" "SRL_DEFER_WGRAD=1"; do
  env $v $T 300 python -u bench.py --steps 40 --warmup 6 > gpurun_out/r5/bench_ab.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/r5/bench_ab.log | cut -c1-140)"
done
