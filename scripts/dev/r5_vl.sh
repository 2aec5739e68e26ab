set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5v
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_value_loss_gpu.py tests/test_dv3_step_oracle_gpu.py tests/test_dv3_overlap_gpu.py tests/test_dreamer_gpu.py tests/test_algos_gpu.py tests/test_imagine_cont_gpu.py > gpurun_out/r5v/tests.log 2>&1; tail -2 gpurun_out/r5v/tests.log
grep -E "^FAILED|^E " gpurun_out/r5v/tests.log | head -8
timeout -k 10 300 python -u bench.py --steps 40 --warmup 6 > gpurun_out/r5v/b0.log 2>&1 && tail -1 gpurun_out/r5v/b0.log | cut -c1-150 &&
STEPS=10 TOP=50 timeout -k 10 400 bash scripts/gpu_trace.sh > gpurun_out/r5v/trace.log 2>&1 && cp gpurun_out/trace_summary.md gpurun_out/r5v/trace.md && head -1 gpurun_out/r5v/trace.md &&
timeout -k 10 300 python -u bench.py --steps 40 --warmup 6 > gpurun_out/r5v/b1.log 2>&1 && tail -1 gpurun_out/r5v/b1.log | cut -c1-150
timeout -k 10 400 python -u bench.py --continuous --steps 20 --warmup 6 > gpurun_out/r5v/c0.log 2>&1 && tail -1 gpurun_out/r5v/c0.log | cut -c1-150
