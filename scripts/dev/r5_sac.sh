#!/bin/bash
# Fused SAC update: GPU tests, same-box A/B (fused / critic-only kernels / autograd), host phase split, kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "${SKIP_AB:-}" ]; then
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_sac_fused_gpu.py tests/test_sac_gpu.py > gpurun_out/sacf_tests.log 2>&1 || { tail -30 gpurun_out/sacf_tests.log; exit 1; }
tail -1 gpurun_out/sacf_tests.log
for mode in ${MODES:-1 critic 0}; do
  SRL_SAC_FUSED=$mode timeout -k 10 300 python bench.py --algo sac --steps 600 --warmup 50 > gpurun_out/r5_bench_sac_$mode.json 2> gpurun_out/r5_bench_sac_$mode.err || { tail -20 gpurun_out/r5_bench_sac_$mode.err; exit 1; }
  echo "mode $mode: $(tail -1 gpurun_out/r5_bench_sac_$mode.json | cut -c1-200)"
done
fi
if [ -z "${SKIP_PHASES:-}" ]; then
  timeout -k 10 300 python scripts/dev/sac_phases.py 400 > gpurun_out/r5_sac_phases.txt 2>&1 || { tail -20 gpurun_out/r5_sac_phases.txt; exit 1; }
  tail -8 gpurun_out/r5_sac_phases.txt
fi
STEPS=200 STEPDUMP=gpurun_out/r5_sac_step.txt bash scripts/gpu_trace.sh --algo sac
