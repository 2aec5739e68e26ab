set -o pipefail
mkdir -p gpurun_out/trace
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace -o run -- \
  python3 bench.py --steps 4 --warmup 4 --profile-steps 4 > gpurun_out/trace_bench.log 2>&1 || exit $?
f=$(find gpurun_out/trace -name '*kernel_trace.csv' | head -1)
python3 scripts/trace_step.py "$f" 4 > gpurun_out/step_seq.tsv
python3 scripts/trace_window.py "$f" 4 80 > gpurun_out/trace_summary.md
rm -f "$f"
head -3 gpurun_out/trace_summary.md
