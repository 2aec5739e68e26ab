#!/bin/bash
# End-of-session (round-3 session 4) validation at HEAD: smoke(), the whole GPU suite, the default bench (as the driver runs it) x2, trace.
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.log 2>&1 || { tail -20 gpurun_out/fin_smoke.log; exit 1; }
grep -v amdgpu.ids gpurun_out/fin_smoke.log | tail -1
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/fin_suite.log 2>&1; rc=$?
tail -1 gpurun_out/fin_suite.log
grep -i -E "AccumulateGrad|stream does not match" gpurun_out/fin_suite.log | head -3
if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR" gpurun_out/fin_suite.log | head -20; exit $rc; fi
for i in 1 2; do
  timeout -k 10 300 python bench.py > gpurun_out/fin_bench_$i.log 2>&1 && tail -1 gpurun_out/fin_bench_$i.log | cut -c1-200 || { tail -20 gpurun_out/fin_bench_$i.log; exit 1; }
done
TOP=90 bash scripts/trace_both.sh > gpurun_out/s4_trace.log 2>&1 || { tail -20 gpurun_out/s4_trace.log; exit 1; }
head -12 gpurun_out/tr2_summary.md
