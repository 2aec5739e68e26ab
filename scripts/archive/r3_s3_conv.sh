#!/bin/bash
# conv: GPU numerics tests, DV3 bench x2, step trace.
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py tests/test_natcnn_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  > gpurun_out/cv_t.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/cv_t.log | head -20; tail -5 gpurun_out/cv_t.log; exit 1; }
tail -2 gpurun_out/cv_t.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/cv_dv3_$i.log 2>&1 && tail -1 gpurun_out/cv_dv3_$i.log | cut -c1-140 || { tail -20 gpurun_out/cv_dv3_$i.log; exit 1; }
done
TOP=90 bash scripts/trace_both.sh > gpurun_out/s3_trace.log 2>&1 || { tail -20 gpurun_out/s3_trace.log; exit 1; }
head -12 gpurun_out/tr2_summary.md
grep "conv::" gpurun_out/tr2_summary.md | cut -c1-140 | head -30
