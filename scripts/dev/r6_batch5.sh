#!/bin/bash
# Round-6 batch 5: 32-channel conv tile variants (SRL_CONV_T32 = 0..3): correctness (conv stack tests) and the
# per-launch roofline of each, then the bench with each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONPATH=. TMPDIR=/tmp
mkdir -p gpurun_out
for v in 1 2 3; do
  SRL_CONV_T32=$v timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/b5_tests_$v.log 2>&1 || { tail -20 gpurun_out/b5_tests_$v.log; exit 1; }
  echo "T32=$v $(tail -1 gpurun_out/b5_tests_$v.log)"
done
for v in 0 1 2 3; do
  SRL_CONV_T32=$v bash scripts/conv_roofline.sh > /dev/null 2>&1 || exit 1
  cp gpurun_out/conv_roofline.md gpurun_out/b5_roof_$v.md
  echo "T32=$v $(grep 'sum of launches' gpurun_out/b5_roof_$v.md)"; grep -E "igemm_kernel<(128|256), 32" gpurun_out/b5_roof_$v.md | cut -c1-60,100-
done
