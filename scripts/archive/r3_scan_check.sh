#!/bin/bash
# Persistent-scan change check: scan / DreamerV3 numerics tests, per-phase timeline, two DV3 benches.
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dreamer_gpu.py tests/test_onehot_gpu.py tests/test_sac_gpu.py tests/test_conv_gpu.py -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > gpurun_out/sc_t.log 2>&1; rc=$?
tail -2 gpurun_out/sc_t.log
if [ $rc -ne 0 ]; then grep -E "Error|assert |FAIL" gpurun_out/sc_t.log | head -20; exit $rc; fi
timeout -k 10 200 python -u scripts/scanp_phases.py > gpurun_out/sc_scanp.txt 2>&1 || { tail -20 gpurun_out/sc_scanp.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/sc_scanp.txt
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/sc_dv3_$i.log 2>&1 && tail -1 gpurun_out/sc_dv3_$i.log | cut -c1-200 || exit 1
done
