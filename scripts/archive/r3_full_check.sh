#!/bin/bash
# Whole GPU suite (one pytest process), then the persistent-scan phase timeline and two DV3 benches.
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/fc_t.log 2>&1; rc=$?
tail -3 gpurun_out/fc_t.log
grep -i -E "AccumulateGrad|stream does not match" gpurun_out/fc_t.log | head -3
if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR|Error" gpurun_out/fc_t.log | head -20; exit $rc; fi
timeout -k 10 200 python -u scripts/scanp_phases.py > gpurun_out/fc_scanp.txt 2>&1 || { tail -20 gpurun_out/fc_scanp.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/fc_scanp.txt
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/fc_dv3_$i.log 2>&1 && tail -1 gpurun_out/fc_dv3_$i.log | cut -c1-200 || exit 1
done
