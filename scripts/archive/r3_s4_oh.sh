#!/bin/bash
# staged one-hot wgrad scatter: numerics, kernel time A/B (SRL_WGRAD_OH_STAGED), DV3 bench
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_wgrad_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/oh_t.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/oh_t.log | head -20; tail -5 gpurun_out/oh_t.log; exit 1; }
tail -1 gpurun_out/oh_t.log
for st in 1 0; do
  rm -rf gpurun_out/ohp
  SRL_WGRAD_OH_STAGED=$st timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ohp -o w -- python3 scripts/wg_sweep.py > gpurun_out/ohp.log 2>&1 || { tail -5 gpurun_out/ohp.log; exit 1; }
  f=$(find gpurun_out/ohp -name '*kernel_stats.csv' | head -1)
  echo "SRL_WGRAD_OH_STAGED=$st:"
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "wgrad" in r["Name"]:
        print(f'   {float(r["AverageNs"])/1e3:8.1f} us  {r["Name"][:70]}')
PY
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/oh_dv3_$i.log 2>&1 && tail -1 gpurun_out/oh_dv3_$i.log | cut -c1-140 || { tail -20 gpurun_out/oh_dv3_$i.log; exit 1; }
done
SRL_WGRAD_OH_STAGED=0 timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/oh_dv3_off.log 2>&1 && tail -1 gpurun_out/oh_dv3_off.log | cut -c1-140
