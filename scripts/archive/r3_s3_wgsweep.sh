#!/bin/bash
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
for wgs in 256 512 1024; do
  rm -rf gpurun_out/wgsw
  SRL_WGRAD_WGS=$wgs SRL_WGRAD_OH_WGS=$((wgs / 2)) timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wgsw -o w -- python3 scripts/wg_sweep.py > gpurun_out/wgsw.log 2>&1 || { tail -5 gpurun_out/wgsw.log; exit 1; }
  f=$(find gpurun_out/wgsw -name '*kernel_stats.csv' | head -1)
  echo "dense WGs $wgs, onehot WGs $((wgs / 2)):"
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "wgrad" in r["Name"]:
        print(f'   {float(r["AverageNs"])/1e3:8.1f} us  {r["Name"][:70]}')
PY
done
