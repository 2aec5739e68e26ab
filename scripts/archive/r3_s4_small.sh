#!/bin/bash
# small-batch player encoder: numerics, per-call timing A/B, kernel times, player tests, DV3 bench
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_small_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/cs_t.log 2>&1 || { grep -E "FAILED|Error|error|assert" gpurun_out/cs_t.log | head -20; tail -5 gpurun_out/cs_t.log; exit 1; }
tail -1 gpurun_out/cs_t.log
timeout -k 10 120 python scripts/small_enc_timing.py 2>&1 | grep player
rm -rf gpurun_out/csp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/csp -o w -- python3 scripts/small_enc_timing.py > gpurun_out/csp.log 2>&1 || { tail -5 gpurun_out/csp.log; exit 1; }
f=$(find gpurun_out/csp -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:16]:
    print(f'   {int(r["Calls"]):6d} calls {float(r["AverageNs"])/1e3:8.2f} us  {r["Name"][:90]}')
PY
timeout -k 10 400 python -u -m pytest tests/test_dreamer_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  > gpurun_out/cs_dv3t.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/cs_dv3t.log | head -20; tail -5 gpurun_out/cs_dv3t.log; exit 1; }
tail -1 gpurun_out/cs_dv3t.log
timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/cs_dv3.log 2>&1 && tail -1 gpurun_out/cs_dv3.log | cut -c1-140
SRL_SMALL_ENCODER=0 timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/cs_dv3_off.log 2>&1 && tail -1 gpurun_out/cs_dv3_off.log | cut -c1-140
timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/cs_dv3b.log 2>&1 && tail -1 gpurun_out/cs_dv3b.log | cut -c1-140
