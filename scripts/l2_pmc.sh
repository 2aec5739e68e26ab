#!/bin/bash
# L2 (TCC) hit rate per kernel over a few eager DV3 bench steps: is the RSSM scan's per-step
# weight staging served from the XCD's L2 or from MALL/HBM?  One counter pass (2 TCC counters).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/l2pmc
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/l2pmc -o l2 -- python3 bench.py --steps 3 --warmup 2 --prefill 64 --no-graphs > gpurun_out/l2pmc/run.log 2>&1 || exit $?
f=$(find gpurun_out/l2pmc -name '*counter_collection.csv' | head -1)
python3 - "$f" <<'PY' > gpurun_out/l2pmc/summary.md
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in rows:
    k = r["Kernel_Name"][:100]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "SQ_WAVES":
        cnt[k] += 1
print("| kernel | dispatches | L2 hits / dispatch | L2 misses / dispatch | hit % |")
print("|---|---:|---:|---:|---:|")
for k, d in sorted(agg.items(), key=lambda x: -(x[1]["TCC_HIT_sum"] + x[1]["TCC_MISS_sum"]))[:30]:
    n = max(cnt[k], 1)
    h, m = d["TCC_HIT_sum"], d["TCC_MISS_sum"]
    print(f"| `{k}` | {cnt[k]} | {h/n:.4g} | {m/n:.4g} | {100*h/max(h+m,1):.1f} |")
PY
rm -f "$f"
cut -c1-300 gpurun_out/l2pmc/summary.md
