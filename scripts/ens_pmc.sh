#!/bin/bash
# PMC pass over the P2E disagreement kernel vs the eager bmm path (scripts/disagreement_timing.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/pmc_ens
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d gpurun_out/pmc_ens -o ens -- python3 scripts/disagreement_timing.py > gpurun_out/pmc_ens/ens.log 2>&1 || exit $?
f=$(find gpurun_out/pmc_ens -name '*counter_collection.csv' | head -1)
python3 - "$f" <<'PY' > gpurun_out/pmc_ens/summary.md
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in rows:
    k = r["Kernel_Name"][:90]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "SQ_WAVES": cnt[k] += 1
names = ["SQ_WAVE_CYCLES", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES", "SQ_LDS_BANK_CONFLICT", "SQ_WAVES"]
print("| kernel | n | " + " | ".join(names) + " | wait% | mfma/busy |")
print("|---|---:|" + "---:|" * (len(names) + 2))
for k, d in sorted(agg.items(), key=lambda x: -x[1]["SQ_WAVE_CYCLES"])[:8]:
    wc = d["SQ_WAVE_CYCLES"] or 1
    print(f"| `{k}` | {cnt[k]} | " + " | ".join(f"{d[n]/max(cnt[k],1):.3g}" for n in names)
          + f" | {100*d['SQ_WAIT_ANY']/wc:.0f} | {d['SQ_VALU_MFMA_BUSY_CYCLES']/max(d['SQ_BUSY_CYCLES'],1):.3g} |")
PY
rm -f "$f"
cat gpurun_out/pmc_ens/summary.md
