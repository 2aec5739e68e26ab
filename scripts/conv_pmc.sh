#!/bin/bash
# PMC pass over the fused conv stack (scripts/conv_bench.py, fused layout only), or over any python command:
#   TAG=natcnn PMC_CMD="bench.py --algo ppo --pixel --steps 2 --warmup 1" bash scripts/conv_pmc.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/pmc
CONV_LAYOUTS=fused timeout -s KILL ${PMC_TLIM:-120} rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d gpurun_out/pmc -o ${TAG:-conv} -- python3 ${PMC_CMD:-scripts/conv_bench.py} > gpurun_out/pmc/${TAG:-conv}.log 2>&1 || exit $?
f=$(find gpurun_out/pmc -name '*counter_collection.csv' | head -1)
python3 - "$f" <<'PY' > gpurun_out/pmc/${TAG:-conv}_summary.md
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in rows:
    k = r["Kernel_Name"][:110]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "SQ_WAVES": cnt[k] += 1
names = ["SQ_WAVE_CYCLES","SQ_WAIT_ANY","SQ_WAIT_INST_ANY","SQ_ACTIVE_INST_ANY","SQ_VALU_MFMA_BUSY_CYCLES","SQ_LDS_BANK_CONFLICT","SQ_BUSY_CYCLES","SQ_WAVES"]
print("| kernel | n | " + " | ".join(names) + " | wait% | instwait% | mfma/busy |")
for k, d in sorted(agg.items(), key=lambda x: -x[1]["SQ_WAVE_CYCLES"])[:25]:
    wc = d["SQ_WAVE_CYCLES"] or 1
    print(f"| `{k}` | {cnt[k]} | " + " | ".join(f"{d[n]/max(cnt[k],1):.3g}" for n in names)
          + f" | {100*d['SQ_WAIT_ANY']/wc:.0f} | {100*d['SQ_WAIT_INST_ANY']/wc:.0f} | {d['SQ_VALU_MFMA_BUSY_CYCLES']/max(d['SQ_BUSY_CYCLES'],1):.3g} |")
PY
rm -f "$f"
cat gpurun_out/pmc/${TAG:-conv}_summary.md | cut -c1-400
