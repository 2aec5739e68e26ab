#!/bin/bash
# PMC pass over the persistent scan (scripts/scanp_phases.py): I-cache, instruction mix, waits.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d gpurun_out/pmc -o scanp -- python3 scripts/scanp_phases.py > gpurun_out/pmc/run.log 2>&1
rc=$?
f=$(find gpurun_out/pmc -name "*counter_collection.csv" | head -1)
[ -n "$f" ] && python3 - "$f" <<'PY' > gpurun_out/scanp_pmc.txt
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
acc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in rows:
    k = r.get("Kernel_Name", "")
    if "scanp::" not in k:
        continue
    name = "fwd" if "fwd_kernel" in k else ("bwd" if "bwd_kernel" in k else "other")
    acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[(name, r["Counter_Name"])] += 1
for n, d in acc.items():
    print(n, {c: round(v / max(cnt[(n, c)], 1)) for c, v in sorted(d.items())})
PY
cat gpurun_out/scanp_pmc.txt
rm -f gpurun_out/pmc/*counter_collection.csv
exit $rc
