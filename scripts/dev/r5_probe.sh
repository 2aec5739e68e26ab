set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/probe
for m in graph eager; do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/probe/$m -o p -- python scripts/dev/branch_probe.py $m > gpurun_out/probe/$m.log 2>&1 || exit 1
  f=$(find gpurun_out/probe/$m -name "*kernel_trace.csv" | head -1)
  echo "== $m"
  python - "$f" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
print(list(rows[0].keys()))
idx = max(i for i, r in enumerate(rows) if "spin" in r["Kernel_Name"] and int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) < 20000)
rows = rows[idx + 1:]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    n = r['Kernel_Name']
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} q{r.get('Queue_Id','?')} s{r.get('Stream_Id','?')} {'SPIN' if 'spin' in n else n[:30]}")
PY
done
