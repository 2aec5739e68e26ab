set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out/probe
for m in graph eager; do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/probe/b$m -o p -- python scripts/dev/scan_bwd_probe.py $m > gpurun_out/probe/b$m.log 2>&1 || { tail gpurun_out/probe/b$m.log; exit 1; }
  f=$(find gpurun_out/probe/b$m -name "*kernel_trace.csv" | head -1)
  echo "== $m"
  python - "$f" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = max(i for i, r in enumerate(rows) if "spin" in r["Kernel_Name"] and int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) < 20000)
rows = rows[idx + 1:]
b = [i for i, r in enumerate(rows) if "scanp::bwd" in r["Kernel_Name"]][0]
rows = rows[max(0, b - 3): b + 30]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} q{r.get('Queue_Id','?')} {r['Kernel_Name'][:40]}")
PY
done
for v in "algo.interaction_serial_order=False" "algo.interaction_serial_order=True" "algo.interaction_serial_order=False" "algo.interaction_serial_order=True"; do
  timeout -k 10 300 python -u bench.py --steps 60 --warmup 6 $v > gpurun_out/probe/bench_ser.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/probe/bench_ser.log | cut -c1-140)"
done
