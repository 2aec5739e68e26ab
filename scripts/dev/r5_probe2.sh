set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out/probe2
i=0
for v in "PROBE_FLUSH_BEFORE=1" "PROBE_FLUSH_BEFORE=1 SRL_SIDE_DELAY_US=30"; do
  i=$((i+1))
  env $v timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/probe2/v$i -o p -- python scripts/dev/scan_bwd_probe.py graph > gpurun_out/probe2/v$i.log 2>&1 || { echo "$v FAILED"; tail -3 gpurun_out/probe2/v$i.log; continue; }
  f=$(find gpurun_out/probe2/v$i -name "*kernel_trace.csv" | head -1)
  python - "$f" "$v" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = max(i for i, r in enumerate(rows) if "spin" in r["Kernel_Name"] and int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) < 20000)
rows = rows[idx + 1:]
b = [r for r in rows if "scanp::bwd" in r["Kernel_Name"]][0]
t0 = int(b["Start_Timestamp"]); t1 = int(b["End_Timestamp"])
side = [r for r in rows if "vectorized" in r["Kernel_Name"] and r["Queue_Id"] != b["Queue_Id"] and int(r["Start_Timestamp"]) >= t0 - 50000][:20]
st = [(int(r["Start_Timestamp"]) - t0) / 1e3 for r in side]
gaps = sorted(st[i + 1] - st[i] for i in range(len(st) - 1))
print(f"{sys.argv[2]:40s} scan {(t1 - t0) / 1e3:.0f} us; side n={len(st)} first {st[0] if st else -1:.0f} last {st[-1] if st else -1:.0f} median gap {gaps[len(gaps)//2] if gaps else -1:.1f}")
PY
done
