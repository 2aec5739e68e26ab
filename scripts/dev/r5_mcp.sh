set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/mcp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/mcp -o dv3 -- python bench.py --steps 4 --warmup 6 --prefill 100 --profile-steps 4 > gpurun_out/mcp/run.log 2>&1 || { tail -5 gpurun_out/mcp/run.log; exit 1; }
ls gpurun_out/mcp/*/ 2>/dev/null | head; find gpurun_out/mcp -name "*.csv" | head
k=$(find gpurun_out/mcp -name "*kernel_trace.csv" | head -1)
m=$(find gpurun_out/mcp -name "*memory_copy_trace.csv" | head -1)
python - "$k" "$m" <<'PY'
import csv, sys
K = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
M = sorted(csv.DictReader(open(sys.argv[2])), key=lambda r: int(r["Start_Timestamp"])) if sys.argv[2] else []
print("copies total", len(M), "keys", list(M[0].keys()) if M else None)
# the last step: between the last two scanp::bwd kernels' region
bw = [r for r in K if "scanp::bwd" in r["Kernel_Name"]]
b = bw[-1]
t0 = int(b["Start_Timestamp"]) - 200_000
t1 = int(b["End_Timestamp"]) + 600_000
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K q" + r["Queue_Id"] + " " + r["Kernel_Name"][:50]) for r in K if t0 <= int(r["Start_Timestamp"]) <= t1]
ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY " + str({k: r[k] for k in r if k in ("Direction", "Size", "Src_Agent_Id", "Dst_Agent_Id", "Queue_Id", "Stream_Id")})) for r in M if t0 <= int(r["Start_Timestamp"]) <= t1]
ev.sort()
for s, e, n in ev:
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {n}")
PY
rm -f $k
