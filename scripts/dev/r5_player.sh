set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5p
timeout -k 10 200 python -u scripts/dev/player_probe.py > gpurun_out/r5p/probe.log 2>&1 && tail -3 gpurun_out/r5p/probe.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5p/tr -o pl -- python scripts/dev/player_probe.py > gpurun_out/r5p/probe_tr.log 2>&1 &&
f=$(find gpurun_out/r5p/tr -name "*kernel_trace.csv" | head -1) && python scripts/trace_step.py "$f" 3 > gpurun_out/r5p/player_step.txt && rm -f "$f" && cat gpurun_out/r5p/player_step.txt | cut -c1-100
