#!/bin/bash
# Step trace (categories + top kernels), ATen call-site attribution, persistent-scan phase timeline.
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
bash scripts/trace_both.sh > gpurun_out/r3p_trace.log 2>&1 || { tail -20 gpurun_out/r3p_trace.log; exit 1; }
head -12 gpurun_out/tr2_summary.md
timeout -k 10 200 python -u scripts/scanp_phases.py > gpurun_out/r3p_scanp.txt 2>&1 || { tail -20 gpurun_out/r3p_scanp.txt; exit 1; }
cat gpurun_out/r3p_scanp.txt
bash scripts/r3_sites.sh > gpurun_out/r3p_sites.txt 2>&1 || { tail -20 gpurun_out/r3p_sites.txt; exit 1; }
head -40 gpurun_out/r3p_sites.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sacprof -o sac -- python3 bench.py --algo sac --steps 200 --warmup 20 --prefill 300 > gpurun_out/r3p_sac.log 2>&1 || { tail -20 gpurun_out/r3p_sac.log; exit 1; }
tail -1 gpurun_out/r3p_sac.log
f=$(find gpurun_out/sacprof -name '*kernel_stats.csv' | head -1)
head -30 "$f"
find gpurun_out/sacprof -name '*kernel_trace.csv' -delete
