set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
T="timeout -k 10"
for v in "SRL_SCANP_NAP=1" "SRL_SCANP_NAP=4" "SRL_SCANP_NAP=16" "SRL_SCANP_NAP=1" "SRL_SCANP_NAP=4"; do
  env $v $T 300 python -u bench.py --steps 40 --warmup 6 > gpurun_out/r5/bench_ab.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/r5/bench_ab.log | cut -c1-140)"
done
SRL_SCANP_NAP=16 STEPS=10 TOP=50 STEPDUMP=gpurun_out/r5/step_seq_nap16.txt $T 400 bash scripts/gpu_trace.sh > gpurun_out/r5/trace_nap.log 2>&1 && head -1 gpurun_out/trace_summary.md
