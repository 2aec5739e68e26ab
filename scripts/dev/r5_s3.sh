set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
T="timeout -k 10"
python -c "import torch; print('prio range', torch.cuda.Stream.priority_range())"
SRL_SIDE_PRIO=-1 STEPS=10 TOP=50 STEPDUMP=gpurun_out/r5/step_seq_prio.txt $T 400 bash scripts/gpu_trace.sh > gpurun_out/r5/trace_prio.log 2>&1 && head -1 gpurun_out/trace_summary.md &&
for v in "SRL_SIDE_PRIO=-1" "SRL_SIDE_PRIO=0" "GPU_MAX_HW_QUEUES=8" "SRL_SIDE_PRIO=-1" "SRL_SIDE_PRIO=0"; do
  env $v $T 300 python -u bench.py --steps 40 --warmup 6 > gpurun_out/r5/bench_ab.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/r5/bench_ab.log | cut -c1-140)"
done
