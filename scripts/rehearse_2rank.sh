#!/bin/bash
# 2 ranks on one GPU over gloo (RCCL refuses two ranks on one device): exercises the multi-rank
# segmented-graph train step, the collectives between phase replays and the pipelined bench step.
set -o pipefail
mkdir -p gpurun_out
export SRL_DIST_BACKEND=gloo
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 10 --warmup 4 --prefill 200 > gpurun_out/rehearse2.log 2>&1 || { tail -30 gpurun_out/rehearse2.log; exit 1; }
grep '"metric"' gpurun_out/rehearse2.log | cut -c1-900
