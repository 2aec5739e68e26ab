#!/bin/bash
# 2 ranks on one GPU over gloo: PPO CartPole (device env) with the segmented-graph multi-rank update
# (per-minibatch graph replays, flat-slab gradient all-reduce between them).
set -o pipefail
mkdir -p gpurun_out
export SRL_DIST_BACKEND=gloo
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --algo ppo --device-env --gpus 2 --steps 6 --warmup 3 > gpurun_out/rehearse2_ppo.log 2>&1 || { tail -30 gpurun_out/rehearse2_ppo.log; exit 1; }
grep '"metric"' gpurun_out/rehearse2_ppo.log | cut -c1-900
