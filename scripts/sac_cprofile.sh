#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/sac
timeout -k 10 300 python -u -m cProfile -o gpurun_out/sac/prof.out sheeprl.py exp=sac env=gym env.id=Pendulum-v1 fabric=mi355x fabric.devices=1 \
  total_steps=6000 algo.learning_starts=1000 metric.log_every=5000 checkpoint.every=0 root_dir=$PWD/gpurun_out/sac/prof > gpurun_out/sac/prof.log 2>&1 || { tail -20 gpurun_out/sac/prof.log; exit 1; }
python -c "
import pstats; p = pstats.Stats('gpurun_out/sac/prof.out'); p.sort_stats('tottime').print_stats(35)" > gpurun_out/sac/prof_top.txt
python -c "
import pstats; p = pstats.Stats('gpurun_out/sac/prof.out'); p.sort_stats('cumtime').print_stats(45)" > gpurun_out/sac/prof_cum.txt
