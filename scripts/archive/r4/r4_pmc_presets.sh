#!/bin/bash
# PMC passes (one counter set each, kernel dispatches serialised by the profiler) of the NatureCNN pixel PPO and the SAC benches
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out/pmc
TAG=natcnn PMC_TLIM=240 PMC_CMD="bench.py --algo ppo --pixel --steps 2 --warmup 1" bash scripts/conv_pmc.sh || exit 1
TAG=sac PMC_TLIM=240 PMC_CMD="bench.py --algo sac --steps 20 --warmup 5 --prefill 300" bash scripts/conv_pmc.sh || exit 1
