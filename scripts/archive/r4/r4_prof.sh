#!/bin/bash
# Round-4 traces of the non-headline presets (continuous DV3, SAC, XL) at HEAD.
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
bash scripts/prof.sh r4_cont 20 --continuous --prefill 200 || exit 1
bash scripts/prof.sh r4_sac 200 --algo sac --prefill 300 || exit 1
TLIM=900 bash scripts/prof.sh r4_xl 6 --xl --prefill 100 || exit 1
