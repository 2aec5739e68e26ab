#!/bin/bash
# Round-4: full-list traces at HEAD (Atari-100k and XL) for the remaining small-kernel / tail analysis.
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
TOP=150 bash scripts/prof.sh r411_dv3 10 || exit 1
TOP=80 TRACE_BY_GRID="igemm,wgrad_kernel,skinny,Cijk_Alik_Bljk_SB_MT128x128x16" TLIM=600 bash scripts/prof.sh r411_xl 6 --xl --prefill 100 || exit 1
