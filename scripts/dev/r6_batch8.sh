#!/bin/bash
# Round-6 batch 8: runtime knobs vs the player bursts after the gradient step (continuous bench, then Atari)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONPATH=. TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # tag env...
  tag=$1; shift
  env "$@" timeout -k 10 400 python bench.py --continuous --steps 20 --warmup 6 > gpurun_out/b8_cont_$tag.log 2>&1 || { tail -5 gpurun_out/b8_cont_$tag.log; return 1; }
  echo "cont $tag: $(tail -1 gpurun_out/b8_cont_$tag.log | cut -c80-150)"
}
run base X=1 && run pktcap1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 && run pktcap0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 && \
run devkarg HIP_FORCE_DEV_KERNARG=1 && run spin30 SRL_SPIN_WAIT_MS=30 && run base2 X=1 && \
true
