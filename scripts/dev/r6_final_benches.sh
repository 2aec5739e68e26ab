#!/bin/bash
# Round-6 final numbers of the secondary benches at HEAD (one run each)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONPATH=. TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # tag args...
  tag=$1; shift
  timeout -k 10 500 python bench.py "$@" > gpurun_out/fin_$tag.log 2>&1 || { echo "$tag FAILED"; tail -5 gpurun_out/fin_$tag.log; return 1; }
  echo "$tag: $(tail -1 gpurun_out/fin_$tag.log | cut -c1-230)"
}
run atari && run continuous --continuous --steps 20 --warmup 6 && run xl --xl --steps 10 --warmup 4 && \
run sac --algo sac && run ppo_dev --algo ppo --device-env && run ppo_pixel --algo ppo --pixel && \
timeout -k 10 300 python scripts/dv3_step_bench.py exp=dreamer_v3_prey --vector 14 --actions 100 --steps 20 > gpurun_out/fin_prey.log 2>&1 && echo "prey: $(tail -1 gpurun_out/fin_prey.log)"
