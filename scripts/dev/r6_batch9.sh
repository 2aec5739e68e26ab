#!/bin/bash
# Round-6 batch 9: the deferred weight-gradient branch enqueued before vs after the persistent scan backward, with
# head delays (bench; the scan-health check at the end of bench.py fails the run if the scan was starved)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONPATH=. TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # tag env...
  tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py > gpurun_out/b9_$tag.log 2>&1 || { tail -5 gpurun_out/b9_$tag.log; return 1; }
  echo "$tag: $(tail -1 gpurun_out/b9_$tag.log | cut -c70-110) $(grep -o '"final_wm_loss": [0-9.]*' gpurun_out/b9_$tag.log)"
}
run after X=1 && run before8 SRL_SIDE_BEFORE_SCAN=1 && run before60 SRL_SIDE_BEFORE_SCAN=1 SRL_SIDE_DELAY_US=60 && \
run before150 SRL_SIDE_BEFORE_SCAN=1 SRL_SIDE_DELAY_US=150 && run before400 SRL_SIDE_BEFORE_SCAN=1 SRL_SIDE_DELAY_US=400 && \
run after2 X=1
