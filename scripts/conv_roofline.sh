#!/bin/bash
# rocprofv3 kernel trace of the conv stack replay (scripts/conv_roofline.py) -> gpurun_out/conv_roofline.md
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/convroof
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/convroof -o conv -- python3 scripts/conv_roofline.py --iters 10 --mult ${MULT:-32} > gpurun_out/convroof.log 2>&1 || { tail -20 gpurun_out/convroof.log; exit 1; }
f=$(find gpurun_out/convroof -name '*kernel_trace.csv' | head -1)
python3 scripts/conv_roofline.py --csv "$f" --iters 10 --mult ${MULT:-32} > gpurun_out/conv_roofline.md
rm -f "$f"
grep "replay" gpurun_out/convroof.log; tail -25 gpurun_out/conv_roofline.md
