#!/bin/bash
# rocprofv3 kernel trace of the XL scan timing script (skinny kernels on, then library GEMMs);
# the rocpd databases come back under gpurun_out/xlprof/ (summarise with scripts/rocpd_summary.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=$PWD
mkdir -p gpurun_out/xlprof
for sk in ${SKS:-1 0}; do
  SRL_SKINNY=$sk timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/xlprof/sk$sk -o run -- \
    python3 scripts/xl_scan_timing.py > gpurun_out/xlprof/sk$sk.log 2>&1 || exit $?
  grep XL gpurun_out/xlprof/sk$sk.log | tail -1
done
