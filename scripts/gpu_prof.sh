#!/bin/bash
# A/B the hipGraph path vs eager, then a rocprofv3 kernel-trace profile of the graphed bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --steps 20 --warmup 4 --prefill 200 --no-graphs > gpurun_out/bench_eager.log 2>&1 || exit $?
tail -1 gpurun_out/bench_eager.log
timeout -k 10 400 python bench.py --steps 20 --warmup 4 --prefill 200 > gpurun_out/bench_graph.log 2>&1 || exit $?
tail -1 gpurun_out/bench_graph.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o dv3 -- python bench.py --steps 10 --warmup 3 --prefill 100 > gpurun_out/prof.log 2>&1 || exit $?
tail -1 gpurun_out/prof.log
ls -R gpurun_out/prof | head -20
