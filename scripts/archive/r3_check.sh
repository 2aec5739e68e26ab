#!/bin/bash
# Round-3 quick check: new DV3 tests (forward reuse, scan timeout, RCCL capture), then the bench A/B.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_dreamer_gpu.py tests/test_rccl_gpu.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "reuse or graph_matches or segmented or timeout or rccl or captured" > gpurun_out/r3_t1.log 2>&1; rc=$?
tail -3 gpurun_out/r3_t1.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/r3_b1.log 2>&1 && tail -1 gpurun_out/r3_b1.log &&
SRL_REUSE_FWD=0 timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/r3_b1_noreuse.log 2>&1 && tail -1 gpurun_out/r3_b1_noreuse.log &&
timeout -k 10 300 python bench.py --steps 40 --warmup 8 --segmented > gpurun_out/r3_b1_seg.log 2>&1 && tail -1 gpurun_out/r3_b1_seg.log
rc2=$?
exit $(( rc != 0 ? rc : rc2 ))
