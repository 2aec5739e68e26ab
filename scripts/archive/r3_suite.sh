#!/bin/bash
# Full GPU suite, then a kernel trace of the bench (per-category summary of the timed window).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r3_suite.log 2>&1; rc=$?
tail -3 gpurun_out/r3_suite.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
STEPS=10 TOP=90 timeout -k 10 600 bash scripts/trace_both.sh
rc2=$?
exit $(( rc != 0 ? rc : rc2 ))
