#!/bin/bash
# Round-4 first GPU call: fault-guard tests, HEAD bench, segmented-mode re-price, traces of the non-headline presets.
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_dv3_step_oracle_gpu.py tests/test_conv_gpu.py tests/test_dreamer_gpu.py tests/test_buffers_gpu.py tests/test_ops_gpu.py tests/test_imagine_cont_gpu.py -x -q -s \
  -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4_tests.log 2>&1; rc=$?
grep ORACLE gpurun_out/r4_tests.log; tail -3 gpurun_out/r4_tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^ERROR|Error" gpurun_out/r4_tests.log | head; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/r4_bench.log 2>&1 && tail -1 gpurun_out/r4_bench.log || { tail -20 gpurun_out/r4_bench.log; exit 1; }
SRL_SCANP_AG=1 timeout -k 10 300 python bench.py > gpurun_out/r4_bench_ag.log 2>&1 && tail -1 gpurun_out/r4_bench_ag.log | cut -c1-200 || exit 1
timeout -k 10 120 python scripts/scanp_phases.py > gpurun_out/r4_scanp.log 2>&1 && head -4 gpurun_out/r4_scanp.log || exit 1
SRL_SCANP_AG=1 timeout -k 10 120 python scripts/scanp_phases.py > gpurun_out/r4_scanp_ag.log 2>&1 && head -4 gpurun_out/r4_scanp_ag.log || exit 1
SRL_IMAG_MERGE=0 timeout -k 10 300 python bench.py > gpurun_out/r4_bench_nomerge.log 2>&1 && tail -1 gpurun_out/r4_bench_nomerge.log | cut -c1-200 || exit 1
SRL_UP_LAST=mfma timeout -k 10 300 python bench.py > gpurun_out/r4_bench_upmfma.log 2>&1 && tail -1 gpurun_out/r4_bench_upmfma.log | cut -c1-200 || exit 1
timeout -k 10 120 python scripts/up_last_timing.py > gpurun_out/r4_uplast.log 2>&1 && tail -1 gpurun_out/r4_uplast.log || exit 1
timeout -k 10 120 python scripts/overlap_probe.py > gpurun_out/r4_overlap.log 2>&1 && tail -1 gpurun_out/r4_overlap.log || exit 1
timeout -k 10 300 python bench.py --segmented --phase-times > gpurun_out/r4_bench_segpt.log 2>&1 && tail -2 gpurun_out/r4_bench_segpt.log || exit 1
timeout -k 10 300 python bench.py --segmented > gpurun_out/r4_bench_seg.log 2>&1 && tail -1 gpurun_out/r4_bench_seg.log || { tail -20 gpurun_out/r4_bench_seg.log; exit 1; }
timeout -k 10 300 python bench.py --continuous > gpurun_out/r4_bench_cont.log 2>&1 && tail -1 gpurun_out/r4_bench_cont.log | cut -c1-200 || exit 1
SRL_IMAG_MERGE=0 timeout -k 10 300 python bench.py --continuous > gpurun_out/r4_bench_cont_nomerge.log 2>&1 && tail -1 gpurun_out/r4_bench_cont_nomerge.log | cut -c1-200 || exit 1
