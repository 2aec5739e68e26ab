#!/bin/bash
# Round-3 re-entry check: the generalized conv stack (L / XL / grayscale shapes) and the kernels added
# late in the previous session (SAC fused critic, continuous DV3 imagination node, one-hot gathers)
# against their eager oracles, then the headline / SAC / continuous benches.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_conv_gpu.py tests/test_sac_gpu.py tests/test_imagine_cont_gpu.py \
  tests/test_onehot_gpu.py tests/test_dreamer_gpu.py -v -p no:cacheprovider --timeout 200 --timeout-method thread \
  > gpurun_out/s2_t.log 2>&1; rc=$?
tail -3 gpurun_out/s2_t.log
if [ $rc -ne 0 ]; then grep -E "Error|assert |FAIL|Mismatch|Warning" gpurun_out/s2_t.log | head -30; fi
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/s2_dv3.log 2>&1 && tail -1 gpurun_out/s2_dv3.log &&
timeout -k 10 300 python bench.py --algo sac --steps 200 --warmup 20 > gpurun_out/s2_sac.log 2>&1 && tail -1 gpurun_out/s2_sac.log &&
SRL_SAC_FUSED=0 timeout -k 10 300 python bench.py --algo sac --steps 200 --warmup 20 > gpurun_out/s2_sac0.log 2>&1 && tail -1 gpurun_out/s2_sac0.log &&
timeout -k 10 400 python bench.py --continuous --steps 20 --warmup 6 > gpurun_out/s2_cont.log 2>&1 && tail -1 gpurun_out/s2_cont.log &&
timeout -k 10 400 python bench.py --xl --steps 6 --warmup 3 > gpurun_out/s2_xl.log 2>&1 && tail -1 gpurun_out/s2_xl.log
