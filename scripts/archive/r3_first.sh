set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/r3_b0.log 2>&1 && tail -1 gpurun_out/r3_b0.log &&
timeout -k 10 300 python bench.py --steps 40 --warmup 8 --segmented > gpurun_out/r3_b0_seg.log 2>&1 && tail -1 gpurun_out/r3_b0_seg.log &&
timeout -k 10 300 python bench.py --steps 20 --warmup 8 --phase-times > gpurun_out/r3_b0_phase.log 2>&1 && tail -2 gpurun_out/r3_b0_phase.log
