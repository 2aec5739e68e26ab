#!/bin/bash
# end-of-session validation at HEAD (clean-built extension): GPU suite, smoke, benches, then every discrete algorithm
# on prey_d_1 through the CLI (the Runner-initialised one-launch column sums on every algorithm's path)
set -u
export TMPDIR=/tmp PYTHONPATH=.
bash scripts/gpu_validate.sh || exit 1
bash scripts/prey_algo_smoke.sh || exit 1
timeout -k 10 300 python bench.py --continuous > gpurun_out/r4_final_cont.log 2>&1 && tail -1 gpurun_out/r4_final_cont.log | cut -c1-160 || { tail -20 gpurun_out/r4_final_cont.log; exit 1; }
timeout -k 10 400 python bench.py --xl > gpurun_out/r4_final_xl.log 2>&1 && tail -1 gpurun_out/r4_final_xl.log | cut -c1-160 || { tail -20 gpurun_out/r4_final_xl.log; exit 1; }
