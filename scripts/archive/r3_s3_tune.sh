#!/bin/bash
# Incremental TunableOp retune seeded with the committed results: the XL bench's shapes and the DV3 bench's
# (new since the wgrad / padding changes); then committed vs retuned on the same box.
set -u
export TMPDIR=/tmp PYTHONPATH=. PYTORCH_TUNABLEOP_VERBOSE=1
mkdir -p gpurun_out
cp sheeprl_prey_amd/configs/tunableop/mi355x_gemm_results.csv gpurun_out/tunableop_new.csv
SRL_TUNABLEOP_FILE=gpurun_out/tunableop_new.csv timeout -k 10 500 python -u bench.py --xl --steps 2 --warmup 2 --prefill 100 \
  --gemm-tuning tune > gpurun_out/tune_xl.log 2>&1 || { tail -20 gpurun_out/tune_xl.log; exit 1; }
SRL_TUNABLEOP_FILE=gpurun_out/tunableop_new.csv timeout -k 10 300 python -u bench.py --steps 3 --warmup 3 --prefill 100 \
  --gemm-tuning tune > gpurun_out/tune_dv3.log 2>&1 || { tail -20 gpurun_out/tune_dv3.log; exit 1; }
wc -l gpurun_out/tunableop_new.csv
unset PYTORCH_TUNABLEOP_VERBOSE
timeout -k 10 300 python bench.py --xl --steps 10 --warmup 3 --prefill 100 > gpurun_out/xl_old.log 2>&1 && echo "xl committed $(tail -1 gpurun_out/xl_old.log | cut -c60-130)" || exit 1
SRL_TUNABLEOP_FILE=gpurun_out/tunableop_new.csv timeout -k 10 300 python bench.py --xl --steps 10 --warmup 3 --prefill 100 > gpurun_out/xl_new.log 2>&1 && echo "xl retuned   $(tail -1 gpurun_out/xl_new.log | cut -c60-130)" || exit 1
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/dv_old.log 2>&1 && echo "dv3 committed $(tail -1 gpurun_out/dv_old.log | cut -c60-130)" || exit 1
  SRL_TUNABLEOP_FILE=gpurun_out/tunableop_new.csv timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/dv_new.log 2>&1 && echo "dv3 retuned   $(tail -1 gpurun_out/dv_new.log | cut -c60-130)" || exit 1
done
