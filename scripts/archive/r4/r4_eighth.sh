#!/bin/bash
# Round-4: curve-config debug run + LN-GRU / continuous numerics, timing, XL A/B and trace.
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
rm -rf /tmp/dv3dbg
timeout -k 10 300 python -u sheeprl.py exp=dreamer_v3 env=gym env.id=CartPole-v1 "mlp_keys.encoder=[state]" "mlp_keys.decoder=[state]" \
  "cnn_keys.encoder=[]" "cnn_keys.decoder=[]" fabric=mi355x fabric.devices=1 env.num_envs=4 env.sync_env=True env.capture_video=False \
  algo.train_every=4 algo.learning_starts=1024 algo.dense_units=512 algo.mlp_layers=2 \
  algo.world_model.recurrent_model.recurrent_state_size=512 algo.world_model.transition_model.hidden_size=512 \
  algo.world_model.representation_model.hidden_size=512 buffer.size=100000 checkpoint.every=100000000 metric.log_every=500 seed=5 \
  total_steps=1600 root_dir=/tmp/dv3dbg run_name=dbg > gpurun_out/r4_curve_dbg.log 2>&1
rc=$?
echo "curve dbg rc=$rc"; tail -40 gpurun_out/r4_curve_dbg.log | cut -c1-400
rm -rf /tmp/dv3dbg
case $rc in 124|134|137|139) exit 1 ;; esac  # a hang / abort / crash: nothing more on the GPU in this call
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_imagine_cont_gpu.py tests/test_dreamer_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "ln_gru or cont or imagine or vector" > gpurun_out/r47_tests.log 2>&1 \
  && tail -1 gpurun_out/r47_tests.log || { tail -20 gpurun_out/r47_tests.log; exit 1; }
timeout -k 10 120 python scripts/gru_timing.py > gpurun_out/r47_gru_timing.log 2>&1 && tail -1 gpurun_out/r47_gru_timing.log || exit 1
for v in 1 0; do
  SRL_GRU_VEC=$v timeout -k 10 500 python bench.py --xl --steps 12 --warmup 4 --prefill 100 > gpurun_out/r47_xl_$v.log 2>&1 \
    && echo "xl vec=$v $(grep '"metric"' gpurun_out/r47_xl_$v.log | tail -1 | cut -c1-160)" || { tail -20 gpurun_out/r47_xl_$v.log; exit 1; }
done
TRACE_BY_GRID="ln_,skinny,gru" TLIM=600 bash scripts/prof.sh r47_xl 6 --xl --prefill 100 || exit 1
