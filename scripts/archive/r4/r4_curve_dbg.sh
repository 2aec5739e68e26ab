#!/bin/bash
# Short GPU run of the CartPole DV3 curve config (vector observations, no CNN) through the CLI: surfaces its error.
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
exit 0
