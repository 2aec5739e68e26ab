#!/bin/bash
# Merge the GEMM shapes of more algorithms' default configs into the committed TunableOp results.
set -o pipefail
mkdir -p gpurun_out/sweep
F=$PWD/gpurun_out/tunableop_merged.csv
cp sheeprl_prey_amd/configs/tunableop/mi355x_gemm_results.csv $F
export SRL_TUNABLEOP_FILE=$F
COMMON="fabric=mi355x fabric.devices=1 fabric.tunable_gemm=tune metric.log_every=100000 checkpoint.every=0"
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python -u sheeprl.py "$@" $COMMON root_dir=/tmp/srl_sweep/$name > gpurun_out/sweep/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc lines=$(wc -l < $F)"
  return $rc
}
run droq exp=droq env=gym env.id=Pendulum-v1 total_steps=1100 algo.learning_starts=1000 &&
run ppo_rec exp=ppo_recurrent env=gym env.id=CartPole-v1 total_steps=2048 &&
run dv2 exp=dreamer_v2 env=synthetic_atari "cnn_keys.encoder=[rgb]" "cnn_keys.decoder=[rgb]" env.sync_env=True total_steps=1100 algo.learning_starts=1024 algo.train_every=5 &&
run dv1 exp=dreamer_v1 env=synthetic_atari "cnn_keys.encoder=[rgb]" "cnn_keys.decoder=[rgb]" env.sync_env=True total_steps=1100 algo.learning_starts=1024 algo.train_every=5
