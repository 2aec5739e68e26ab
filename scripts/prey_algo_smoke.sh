#!/bin/bash
# Every discrete-action algorithm on the fork's predator-prey env prey_d_1 (vector obs, Discrete(100)) through the
# CLI on the GPU fast paths, a few hundred steps each: catches kernels whose class / action limits the prey actor
# exceeds (the DV3 imagination did, before the wide unimix kernels).  Prints one PASS / FAIL line per algorithm.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=$PWD
mkdir -p gpurun_out/prey_smoke
rc_all=0
run() {  # name, overrides...
  local name=$1; shift
  local root=$PWD/gpurun_out/prey_smoke/run_$name
  timeout -k 10 ${SMOKE_TLIM:-240} python -u sheeprl.py env=prey fabric=mi355x fabric.devices=1 env.sync_env=True \
    env.capture_video=False checkpoint.every=100000000 metric.log_every=100 "mlp_keys.encoder=[state]" "$@" \
    root_dir=$root run_name=$name > gpurun_out/prey_smoke/$name.log 2>&1
  local rc=$?
  rm -rf $root
  if [ $rc -eq 0 ]; then echo "PASS $name"; else echo "FAIL $name (exit $rc)"; tail -5 gpurun_out/prey_smoke/$name.log; rc_all=1; fi
  # a GPU fault / abort / time limit ends the script: nothing more runs on the GPU after it
  case $rc in 124|134|137|139) exit $rc ;; esac
}
run ppo exp=ppo total_steps=2048 algo.rollout_steps=256
run ppo_recurrent exp=ppo_recurrent env.id=prey_d_1 env.mask_velocities=False env.num_envs=4 total_steps=2048 algo.rollout_steps=256
run dreamer_v3 exp=dreamer_v3 total_steps=600 algo.learning_starts=512 algo.per_rank_sequence_length=16 "mlp_keys.decoder=[state]" "cnn_keys.encoder=[]" "cnn_keys.decoder=[]" algo.dense_units=64 algo.world_model.recurrent_model.recurrent_state_size=64
run dreamer_v2 exp=dreamer_v2 total_steps=600 algo.learning_starts=512 algo.per_rank_sequence_length=16 "mlp_keys.decoder=[state]" "cnn_keys.encoder=[]" "cnn_keys.decoder=[]"
run dreamer_v1 exp=dreamer_v1 total_steps=600 algo.learning_starts=512 algo.per_rank_sequence_length=16 "mlp_keys.decoder=[state]" "cnn_keys.encoder=[]" "cnn_keys.decoder=[]"
run p2e_dv2 exp=p2e_dv2 total_steps=600 algo.learning_starts=512 algo.per_rank_sequence_length=16 "mlp_keys.decoder=[state]" "cnn_keys.encoder=[]" "cnn_keys.decoder=[]"
run p2e_dv1 exp=p2e_dv1 total_steps=600 algo.learning_starts=512 algo.per_rank_sequence_length=16 "mlp_keys.decoder=[state]" "cnn_keys.encoder=[]" "cnn_keys.decoder=[]"
exit $rc_all
