#!/bin/bash
# PPO actor fleet on the Atari-shaped 84x84 pixel env: 1 learner + 2 actor ranks sharing one GPU over
# gloo (RCCL refuses several ranks on one device).  Prints wall time and the learner's logged metrics.
set -o pipefail
mkdir -p gpurun_out/fleet
export SRL_DIST_BACKEND=gloo
STEPS=${STEPS:-20480}
s0=$(date +%s.%N)
timeout -k 10 500 python -u sheeprl.py exp=ppo_decoupled algo.topology=actor_fleet env=synthetic_atari env.id=PongNoFrameskip-v4 \
  env.screen_size=84 env.grayscale=True env.frame_stack=4 "cnn_keys.encoder=[rgb]" "mlp_keys.encoder=[]" env.num_envs=8 \
  env.sync_env=True algo.update_epochs=4 per_rank_batch_size=256 fabric.devices=3 fabric.accelerator=cuda total_steps=$STEPS \
  metric.log_every=4096 checkpoint.every=0 algo.weight_lag=${LAG:-0} root_dir=$PWD/gpurun_out/fleet/run > gpurun_out/fleet/fleet.log 2>&1 || { tail -30 gpurun_out/fleet/fleet.log; exit 1; }
s1=$(date +%s.%N)
python - "$s0" "$s1" "$STEPS" <<'PY'
import glob, json, sys
s0, s1, steps = float(sys.argv[1]), float(sys.argv[2]), int(sys.argv[3])
f = sorted(glob.glob("gpurun_out/fleet/run/*/version_0/metrics.jsonl"))
rows = [json.loads(l) for l in open(f[-1])] if f else []
print(json.dumps({"topology": "actor_fleet 1 learner + 2 actors (gloo, one GPU)", "weight_lag": int(__import__("os").environ.get("LAG", "0")), "policy_steps": steps,
                  "wall_s_incl_startup": round(s1 - s0, 2), "metrics": rows[-6:]}))
PY
rm -rf gpurun_out/fleet/run
