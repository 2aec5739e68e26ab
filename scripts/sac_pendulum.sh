#!/bin/bash
# SAC (exp=sac, batch 256, 256x2 MLPs) on the native Pendulum-v1 through the real CLI training loop:
# one env step + one gradient step per policy step after learning_starts.  Prints wall-clock
# policy steps/s of the training part and the logged throughput metrics.
set -o pipefail
mkdir -p gpurun_out/sac
STEPS=${STEPS:-20000}
s0=$(date +%s.%N)
timeout -k 10 600 python -u sheeprl.py exp=sac env=gym env.id=Pendulum-v1 fabric=mi355x fabric.devices=1 \
  total_steps=$STEPS algo.learning_starts=1000 metric.log_every=5000 checkpoint.every=0 \
  root_dir=$PWD/gpurun_out/sac/run > gpurun_out/sac/sac.log 2>&1 || { tail -30 gpurun_out/sac/sac.log; exit 1; }
s1=$(date +%s.%N)
python - "$s0" "$s1" "$STEPS" <<'PY'
import glob, json, sys
s0, s1, steps = float(sys.argv[1]), float(sys.argv[2]), int(sys.argv[3])
f = sorted(glob.glob("gpurun_out/sac/run/*/version_0/metrics.jsonl"))[-1]
rows = [json.loads(l) for l in open(f)]
keep = {k: v for r in rows for k, v in r.items() if k.startswith("Time/") or k.startswith("Rewards") or k == "Test/cumulative_reward"}
print(json.dumps({"sac_pendulum_total_steps": steps, "cli_wall_s": round(s1 - s0, 2),
                  "policy_steps_per_s_wall_incl_startup": round(steps / (s1 - s0), 1), **keep}))
PY
