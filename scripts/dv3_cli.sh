#!/bin/bash
# DreamerV3 Atari-100k recipe through the real CLI loop (synthetic Atari frames): wall clock and the
# logged throughput metrics (Time/sps_*), for comparison with bench.py's harness.
set -o pipefail
mkdir -p gpurun_out/dv3cli
STEPS=${STEPS:-6000}
s0=$(date +%s.%N)
timeout -k 10 900 python -u sheeprl.py exp=dreamer_v3_100k_ms_pacman env=synthetic_atari fabric=mi355x fabric.devices=1 \
  total_steps=$STEPS algo.learning_starts=1024 metric.log_every=2000 checkpoint.every=0 env.sync_env=True "cnn_keys.encoder=[rgb]" "cnn_keys.decoder=[rgb]" \
  root_dir=$PWD/gpurun_out/dv3cli/run > gpurun_out/dv3cli/dv3.log 2>&1 || { tail -30 gpurun_out/dv3cli/dv3.log; exit 1; }
s1=$(date +%s.%N)
python - "$s0" "$s1" "$STEPS" <<'PY'
import glob, json, sys
s0, s1, steps = float(sys.argv[1]), float(sys.argv[2]), int(sys.argv[3])
f = sorted(glob.glob("gpurun_out/dv3cli/run/*/version_0/metrics.jsonl"))[-1]
rows = [json.loads(l) for l in open(f)]
t = [r for r in rows if any(k.startswith("Time/") for k in r)]
print(json.dumps({"dv3_cli_total_policy_steps": steps, "env_steps": steps, "cli_wall_s": round(s1 - s0, 2), "time_metrics": t,
                  "losses_last": {k: v for r in rows for k, v in r.items() if k.startswith("Loss/")}}))
PY
rm -rf gpurun_out/dv3cli/run  # logs / checkpoints: too large to copy back
