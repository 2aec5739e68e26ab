"""DreamerV3 on the fork's predator-prey cellworld (exp=dreamer_v3_prey, prey_d_1) through the real CLI on the GPU
fast path; writes a markdown summary of Rewards/rew_avg, Game/success_rate (goal reached, the env's ``is success``)
and the sps metrics per log interval, plus the wall-clock.

usage: python scripts/prey_curve.py <out.md> [total_steps] [seed]"""
import glob
import json
import os
import subprocess
import sys
import time

OUT = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prey_curve.md"
TOTAL = int(sys.argv[2]) if len(sys.argv) > 2 else 450000
SEED = int(sys.argv[3]) if len(sys.argv) > 3 else 7
root = os.path.abspath("gpurun_out/prey_run")
cmd = [sys.executable, "-u", "sheeprl.py", "exp=dreamer_v3_prey", "fabric=mi355x", "fabric.devices=1", f"total_steps={TOTAL}",
       "metric.log_every=10000", "checkpoint.every=100000000", "env.sync_env=True", "env.capture_video=False", f"seed={SEED}",
       f"root_dir={root}", "run_name=prey"]
t0 = time.perf_counter()
with open("gpurun_out/prey_run.log", "w") as log:
    rc = subprocess.run(cmd, stdout=log, stderr=subprocess.STDOUT).returncode
wall = time.perf_counter() - t0
files = sorted(glob.glob(f"{root}/prey/version_*/metrics.jsonl"))
rows = [json.loads(line) for line in open(files[-1])] if files else []
subprocess.run(["rm", "-rf", root])
by_step = {}
for r in rows:
    by_step.setdefault(r.get("step"), {}).update(r)
lines = [f"# DreamerV3 on prey_d_1 (exp=dreamer_v3_prey, GPU, CLI; {TOTAL} policy steps, seed {SEED})", "",
         "`" + " ".join(cmd[2:-2]) + "`", "", f"exit code {rc}; wall-clock {wall:.1f} s incl. start-up and graph capture", "",
         "| policy step | Rewards/rew_avg | Game/success_rate | Time/sps_train | Time/sps_env_interaction |", "|---:|---:|---:|---:|---:|"]
for st in sorted(k for k in by_step if k is not None):
    r = by_step[st]
    f = lambda k: f"{r[k]:.3f}" if isinstance(r.get(k), (int, float)) else ""  # noqa: E731
    lines.append(f"| {st} | {f('Rewards/rew_avg')} | {f('Game/success_rate')} | {f('Time/sps_train')} | {f('Time/sps_env_interaction')} |")
open(OUT, "w").write("\n".join(lines) + "\n")
print("\n".join(lines[:6]))
print("\n".join(lines[-6:]))
sys.exit(rc)
