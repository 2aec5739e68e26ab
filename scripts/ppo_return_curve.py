"""PPO CartPole-v1 learning curves (exp=ppo, 65536 policy steps) through the real CLI, host env vs
GPU-resident env (env.device=True), wall-clock included.  Writes a markdown summary.

usage: python scripts/ppo_return_curve.py <out.md> [extra hydra overrides]"""
import glob
import json
import os
import subprocess
import sys
import time

OUT = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ppo_return_curve.md"
EXTRA = sys.argv[2:]
BASE = ["exp=ppo", "env.id=CartPole-v1", "mlp_keys.encoder=[state]", "fabric.accelerator=cuda",
        "metric.log_every=4096", "checkpoint.every=100000000", "env.capture_video=False"]


def run(name, over):
    root = f"ppo_curve_{name}"
    t0 = time.perf_counter()
    subprocess.run([sys.executable, "-m", "sheeprl_prey_amd"] + BASE + over + EXTRA + [f"root_dir={root}", f"run_name={name}"],
                   check=True, stdout=subprocess.DEVNULL)
    wall = time.perf_counter() - t0
    f = sorted(glob.glob(f"logs/runs/{root}/{name}/version_*/metrics.jsonl"))[-1]
    rows = [json.loads(line) for line in open(f)]
    curve = [(r["step"], r["Rewards/rew_avg"]) for r in rows if "Rewards/rew_avg" in r]
    return wall, curve


lines = ["# PPO CartPole-v1 return curves (exp=ppo: 65536 policy steps, 1 env, rollout 128, 10 epochs)\n"]
for name, over in (("device_env", ["env.device=True"]), ("host_env", ["env.sync_env=True"])):
    wall, curve = run(name, over)
    lines.append(f"## {name}: wall-clock {wall:.1f} s for the whole CLI run (incl. startup and the final test episode)\n")
    lines.append("| policy step | Rewards/rew_avg |\n|---:|---:|")
    lines += [f"| {s} | {r:.1f} |" for s, r in curve]
    lines.append("")
os.makedirs(os.path.dirname(OUT) or ".", exist_ok=True)
open(OUT, "w").write("\n".join(lines) + "\n")
print("\n".join(lines))
