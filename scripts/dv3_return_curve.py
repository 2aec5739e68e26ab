"""DreamerV3 learning curve on CartPole-v1 through the real CLI on the GPU fast path (fused HIP ops +
hipGraph step), plus a short ``fabric.fused_ops=False`` run (eager fp32 reference ops, same seed) whose
world-model loss is overlaid on the fused run's for the first steps.  Writes a markdown summary.

Model: the Atari-100k dims (dense 512, mlp 2, deter 512, hidden 512, stoch 32x32) on the vector
observation; 4 envs, one gradient step every 4 policy steps (replay ratio 256).

usage: python scripts/dv3_return_curve.py <out.md> [total_steps] [eager_steps]"""
import glob
import json
import os
import subprocess
import sys
import time

OUT = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/dv3_return_curve.md"
TOTAL = int(sys.argv[2]) if len(sys.argv) > 2 else 40000
EAGER = int(sys.argv[3]) if len(sys.argv) > 3 else 4000
BASE = ["exp=dreamer_v3", "env=gym", "env.id=CartPole-v1", "mlp_keys.encoder=[state]", "mlp_keys.decoder=[state]",
        "cnn_keys.encoder=[]", "cnn_keys.decoder=[]", "fabric=mi355x", "fabric.devices=1", "env.num_envs=4",
        "env.sync_env=True", "env.capture_video=False", "algo.train_every=4", "algo.learning_starts=1024",
        "algo.dense_units=512", "algo.mlp_layers=2", "algo.world_model.recurrent_model.recurrent_state_size=512",
        "algo.world_model.transition_model.hidden_size=512", "algo.world_model.representation_model.hidden_size=512",
        "buffer.size=100000", "checkpoint.every=100000000", "metric.log_every=500", "seed=5"]


def run(name, over):
    root = os.path.abspath(f"gpurun_out/dv3curve_{name}")
    t0 = time.perf_counter()
    log = open(f"gpurun_out/dv3curve_{name}.log", "w")
    rc = subprocess.run([sys.executable, "-u", "sheeprl.py"] + BASE + over + [f"root_dir={root}", f"run_name={name}"],
                        stdout=log, stderr=subprocess.STDOUT).returncode
    if rc != 0:
        subprocess.run(["rm", "-rf", root])  # the replay memmaps: too large to copy back
        log.close()
        print("".join(open(f"gpurun_out/dv3curve_{name}.log").readlines()[-40:]))
        raise SystemExit(f"{name} run failed with exit code {rc}")
    wall = time.perf_counter() - t0
    f = sorted(glob.glob(f"{root}/{name}/version_*/metrics.jsonl"))[-1]
    rows = [json.loads(line) for line in open(f)]
    subprocess.run(["rm", "-rf", root])
    return wall, rows


os.makedirs("gpurun_out", exist_ok=True)
wall_f, rows_f = run("fused", [f"total_steps={TOTAL}"])
wall_e, rows_e = run("eager", [f"total_steps={EAGER}", "fabric.fused_ops=False", "fabric.cuda_graphs=False"])
curve = [(r["step"], r["Rewards/rew_avg"]) for r in rows_f if "Rewards/rew_avg" in r]
wm_f = {r["step"]: r["Loss/world_model_loss"] for r in rows_f if "Loss/world_model_loss" in r}
wm_e = {r["step"]: r["Loss/world_model_loss"] for r in rows_e if "Loss/world_model_loss" in r}
sps = [(r["step"], r.get("Time/sps_env_interaction"), r.get("Time/sps_train")) for r in rows_f if "Time/sps_train" in r]
lines = [f"# DreamerV3 CartPole-v1 learning curve (GPU fast path, CLI; {TOTAL} policy steps)\n",
         "Random policy mean return on CartPole-v1 is ~22; the 5x bar is 110.\n",
         f"fused run: {wall_f:.1f} s wall-clock (incl. start-up, capture and the final test episode); eager-ops run "
         f"({EAGER} steps): {wall_e:.1f} s\n",
         "| policy step | Rewards/rew_avg |", "|---:|---:|"]
lines += [f"| {s} | {r:.1f} |" for s, r in curve]
lines += ["", "## world-model loss, fused HIP ops vs eager reference ops (same seed, same config)\n",
          "| policy step | fused | eager |", "|---:|---:|---:|"]
lines += [f"| {s} | {wm_f[s]:.4f} | {wm_e.get(s, float('nan')):.4f} |" for s in sorted(wm_f) if s <= EAGER]
lines += ["", "## throughput of the fused run\n", "| policy step | Time/sps_env_interaction | Time/sps_train |", "|---:|---:|---:|"]
lines += [f"| {s} | {a} | {b} |" for s, a, b in sps]
open(OUT, "w").write("\n".join(lines) + "\n")
print("\n".join(lines))
best = max((r for _, r in curve), default=0.0)
print(json.dumps({"best_rew_avg": best, "final_rew_avg": curve[-1][1] if curve else None, "wall_s": round(wall_f, 1)}))
