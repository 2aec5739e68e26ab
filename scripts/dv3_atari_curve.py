"""DreamerV3 learning curve from PIXELS through the real CLI on the GPU fast path (HIP conv stack, persistent scan,
fused heads, captured train step): the Atari-100k recipe (``exp=dreamer_v3_100k_ms_pacman``) on the synthetic
Atari env (``envs/synthetic.py``: the action moves sprite 0 on a 3x3 stencil, every other sprite it touches is a
reward of 1 and respawns), 250-step episodes.  On this env a random policy scores 13.8 +- 4.4 per episode and a
hand-written "chase the nearest sprite" policy 89.1 +- 9.8 (20 episodes each, computed by this script on the host).

usage: python scripts/dv3_atari_curve.py <out.md> [total_policy_steps]"""
import glob
import json
import os
import subprocess
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

OUT = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/dv3_atari_curve.md"
TOTAL = int(sys.argv[2]) if len(sys.argv) > 2 else 30000
EP_LEN = 250


def baselines(eps: int = 20):
    from sheeprl_prey_amd.envs.synthetic import SyntheticAtari

    def run(policy):
        tot = []
        for s in range(eps):
            env = SyntheticAtari(screen_size=64, episode_length=EP_LEN, seed=s)
            env.reset(seed=s)
            rng = np.random.default_rng(100 + s)
            r_ep = 0.0
            for _ in range(EP_LEN):
                _, r, term, trunc, _ = env.step(policy(env, rng))
                r_ep += r
                if term or trunc:
                    break
            tot.append(r_ep)
        return float(np.mean(tot)), float(np.std(tot))

    def chase(env, rng):
        p0 = np.array(env._pos[0])
        d = np.array(env._pos[1:]) - p0
        dx, dy = np.sign(d[np.argmin(np.abs(d).sum(1))]).astype(int)
        return (dy + 1) * 3 + (dx + 1)

    return run(lambda env, rng: int(rng.integers(9))), run(chase)


def main():
    os.makedirs("gpurun_out", exist_ok=True)
    (rm, rs), (cm, cs) = baselines()
    root = os.path.abspath("gpurun_out/dv3atari_run")
    args = ["exp=dreamer_v3_100k_ms_pacman", "env=synthetic_atari", "fabric=mi355x", "fabric.devices=1",
            f"total_steps={TOTAL}", "algo.learning_starts=1024", "metric.log_every=1000", "checkpoint.every=100000000",
            "env.sync_env=True", "env.capture_video=False", "cnn_keys.encoder=[rgb]", "cnn_keys.decoder=[rgb]",
            f"env.wrapper.episode_length={EP_LEN}", "seed=7", f"root_dir={root}", "run_name=atari"]
    t0 = time.perf_counter()
    with open("gpurun_out/dv3atari.log", "w") as log:
        rc = subprocess.run([sys.executable, "-u", "sheeprl.py"] + args, stdout=log, stderr=subprocess.STDOUT).returncode
    wall = time.perf_counter() - t0
    files = sorted(glob.glob(f"{root}/atari/version_*/metrics.jsonl"))
    rows = [json.loads(line) for line in open(files[-1])] if files else []
    subprocess.run(["rm", "-rf", root])  # replay memmaps / checkpoints: too large to copy back
    if rc != 0:
        print("".join(open("gpurun_out/dv3atari.log").readlines()[-40:]))
        raise SystemExit(f"run failed with exit code {rc}")
    curve = [(r["step"], r["Rewards/rew_avg"]) for r in rows if "Rewards/rew_avg" in r]
    loss = [(r["step"], r.get("Loss/world_model_loss"), r.get("Loss/policy_loss"), r.get("Loss/observation_loss"))
            for r in rows if "Loss/world_model_loss" in r]
    sps = [(r["step"], r.get("Time/sps_train")) for r in rows if "Time/sps_train" in r]
    lines = [f"# DreamerV3 from pixels: synthetic Atari, {EP_LEN}-step episodes (GPU fast path, CLI; {TOTAL} policy steps)\n",
             f"Episode return baselines on this env (20 episodes, host): random policy {rm:.1f} +- {rs:.1f}; "
             f"chase-the-nearest-sprite heuristic {cm:.1f} +- {cs:.1f}.\n",
             f"Run: `python sheeprl.py {' '.join(a for a in args if not a.startswith('root_dir'))}`; "
             f"{wall:.1f} s wall-clock incl. start-up and capture.\n",
             "| policy step | Rewards/rew_avg |", "|---:|---:|"]
    lines += [f"| {s} | {r:.1f} |" for s, r in curve]
    lines += ["", "## losses\n", "| policy step | world model | policy | observation |", "|---:|---:|---:|---:|"]
    lines += [f"| {s} | {a:.4f} | {b:.4f} | {c:.4f} |" for s, a, b, c in loss if None not in (a, b, c)]
    lines += ["", "## training throughput\n", "| policy step | Time/sps_train |", "|---:|---:|"]
    lines += [f"| {s} | {v} |" for s, v in sps]
    open(OUT, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[:6 + len(curve)]))
    print(json.dumps({"random": rm, "chase": cm, "best_rew_avg": max((r for _, r in curve), default=None),
                      "final_rew_avg": curve[-1][1] if curve else None, "wall_s": round(wall, 1)}))


if __name__ == "__main__":
    main()
