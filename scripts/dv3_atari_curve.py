"""DreamerV3 learning curve from PIXELS through the real CLI on the GPU fast path (HIP conv stack, persistent scan,
fused heads, captured train step): the Atari-100k recipe (``exp=dreamer_v3_100k_ms_pacman``) on the synthetic
Atari env (``envs/synthetic.py``: the action moves sprite 0 on a 3x3 stencil, every other sprite it touches is a
reward of 1 and respawns), 250-step episodes.  On this env a random policy scores 13.8 +- 4.4 per episode and a
hand-written "chase the nearest sprite" policy 89.1 +- 9.8 (20 episodes each, computed by this script on the host).

With ``--walker``: the continuous path instead (``exp=dreamer_v3_dmc_walker_walk`` on the walker_walk-shaped
synthetic control env: 64x64 renders + 24-dim state, 6-dim TruncatedNormal actions, 1000-step episodes, the
imagination back-propagating through the dynamics in ``imagine_cont.py``); host baselines: uniform random actions,
zero actions, and the one-step greedy action sign(B^T w) of the env's own linear system.

With ``--prey``: the fork's own preset (``exp=dreamer_v3_prey``) on the predator-prey cellworld ``prey_d_1``
(``envs/prey``: vector observation, Discrete(100) speed x turning actions, -distance per step, +100 at the goal,
-50 on capture); host baseline: a uniform random policy (100 episodes).

usage: python scripts/dv3_atari_curve.py <out.md> [total_policy_steps] [--walker | --prey]"""
import glob
import json
import os
import subprocess
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

WALKER = "--walker" in sys.argv
PREY = "--prey" in sys.argv
_pos = [a for a in sys.argv[1:] if not a.startswith("--")]
OUT = _pos[0] if len(_pos) > 0 else "gpurun_out/dv3_atari_curve.md"
TOTAL = int(_pos[1]) if len(_pos) > 1 else 30000
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


def walker_baselines(eps: int = 5):
    from sheeprl_prey_amd.envs.synthetic import SyntheticControl

    def run(policy):
        tot = []
        for s in range(eps):
            env = SyntheticControl(seed=s)
            env.reset(seed=s)
            rng = np.random.default_rng(s)
            r_ep, done = 0.0, False
            while not done:
                _, r, term, trunc, _ = env.step(policy(env, rng))
                r_ep += r
                done = term or trunc
            tot.append(r_ep)
        return float(np.mean(tot)), float(np.std(tot))

    return (run(lambda env, rng: rng.uniform(-1, 1, env.act_dim)), run(lambda env, rng: np.zeros(env.act_dim)),
            run(lambda env, rng: np.sign(env._B.T @ env._w)))


def prey_baseline(eps: int = 100):
    from sheeprl_prey_amd.envs.registry import make

    env = make("prey_d_1")
    rng = np.random.default_rng(0)
    tot, goals = [], 0
    for ep in range(eps):
        env.reset(seed=ep)
        r_ep, n = 0.0, 0
        while True:
            _, r, term, trunc, _ = env.step(int(rng.integers(env.action_space.n)))
            r_ep += r
            n += 1
            if term or trunc or n >= 300:
                goals += int(term)
                break
        tot.append(r_ep)
    return float(np.mean(tot)), float(np.std(tot)), goals / eps


def main():
    os.makedirs("gpurun_out", exist_ok=True)
    if PREY:
        rm, rs, gr = prey_baseline()
        cm = None
        root = os.path.abspath("gpurun_out/dv3prey_run")
        args = ["exp=dreamer_v3_prey", "fabric=mi355x", "fabric.devices=1", f"total_steps={TOTAL}", "metric.log_every=5000",
                "checkpoint.every=100000000", "env.sync_env=True", "env.capture_video=False", "seed=7",
                f"root_dir={root}", "run_name=atari"]
        title = f"# DreamerV3 on the predator-prey cellworld prey_d_1 (exp=dreamer_v3_prey, GPU, CLI; {TOTAL} policy steps)\n"
        base = (f"Baseline (100 episodes, host): uniform random policy {rm:.1f} +- {rs:.1f} per episode, goal reached in "
                f"{100 * gr:.0f} % of episodes (captured or timed out otherwise).\n")
    elif WALKER:
        (rm, rs), (zm, zs), (cm, cs) = walker_baselines()
        root = os.path.abspath("gpurun_out/dv3walker_run")
        args = ["exp=dreamer_v3_dmc_walker_walk", "env=gym", "env.id=walker_walk_synthetic", "fabric=mi355x",
                "fabric.devices=1", f"total_steps={TOTAL}", "algo.learning_starts=1024", "metric.log_every=2000",
                "checkpoint.every=100000000", "env.sync_env=True", "env.capture_video=False", "cnn_keys.encoder=[rgb]",
                "cnn_keys.decoder=[rgb]", "mlp_keys.encoder=[state]", "mlp_keys.decoder=[state]", "buffer.memmap=False",
                "seed=7", f"root_dir={root}", "run_name=atari"]
        title = (f"# DreamerV3 continuous (pixels + state): walker_walk-shaped synthetic env, 1000-step episodes "
                 f"(GPU fast path, CLI; {TOTAL} policy steps)\n")
        base = (f"Episode return baselines on this env (5 episodes, host): uniform random actions {rm:.1f} +- {rs:.1f}; zero "
                f"actions {zm:.1f} +- {zs:.1f}; one-step greedy sign(B^T w) {cm:.1f} +- {cs:.1f}.\n")
    else:
        (rm, rs), (cm, cs) = baselines()
        root = os.path.abspath("gpurun_out/dv3atari_run")
        args = ["exp=dreamer_v3_100k_ms_pacman", "env=synthetic_atari", "fabric=mi355x", "fabric.devices=1",
                f"total_steps={TOTAL}", "algo.learning_starts=1024", "metric.log_every=1000", "checkpoint.every=100000000",
                "env.sync_env=True", "env.capture_video=False", "cnn_keys.encoder=[rgb]", "cnn_keys.decoder=[rgb]",
                f"env.wrapper.episode_length={EP_LEN}", "seed=7", f"root_dir={root}", "run_name=atari"]
        title = (f"# DreamerV3 from pixels: synthetic Atari, {EP_LEN}-step episodes (GPU fast path, CLI; {TOTAL} policy "
                 f"steps)\n")
        base = (f"Episode return baselines on this env (20 episodes, host): random policy {rm:.1f} +- {rs:.1f}; "
                f"chase-the-nearest-sprite heuristic {cm:.1f} +- {cs:.1f}.\n")
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
    lines = [title, base,
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
    print(json.dumps({"random": rm, "heuristic": cm, "best_rew_avg": max((r for _, r in curve), default=None),
                      "final_rew_avg": curve[-1][1] if curve else None, "wall_s": round(wall, 1)}))


if __name__ == "__main__":
    main()
