"""Time DreamerV3 train steps (world model + actor + critic, hipGraph-captured) for any preset on
synthetic data - e.g. the XL Crafter model the 100k bench does not cover.

    python scripts/dv3_step_bench.py exp=dreamer_v3_XL_crafter [overrides] --actions 17 --steps 10
    python scripts/dv3_step_bench.py exp=dreamer_v3_prey --vector 14 --actions 100     (vector observations)
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--actions", type=int, default=17)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--vector", type=int, default=0, help="vector observation size (0: 64x64 rgb frames)")
    ap.add_argument("--marker", action="store_true", help="a sleep kernel before the timed steps (scripts/trace_window.py)")
    ap.add_argument("overrides", nargs="*")
    a = ap.parse_args()
    from sheeprl_prey_amd.algos.dreamer_v3.agent import build_models
    from sheeprl_prey_amd.algos.dreamer_v3.dreamer_v3 import DreamerV3Trainer
    from sheeprl_prey_amd.algos.dreamer_v3.utils import Moments
    from sheeprl_prey_amd.config.compose import compose
    from sheeprl_prey_amd.envs import spaces
    from sheeprl_prey_amd.parallel.flat_optim import build_optimizer
    from sheeprl_prey_amd.parallel.runner import Runner
    from sheeprl_prey_amd.utils.utils import dotdict

    keys = (["cnn_keys.encoder=[]", "cnn_keys.decoder=[]", "mlp_keys.encoder=[state]", "mlp_keys.decoder=[state]"] if a.vector
            else ["cnn_keys.encoder=[rgb]", "cnn_keys.decoder=[rgb]", "mlp_keys.encoder=[]", "mlp_keys.decoder=[]"])
    cfg = dotdict(compose(list(a.overrides) + keys + ["fabric.accelerator=cuda", "fabric.cuda_graphs=True"]))
    runner = Runner(**dict(cfg.fabric))
    runner._init_distributed()  # device + TunableOp mode (fabric.tunable_gemm), as the CLI's launch does
    torch.manual_seed(0)
    obs_space = spaces.Dict({"state": spaces.Box(-10, 10, (a.vector,), "float32")} if a.vector else
                            {"rgb": spaces.Box(0, 255, (3, 64, 64), "uint8")})
    A = a.actions
    wm, actor, critic, target = build_models(runner, [A], False, cfg, obs_space)
    opts = [build_optimizer(c, m.parameters()) for c, m in
            ((cfg.algo.world_model.optimizer, wm), (cfg.algo.actor.optimizer, actor), (cfg.algo.critic.optimizer, critic))]
    tr = DreamerV3Trainer(runner, cfg, wm, actor, critic, target, *opts, Moments(None).cuda(), False, [A])
    T, B = cfg.per_rank_sequence_length, cfg.per_rank_batch_size
    g = torch.Generator(device="cuda").manual_seed(1)
    data = {
        **({"state": torch.randn(T, B, a.vector, device="cuda", generator=g)} if a.vector else
           {"rgb": torch.randint(0, 255, (T, B, 3, 64, 64), dtype=torch.uint8, device="cuda", generator=g)}),
        "actions": torch.nn.functional.one_hot(torch.randint(0, A, (T, B), device="cuda", generator=g), A).float(),
        "rewards": torch.randn(T, B, 1, device="cuda", generator=g),
        "dones": torch.zeros(T, B, 1, device="cuda"),
        "is_first": torch.zeros(T, B, 1, device="cuda"),
    }
    n_params = sum(p.numel() for m in (wm, actor, critic) for p in m.parameters())
    for _ in range(a.warmup):
        out = tr.train_step(data)
    torch.cuda.synchronize()
    if a.marker:
        torch.cuda._sleep(1000)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        out = tr.train_step(data)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    print(f"{a.overrides}: params {n_params / 1e6:.1f}M  B{B} T{T}  {dt * 1e3:.2f} ms/train step  "
          f"wm_loss {float(out['Loss/world_model_loss']):.3f}  graphed {tr.graphed.graph is not None}", flush=True)


if __name__ == "__main__":
    main()
