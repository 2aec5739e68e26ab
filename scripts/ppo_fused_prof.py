"""Fused PPO update (ops/csrc/ppo_train.hip): ms per update and workgroup-0 phase cycles for 1..8 workgroups."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import torch, time
from tests.test_ppo_fused_gpu import _Runner
from sheeprl_prey_amd.algos.ppo.agent import PPOAgent
from sheeprl_prey_amd.algos.ppo.ppo import FusedPPOTrainer
from sheeprl_prey_amd.config.compose import compose
from sheeprl_prey_amd.envs.device import CartPoleDevice
from sheeprl_prey_amd.parallel.flat_optim import build_optimizer
from sheeprl_prey_amd.utils.utils import dotdict
cfg = dotdict(compose(["exp=ppo", "mlp_keys.encoder=[state]", "fabric.accelerator=cuda"]))
agent = PPOAgent([2], CartPoleDevice.single_observation_space, cfg.algo.encoder, cfg.algo.actor, cfg.algo.critic, [], ["state"], 64, cfg.distribution, False).cuda()
opt = build_optimizer(cfg.algo.optimizer, agent.parameters())
r = _Runner(); n = 128
f = FusedPPOTrainer(r, agent, opt, cfg, n, FusedPPOTrainer.plan(r, agent, opt, cfg))
d = {"state": torch.randn(n, 4, device="cuda"), "actions": torch.nn.functional.one_hot(torch.randint(0, 2, (n,), device="cuda"), 2).float(),
     "logprobs": -0.7 * torch.ones(n, 1, device="cuda"), "values": torch.randn(n, 1, device="cuda"), "returns": torch.randn(n, 1, device="cuda"),
     "advantages": torch.randn(n, 1, device="cuda")}
f.prof = torch.zeros(4, dtype=torch.int64, device="cuda")
for nwg in (1, 2, 4, 8):
    f.nwg = nwg
    for _ in range(3): f(d)
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(20): f(d)
    torch.cuda.synchronize(); dt = (time.perf_counter() - t) / 20 * 1e3
    print(f"nwg={nwg}: {dt:.3f} ms/update; wg0 cycles per update chunk/publish+bar/reduce+adam/bar+reload:", [int(x) for x in f.prof.tolist()], "err", f.err.item())
