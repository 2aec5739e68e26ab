"""One-launch PPO update (ops/csrc/ppo_train.hip) against the eager autograd path
(``ppo.train``'s ``_minibatch_step`` loop over the same minibatch order): weights, Adam moments,
optimiser step counter and reported loss means after a full update, for the default CartPole agent
and for variants exercising advantage normalisation, value clipping, entropy bonus, global-norm
clipping, ReLU layers and a partial last minibatch."""
import copy

import pytest
import torch

from sheeprl_prey_amd.algos.ppo.agent import PPOAgent
from sheeprl_prey_amd.algos.ppo.ppo import FusedPPOTrainer, _minibatch_step
from sheeprl_prey_amd.config.compose import compose
from sheeprl_prey_amd.envs.device import CartPoleDevice
from sheeprl_prey_amd.parallel.flat_optim import build_optimizer
from sheeprl_prey_amd.utils.utils import dotdict

pytestmark = pytest.mark.gpu


class _Runner:
    device = torch.device("cuda")
    world_size = 1
    cuda_graphs = False

    def backward(self, loss, optimizer=None):
        loss.backward()

    def clip_gradients(self, module=None, optimizer=None, max_norm=1.0):
        return optimizer.clip_grad_norm_(max_norm)


CASES = {
    "default": ([], 128),
    "norm_clip_ent": (["algo.normalize_advantages=True", "algo.clip_vloss=True", "algo.ent_coef=0.01",
                       "algo.max_grad_norm=0.5", "algo.update_epochs=3"], 128),
    "relu_partial": (["algo.dense_act=torch.nn.ReLU", "algo.update_epochs=2", "algo.dense_units=32"], 100),
}


@pytest.mark.parametrize("nwg", [1, 8])
@pytest.mark.parametrize("case", list(CASES))
def test_fused_ppo_update_matches_autograd(case, nwg):
    """nwg = 1: one workgroup runs every chunk; 8: one workgroup per 16-row chunk of each minibatch
    (capped at bs / 16), grid barriers between the optimiser steps."""
    extra, n = CASES[case]
    cfg = dotdict(compose(["exp=ppo", "mlp_keys.encoder=[state]", "fabric.accelerator=cuda"] + extra))
    torch.manual_seed(0)
    obs_space = CartPoleDevice.single_observation_space
    agent_a = PPOAgent([2], obs_space, cfg.algo.encoder, cfg.algo.actor, cfg.algo.critic, [], ["state"],
                       cfg.env.screen_size, cfg.distribution, False).cuda()
    agent_b = copy.deepcopy(agent_a)
    opt_a = build_optimizer(cfg.algo.optimizer, agent_a.parameters())
    opt_b = build_optimizer(cfg.algo.optimizer, agent_b.parameters())
    runner = _Runner()
    plan = FusedPPOTrainer.plan(runner, agent_a, opt_a, cfg)
    assert plan is not None, "the exp=ppo agent must be covered by the fused update"
    g = torch.Generator(device="cuda").manual_seed(1)
    state = torch.randn(n, 4, device="cuda", generator=g)
    idx = torch.randint(0, 2, (n,), device="cuda", generator=g)
    with torch.no_grad():
        _, lp, _, val = agent_b({"state": state}, [torch.nn.functional.one_hot(idx, 2).float()])
    data = {"state": state, "actions": torch.nn.functional.one_hot(idx, 2).float(),
            "logprobs": lp + 0.05 * torch.randn(n, 1, device="cuda", generator=g),
            "values": val + 0.1 * torch.randn(n, 1, device="cuda", generator=g),
            "returns": torch.randn(n, 1, device="cuda", generator=g),
            "advantages": torch.randn(n, 1, device="cuda", generator=g)}
    E, bs = int(cfg.algo.update_epochs), int(cfg.per_rank_batch_size)
    perm = torch.argsort(torch.rand(E, n, device="cuda", generator=g), dim=1)

    fused = FusedPPOTrainer(runner, agent_a, opt_a, cfg, n, plan)
    fused.nwg = nwg
    fused(data, None, perm=perm)
    torch.cuda.synchronize()
    assert fused.err.item() == 0.0

    sums, steps = torch.zeros(3, device="cuda"), 0
    for e in range(E):
        for start in range(0, n, bs):
            sel = perm[e, start : start + bs]
            batch = {k: v.index_select(0, sel) for k, v in data.items()}
            pg, vl, el = _minibatch_step(runner, agent_b, opt_b, batch, ["state"], cfg, cfg.algo.clip_coef, cfg.algo.ent_coef)
            sums += torch.stack((pg.detach(), vl.detach(), el.detach()))
            steps += 1
    torch.cuda.synchronize()

    assert opt_a.scalars[0].item() == opt_b.scalars[0].item() == steps
    torch.testing.assert_close(fused.out, sums / steps, rtol=1e-4, atol=1e-5)
    for (na, pa), (nb, pb) in zip(agent_a.named_parameters(), agent_b.named_parameters()):
        torch.testing.assert_close(pa, pb, rtol=1e-3, atol=2e-5, msg=lambda m: f"{na}: {m}")
    torch.testing.assert_close(opt_a.exp_avg, opt_b.exp_avg, rtol=1e-3, atol=1e-6)
    torch.testing.assert_close(opt_a.exp_avg_sq, opt_b.exp_avg_sq, rtol=1e-3, atol=1e-9)
    assert opt_a.exp_avg.abs().max().item() > 0  # the update did something
