"""Device-resident CartPole (envs/device.py) against the host CartPoleEnv dynamics, autoreset and
time-limit semantics; the HIP kernel against the torch path on GPU."""
import numpy as np
import pytest
import torch

from sheeprl_prey_amd.envs.classic import CartPoleEnv
from sheeprl_prey_amd.envs.device import CartPoleDevice


def _run_host(state0, actions):
    env = CartPoleEnv()
    env.reset(seed=0)
    env.state = tuple(float(v) for v in state0)
    out = []
    for a in actions:
        o, r, term, trunc, _ = env.step(int(a))
        out.append((o, r, term))
        if term:
            break
    return out


def test_device_cartpole_matches_host_dynamics():
    rng = np.random.default_rng(0)
    dev = CartPoleDevice(3, "cpu", max_episode_steps=500)
    dev.reset(seed=1)
    state0 = dev.state.clone().numpy()
    acts = rng.integers(0, 2, size=(60, 3))
    hosts = [_run_host(state0[i], acts[:, i]) for i in range(3)]
    for t in range(60):
        out = dev.step(torch.as_tensor(acts[t]))
        for i in range(3):
            if t < len(hosts[i]):
                o, r, term = hosts[i][t]
                np.testing.assert_allclose(out["final_obs"][i].numpy(), o, rtol=1e-5, atol=1e-6)
                assert out["reward"][i].item() == r
                assert bool(out["terminated"][i].item()) == term
                if term:  # autoreset: next obs is a fresh small state, episode stats reported
                    assert out["obs"][i].abs().max().item() <= 0.05
                    assert out["done_len"][i].item() == t + 1
                    assert out["done_ret"][i].item() == t + 1


def test_device_cartpole_time_limit_truncates():
    dev = CartPoleDevice(2, "cpu", max_episode_steps=5)
    dev.reset(seed=0)
    for t in range(5):
        out = dev.step(torch.tensor([0, 1]))
        # the pole cannot fall within 5 steps from |state| <= 0.05
    assert out["truncated"].tolist() == [1.0, 1.0]
    assert out["terminated"].tolist() == [0.0, 0.0]
    assert out["done_len"].tolist() == [5.0, 5.0]
    assert dev.steps.tolist() == [0, 0]


@pytest.mark.gpu
def test_device_cartpole_kernel_matches_torch_path():
    cpu = CartPoleDevice(257, "cpu")
    gpu = CartPoleDevice(257, "cuda")
    cpu.reset(seed=3)
    gpu.state.copy_(cpu.state)
    gpu.obs.copy_(cpu.obs)
    g = torch.Generator().manual_seed(0)
    for t in range(80):
        a = torch.randint(0, 2, (257,), generator=g)
        u = torch.rand(257, 4, generator=g)
        cpu._step_torch(a, u)
        from sheeprl_prey_amd import ops

        ops._ext().cartpole_step(gpu.state, gpu.steps, gpu.ep_ret, a.cuda(), u.cuda(), gpu.obs, gpu.reward, gpu.terminated,
                                 gpu.truncated, gpu.final_obs, gpu.done_ret, gpu.done_len, gpu.max_steps)
        torch.testing.assert_close(gpu.state.cpu(), cpu.state, rtol=1e-4, atol=1e-5)
        for k in ("reward", "terminated", "truncated", "done_ret", "done_len"):
            torch.testing.assert_close(getattr(gpu, k).cpu(), getattr(cpu, k))


def _ppo_setup(n_envs, T, max_steps, units=64):
    from sheeprl_prey_amd.algos.ppo.agent import PPOAgent
    from sheeprl_prey_amd.config.compose import compose
    from sheeprl_prey_amd.utils.utils import dotdict

    cfg = dotdict(compose(["exp=ppo", "mlp_keys.encoder=[state]", f"algo.rollout_steps={T}", f"env.num_envs={n_envs}",
                           f"algo.dense_units={units}", f"algo.encoder.mlp_features_dim={units}"]))
    env = CartPoleDevice(n_envs, "cuda", max_episode_steps=max_steps, seed=0)
    env.reset(seed=0)
    torch.manual_seed(0)
    agent = PPOAgent([2], env.single_observation_space, cfg.algo.encoder, cfg.algo.actor, cfg.algo.critic, [], ["state"],
                     cfg.env.screen_size, cfg.distribution, False).cuda()
    return cfg, env, agent


@pytest.mark.gpu
# (LDS-staged weights, layer width): register-resident kernel (<= 64), LDS-activation kernel (> 64),
# global-memory weights
@pytest.mark.parametrize("lds_weights,units", [(True, 64), (True, 128), (False, 64)])
def test_fused_ppo_rollout_matches_policy_and_dynamics(lds_weights, units):
    """One-launch rollout kernel (ops/csrc/ppo_rollout.hip): log-probs / values against the torch
    agent on the stored states, env transitions against the torch CartPole step, truncation
    bootstrap r = 1 + V(final_obs), and sampled actions distributed as the policy."""
    from sheeprl_prey_amd.algos.ppo.ppo import FusedCartPoleRollout

    N, T = 98, 48  # not a multiple of the 4 envs per workgroup
    cfg, env, agent = _ppo_setup(N, T, max_steps=20, units=units)
    assert FusedCartPoleRollout.supported(agent, env)
    ro = FusedCartPoleRollout(agent, env, cfg, seed=1, lds_weights=lds_weights)
    obs0 = env.obs.clone()
    buf = {k: v.clone() for k, v in ro().items()}
    torch.cuda.synchronize()
    torch.testing.assert_close(buf["state"][0], obs0)
    a = buf["actions"]
    assert torch.all((a == 0) | (a == 1)) and torch.all(a.sum(-1) == 1)
    idx = a.argmax(-1)  # [T, N]
    with torch.no_grad():
        feat = agent.feature_extractor({"state": buf["state"]})
        logits = agent.actor_heads[0](agent.actor_backbone(feat))
        values = agent.critic(feat)
    logp_all = torch.log_softmax(logits, -1)
    torch.testing.assert_close(buf["logprobs"][..., 0], logp_all.gather(-1, idx[..., None])[..., 0], rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(buf["values"], values, rtol=1e-4, atol=1e-4)
    # sampling law: mean P(a=1) over all draws vs the empirical frequency (2σ ≈ 0.015 here)
    assert abs(logp_all[..., 1].exp().mean().item() - idx.float().mean().item()) < 0.05
    # dynamics, autoreset, truncation
    sim = CartPoleDevice(N, "cpu", max_episode_steps=10**9)
    n_trunc = 0
    for t in range(T - 1):
        sim.state.copy_(buf["state"][t].cpu())
        sim._step_torch(idx[t].cpu(), torch.zeros(N, 4))
        done = buf["dones"][t, :, 0].cpu() > 0
        live = ~done
        torch.testing.assert_close(buf["state"][t + 1].cpu()[live], sim.final_obs[live], rtol=1e-4, atol=1e-5)
        assert torch.all(buf["state"][t + 1].cpu()[done].abs() <= 0.05)
        trunc = done & (sim.terminated == 0)
        term = done & (sim.terminated > 0)
        assert torch.all(buf["rewards"][t, :, 0].cpu()[~trunc] == 1.0)
        if trunc.any():
            n_trunc += int(trunc.sum())
            with torch.no_grad():
                vf = agent.get_value({"state": sim.final_obs[trunc].cuda()})[:, 0].cpu()
            torch.testing.assert_close(buf["rewards"][t, :, 0].cpu()[trunc], 1.0 + vf, rtol=1e-4, atol=1e-4)
            assert torch.all(ro.stats["done_len"][t].cpu()[trunc] == 20)
        assert torch.all((ro.stats["done_len"][t].cpu() > 0) == done)
        assert torch.all(ro.stats["done_len"][t].cpu()[term] <= 20)
    assert n_trunc > 0  # the 20-step limit was exercised
    # continuity across launches: the next rollout starts where this one left the envs
    last = env.obs.clone()
    buf2 = ro()
    torch.testing.assert_close(buf2["state"][0], last)
