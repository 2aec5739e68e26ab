"""DroQ agent (reference ``sheeprl/algos/droq/agent.py``): the batched critic ensemble keeps the
reference's per-critic API - member i's Q value, target Q value and target EMA - as views of member i."""
import copy

import pytest
import torch

from sheeprl_prey_amd.algos.droq.agent import DROQAgent, DROQCritic, build_agent
from sheeprl_prey_amd.algos.sac.agent import SACCriticEnsemble
from sheeprl_prey_amd.config.compose import compose
from sheeprl_prey_amd.envs import spaces
from sheeprl_prey_amd.parallel.runner import Runner
from sheeprl_prey_amd.utils.utils import dotdict


def _agent(dropout=0.01, n=2):
    cfg = dotdict(compose(["exp=droq", "fabric.accelerator=cpu", f"algo.critic.dropout={dropout}",
                           f"algo.critic.n={n}", "algo.critic.hidden_size=16", "algo.actor.hidden_size=16"]))
    torch.manual_seed(0)
    runner = Runner(**dict(cfg.fabric))
    return build_agent(runner, cfg, 5, spaces.Box(-1.0, 1.0, (2,))), cfg


def test_build_agent_uses_dropout_layernorm_critics():
    agent, cfg = _agent(dropout=0.05, n=3)
    assert isinstance(agent, DROQAgent) and isinstance(agent.critic, DROQCritic)
    assert agent.num_critics == 3 and agent.critics is agent.critic
    assert agent.critic.model.dropout == pytest.approx(0.05)
    assert agent.critic.model.norms is not None and len(agent.critic.model.norms) == 2
    with pytest.raises(TypeError):
        DROQAgent(agent.actor, SACCriticEnsemble(7, n=2, hidden_size=16), target_entropy=-2.0)


def test_ith_q_values_are_ensemble_columns():
    agent, _ = _agent(dropout=0.0, n=3)
    agent.eval()
    obs, act = torch.randn(8, 5), torch.rand(8, 2) * 2 - 1
    q = agent.get_q_values(obs, act)
    qt = agent.get_target_q_values(obs, act)
    assert q.shape == (8, 3)
    for i in range(3):
        torch.testing.assert_close(agent.get_ith_q_value(obs, act, i), q[:, i : i + 1])
        torch.testing.assert_close(agent.get_ith_target_q_value(obs, act, i), qt[:, i : i + 1])
    with pytest.raises(ValueError):
        agent.get_ith_q_value(obs, act, 3)


def test_per_critic_target_ema_moves_only_that_member():
    agent, _ = _agent(dropout=0.0, n=2)
    with torch.no_grad():
        for p in agent.critic.parameters():
            p.add_(1.0)
    before = copy.deepcopy(agent.critic_target.state_dict())
    agent.qfs_target_ema(critic_idx=1)
    tau = agent.tau
    for (name, tp), p in zip(agent.critic_target.named_parameters(), agent.critic.parameters()):
        old = before[name]
        torch.testing.assert_close(tp[0], old[0])  # member 0 untouched
        torch.testing.assert_close(tp[1], old[1] + tau * (p[1] - old[1]))
    # all members at once == each member in turn
    a2 = copy.deepcopy(agent)
    agent.qfs_target_ema()
    a2.qfs_target_ema(critic_idx=0)
    a2.qfs_target_ema(critic_idx=1)
    for tp, tp2 in zip(agent.critic_target.parameters(), a2.critic_target.parameters()):
        torch.testing.assert_close(tp, tp2)
