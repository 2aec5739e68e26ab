"""DreamerV1 (reference: ``sheeprl/algos/dreamer_v1/dreamer_v1.py:30-798``).

Gradient step as a ``PhasedStep`` (hipGraph on one GPU, per-phase graphs + RCCL on N):
  wm     : encoder -> Gaussian RSSM scan -> decoder / reward heads, free-nats KL loss
  behave : world-model Adam step, differentiable imagination, actor loss -mean(discount * lambda)
           (backpropagated through the world model into the actor only)
  critic : actor Adam step, unit-Normal critic NLL on detached lambda targets
  final  : critic Adam step
"""
from __future__ import annotations

from typing import Any, Dict, List, Sequence

import torch
from torch import Tensor

from sheeprl_prey_amd.algos.common import action_info, build_envs, check_obs_keys, load_resume, setup_logger
from sheeprl_prey_amd.algos.dreamer_loop import DreamerSpec, build_replay, restore_rb, run_dreamer_loop
from sheeprl_prey_amd.algos.dreamer_v1.agent import PlayerDV1, build_models
from sheeprl_prey_amd.algos.dreamer_v1.loss import actor_loss, critic_loss, reconstruction_loss
from sheeprl_prey_amd.algos.dreamer_v1.utils import compute_lambda_values, test
from sheeprl_prey_amd.algos.dreamer_v2.dreamer_v2 import check_keys
from sheeprl_prey_amd.parallel.flat_optim import build_optimizer
from sheeprl_prey_amd.parallel.graphs import PhasedStep
from sheeprl_prey_amd.utils.metric import MeanMetric, MetricAggregator
from sheeprl_prey_amd.utils.registry import register_algorithm

METRIC_KEYS = (
    "Loss/world_model_loss", "Loss/value_loss", "Loss/policy_loss", "Loss/observation_loss", "Loss/reward_loss",
    "Loss/state_loss", "Loss/continue_loss", "State/kl", "State/post_entropy", "State/prior_entropy",
    "Grads/world_model", "Grads/actor", "Grads/critic",
)


def normal_entropy(std: Tensor) -> Tensor:
    return (0.5 + 0.5 * torch.log(2 * torch.pi * std.pow(2))).sum(-1)


class DreamerV1Trainer:
    def __init__(self, runner, cfg, world_model, actor, critic, world_optimizer, actor_optimizer, critic_optimizer):
        self.runner, self.cfg = runner, cfg
        self.world_model, self.actor, self.critic = world_model, actor, critic
        self.world_optimizer, self.actor_optimizer, self.critic_optimizer = world_optimizer, actor_optimizer, critic_optimizer
        self.wm_params = [p for p in world_model.parameters() if p.requires_grad]
        self.actor_params = [p for p in actor.parameters() if p.requires_grad]
        self.critic_params = [p for p in critic.parameters() if p.requires_grad]
        self._st: Dict[str, Any] = {}
        self.detach_heads = False  # Plan2Explore trains the reward/continue heads on detached latents
        self.step = PhasedStep(runner, [self._phase_wm, self._phase_behaviour, self._phase_critic, self._phase_final],
                               [self._coll(world_optimizer, True), self._coll(actor_optimizer), self._coll(critic_optimizer)],
                               graphs=bool(cfg.fabric.get("cuda_graphs", False)), name="dreamer_v1_train")

    def _coll(self, opt, faults: bool = False):
        def f(dry: bool = False):
            if not dry:
                self.runner.sync_gradients(opt, faults=faults)
        return f

    def train_step(self, data: Dict[str, Tensor]) -> Dict[str, Tensor]:
        return self.step(data)

    def _clip(self, module, opt, clip) -> Tensor:
        if clip is not None and clip > 0:
            return self.runner.clip_gradients(module, opt, max_norm=clip).detach()
        return torch.zeros((), device=opt.device)

    def _phase_wm(self, data: Dict[str, Tensor]) -> None:
        cfg, st = self.cfg, self._st
        wm = self.world_model
        wm_cfg = cfg.algo.world_model
        T, B = data["rewards"].shape[:2]
        S, R = wm_cfg.stochastic_size, wm_cfg.recurrent_model.recurrent_state_size
        dev = data["rewards"].device
        batch_obs = {k: data[k] / 255.0 - 0.5 for k in cfg.cnn_keys.encoder}
        batch_obs.update({k: data[k] for k in cfg.mlp_keys.encoder})
        embedded = wm.encoder(batch_obs)
        h = torch.zeros(1, B, R, device=dev)
        post = torch.zeros(1, B, S, device=dev)
        hs, posts, pm, ps, qm, qs = [], [], [], [], [], []
        for i in range(T):
            h, post, _, (m1, s1), (m2, s2) = wm.rssm.dynamic(post, h, data["actions"][i : i + 1], embedded[i : i + 1])
            hs.append(h)
            posts.append(post)
            pm.append(m1)
            ps.append(s1)
            qm.append(m2)
            qs.append(s2)
        recurrent_states, posteriors = torch.cat(hs), torch.cat(posts)
        post_mean, post_std, prior_mean, prior_std = torch.cat(pm), torch.cat(ps), torch.cat(qm), torch.cat(qs)
        latent = torch.cat((posteriors, recurrent_states), -1)
        recon = wm.observation_model(latent)
        head_in = latent.detach() if self.detach_heads else latent
        reward_mean = wm.reward_model(head_in)
        cont_logits = cont_targets = None
        if wm_cfg.use_continues and wm.continue_model is not None:
            cont_logits = wm.continue_model(head_in)
            cont_targets = (1 - data["dones"]) * cfg.algo.gamma
        rec_loss, kl, state_loss, reward_loss, obs_loss, cont_loss = reconstruction_loss(
            recon, batch_obs, reward_mean, data["rewards"], post_mean, post_std, prior_mean, prior_std,
            wm_cfg.kl_free_nats, wm_cfg.kl_regularizer, cont_logits, cont_targets, wm_cfg.continue_scale_factor)
        self.world_optimizer.zero_grad()
        rec_loss.backward(inputs=self.wm_params)
        st["embedded"] = embedded.detach()
        st["out"] = {
            "Loss/world_model_loss": rec_loss.detach(), "Loss/observation_loss": obs_loss.detach(),
            "Loss/reward_loss": reward_loss.detach(), "Loss/state_loss": state_loss.detach(),
            "Loss/continue_loss": cont_loss.detach(), "State/kl": kl.detach(),
            "State/post_entropy": normal_entropy(post_std.detach()).mean(),
            "State/prior_entropy": normal_entropy(prior_std.detach()).mean(),
        }
        st["posteriors"] = posteriors.detach()
        st["recurrent_states"] = recurrent_states.detach()

    def _wm_step(self) -> None:
        self._st["out"]["Grads/world_model"] = self._clip(self.world_model, self.world_optimizer,
                                                          self.cfg.algo.world_model.clip_gradients)
        self.world_optimizer.step()

    def _phase_behaviour(self, data: Dict[str, Tensor]) -> None:
        self._wm_step()
        self._behaviour(self.actor, self.critic, self.actor_optimizer, self.actor_params, "")

    def _behaviour(self, actor, critic, actor_optimizer, actor_params, tag: str, reward_fn=None) -> None:
        """Differentiable imagination with ``actor``; actor loss -mean(discount*lambda) backpropagated
        through the world model into ``actor_params`` only (reference ``dreamer_v1.py:137-180``)."""
        cfg, st = self.cfg, self._st
        wm = self.world_model
        wm_cfg = cfg.algo.world_model
        trajectories, imagined_actions = imagine(wm, actor, st["posteriors"], st["recurrent_states"], cfg.algo.horizon)
        values = critic(trajectories)
        rewards = reward_fn(trajectories, imagined_actions) if reward_fn is not None else wm.reward_model(trajectories)
        if wm_cfg.use_continues and wm.continue_model is not None:
            continues = torch.sigmoid(wm.continue_model(trajectories))
        else:
            continues = torch.ones_like(rewards.detach()) * cfg.algo.gamma
        lambda_values = compute_lambda_values(rewards, values, continues, last_values=values[-1],
                                              horizon=cfg.algo.horizon, lmbda=cfg.algo.lmbda)
        with torch.no_grad():
            discount = torch.cumprod(torch.cat((torch.ones_like(continues[:1]), continues[:-2]), 0), 0)
        actor_optimizer.zero_grad()
        policy_loss = actor_loss(discount * lambda_values)
        policy_loss.backward(inputs=actor_params)
        st["out"]["Loss/policy_loss" + tag] = policy_loss.detach()
        st["trajectories" + tag] = trajectories.detach()
        st["lambda_values" + tag] = lambda_values.detach()
        st["values" + tag] = values.detach()
        st["discount" + tag] = discount

    def _critic_loss(self, critic, critic_params, tag: str) -> Tensor:
        st = self._st
        qv = critic(st["trajectories" + tag])[:-1]
        value_loss = critic_loss(qv, st["lambda_values" + tag], st["discount" + tag][..., 0])
        value_loss.backward(inputs=critic_params)
        return value_loss.detach()

    def _phase_critic(self, data: Dict[str, Tensor]) -> None:
        cfg, st = self.cfg, self._st
        st["out"]["Grads/actor"] = self._clip(self.actor, self.actor_optimizer, cfg.algo.actor.clip_gradients)
        self.actor_optimizer.step()
        self.critic_optimizer.zero_grad()
        st["out"]["Loss/value_loss"] = self._critic_loss(self.critic, self.critic_params, "")

    def _phase_final(self, data: Dict[str, Tensor]) -> Dict[str, Tensor]:
        st = self._st
        st["out"]["Grads/critic"] = self._clip(self.critic, self.critic_optimizer, self.cfg.algo.critic.clip_gradients)
        self.critic_optimizer.step()
        return dict(st["out"])


def imagine(wm, actor, posteriors: Tensor, recurrent_states: Tensor, horizon: int):
    """DreamerV1 imagination: ``[H, N, L]`` latents (start state excluded) and the ``[H, N, A]``
    actions that produced them."""
    S, R = posteriors.shape[-1], recurrent_states.shape[-1]
    prior = posteriors.reshape(1, -1, S)
    h = recurrent_states.reshape(1, -1, R)
    latent = torch.cat((prior, h), -1)
    traj: List[Tensor] = []
    acts: List[Tensor] = []
    for _ in range(horizon):
        actions = torch.cat(actor(latent.detach())[0], dim=-1)
        acts.append(actions[0])
        prior, h = wm.rssm.imagination(prior, h, actions)
        latent = torch.cat((prior, h), -1)
        traj.append(latent[0])
    return torch.stack(traj), torch.stack(acts)


@register_algorithm()
def main(runner, cfg: Dict[str, Any]):
    cfg, state = load_resume(runner, cfg)
    device = runner.device
    rank, world_size = runner.global_rank, runner.world_size
    runner.seed_everything(cfg.seed + rank)
    cfg.env.screen_size = 64
    cfg.env.frame_stack = 1

    logger, log_dir = setup_logger(runner, cfg)
    envs = build_envs(runner, cfg, log_dir)
    obs_space = envs.single_observation_space
    is_continuous, _, actions_dim = action_info(envs.single_action_space)
    check_obs_keys(cfg, obs_space)
    check_keys(cfg)
    world_model, actor, critic = build_models(runner, actions_dim, is_continuous, cfg, obs_space,
                                              state["world_model"] if state else None,
                                              state["actor"] if state else None, state["critic"] if state else None)
    player = PlayerDV1(world_model.encoder, world_model.rssm.recurrent_model, world_model.rssm.representation_model,
                       actor, actions_dim, cfg.algo.player.expl_amount, cfg.env.num_envs,
                       cfg.algo.world_model.stochastic_size, cfg.algo.world_model.recurrent_model.recurrent_state_size,
                       device, min_std=cfg.algo.world_model.min_std)
    world_optimizer = build_optimizer(cfg.algo.world_model.optimizer, world_model.parameters())
    actor_optimizer = build_optimizer(cfg.algo.actor.optimizer, actor.parameters())
    critic_optimizer = build_optimizer(cfg.algo.critic.optimizer, critic.parameters())
    if state:
        world_optimizer.load_state_dict(state["world_optimizer"])
        actor_optimizer.load_state_dict(state["actor_optimizer"])
        critic_optimizer.load_state_dict(state["critic_optimizer"])
    trainer = DreamerV1Trainer(runner, cfg, world_model, actor, critic, world_optimizer, actor_optimizer,
                               critic_optimizer)
    aggregator = MetricAggregator({n: MeanMetric(sync_on_compute=cfg.metric.sync_on_compute) for n in (
        "Rewards/rew_avg", "Game/ep_len_avg", "Params/exploration_amout", *METRIC_KEYS)})
    buffer_size = cfg.buffer.size // int(cfg.env.num_envs * world_size) if not cfg.dry_run else 4
    cfg.buffer.type = "sequential"
    rb, btype = build_replay(cfg, runner, log_dir, buffer_size)
    if state and cfg.buffer.checkpoint:
        restore_rb(rb, state, runner)
    spec = DreamerSpec(
        variant="dv1", player=player, train_step=trainer.train_step,
        checkpoint_state=lambda: {
            "world_model": world_model.state_dict(), "actor": actor.state_dict(), "critic": critic.state_dict(),
            "world_optimizer": world_optimizer.state_dict(), "actor_optimizer": actor_optimizer.state_dict(),
            "critic_optimizer": critic_optimizer.state_dict()},
        test=lambda: test(player, runner, cfg, log_dir), actor_cls_name=str(cfg.env.id))
    run_dreamer_loop(runner, cfg, state, envs, spec, aggregator, rb, btype, actions_dim, is_continuous, log_dir,
                     expl_decay_steps=state["expl_decay_steps"] if state else 0)
