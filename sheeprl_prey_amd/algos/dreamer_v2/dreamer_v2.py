"""DreamerV2 (reference: ``sheeprl/algos/dreamer_v2/dreamer_v2.py:38-882``).

One gradient step = four phases separated by their gradient all-reduces, run as a ``PhasedStep``
(one hipGraph on a single GPU, per-phase graphs with RCCL between them on N GPUs):
  wm      : encoder -> RSSM posterior scan -> decoder / reward / continue heads, KL-balanced loss
  behave  : world-model Adam step, imagination (H steps of actor + RSSM prior), lambda returns,
            REINFORCE/dynamics actor loss
  critic  : actor Adam step, unit-Normal critic NLL on the lambda targets
  final   : critic Adam step
With ``objective_mix == 1`` (pure REINFORCE) the imagination carries no gradient the loss uses, so
it runs under ``no_grad`` (identical gradients, no imagination backward graph).
"""
from __future__ import annotations

from typing import Any, Dict, List, Sequence

import numpy as np
import torch
from torch import Tensor

from sheeprl_prey_amd import ops
from sheeprl_prey_amd.algos.common import action_info, build_envs, check_obs_keys, load_resume, setup_logger
from sheeprl_prey_amd.algos.dreamer_loop import DreamerSpec, build_replay, restore_rb, run_dreamer_loop
from sheeprl_prey_amd.algos.dreamer_v2.agent import PlayerDV2, build_models
from sheeprl_prey_amd.algos.dreamer_v2.loss import HALF_LOG_2PI, normal_nll, reconstruction_loss
from sheeprl_prey_amd.algos.dreamer_v2.utils import compute_lambda_values, test
from sheeprl_prey_amd.parallel.flat_optim import build_optimizer, flatten_like
from sheeprl_prey_amd.parallel.graphs import PhasedStep
from sheeprl_prey_amd.utils.metric import MeanMetric, MetricAggregator
from sheeprl_prey_amd.utils.registry import register_algorithm

METRIC_KEYS = (
    "Loss/world_model_loss", "Loss/value_loss", "Loss/policy_loss", "Loss/observation_loss", "Loss/reward_loss",
    "Loss/state_loss", "Loss/continue_loss", "State/kl", "State/post_entropy", "State/prior_entropy",
    "Grads/world_model", "Grads/actor", "Grads/critic",
)


def categorical_entropy(logits: Tensor) -> Tensor:
    lp = logits.log_softmax(-1)
    return -(lp.exp() * lp).sum(-1)


class DreamerV2Trainer:
    def __init__(self, runner, cfg, world_model, actor, critic, target_critic, world_optimizer, actor_optimizer,
                 critic_optimizer, is_continuous: bool, actions_dim: Sequence[int]):
        self.runner, self.cfg = runner, cfg
        self.world_model, self.actor, self.critic, self.target_critic = world_model, actor, critic, target_critic
        self.world_optimizer, self.actor_optimizer, self.critic_optimizer = world_optimizer, actor_optimizer, critic_optimizer
        self.is_continuous = is_continuous
        self.actions_dim = list(actions_dim)
        self.target_flat = flatten_like(target_critic, critic_optimizer)
        self.wm_params = [p for p in world_model.parameters() if p.requires_grad]
        self.actor_params = [p for p in actor.parameters() if p.requires_grad]
        self.critic_params = [p for p in critic.parameters() if p.requires_grad]
        self._st: Dict[str, Any] = {}
        self.detach_heads = False  # Plan2Explore trains the reward/continue heads on detached latents
        self.step = PhasedStep(runner, [self._phase_wm, self._phase_behaviour, self._phase_critic, self._phase_final],
                               [self._coll(world_optimizer, True), self._coll(actor_optimizer), self._coll(critic_optimizer)],
                               graphs=bool(cfg.fabric.get("cuda_graphs", False)), name="dreamer_v2_train")

    def _coll(self, opt, faults: bool = False):
        def f(dry: bool = False):
            if not dry:
                self.runner.sync_gradients(opt, faults=faults)
        return f

    @torch.no_grad()
    def update_target(self, tau: float = 1.0) -> None:
        """Hard copy (tau=1) of the critic into the target critic: one slab copy."""
        self.target_flat.lerp_(self.critic_optimizer.flat_param, float(tau))

    def train_step(self, data: Dict[str, Tensor]) -> Dict[str, Tensor]:
        return self.step(data)

    def _clip(self, module, opt, clip) -> Tensor:
        if clip is not None and clip > 0:
            return self.runner.clip_gradients(module, opt, max_norm=clip).detach()
        return torch.zeros((), device=opt.device)

    # ------------------------------------------------------------------ world model
    def _phase_wm(self, data: Dict[str, Tensor]) -> None:
        cfg, st = self.cfg, self._st
        wm = self.world_model
        wm_cfg = cfg.algo.world_model
        T, B = data["rewards"].shape[:2]
        stoch, disc = wm_cfg.stochastic_size, wm_cfg.discrete_size
        R = wm_cfg.recurrent_model.recurrent_state_size
        dev = data["rewards"].device
        batch_obs = {k: data[k] / 255.0 - 0.5 for k in cfg.cnn_keys.encoder}
        batch_obs.update({k: data[k] for k in cfg.mlp_keys.encoder})
        is_first = data["is_first"].clone()
        is_first[0] = 1.0
        embedded = wm.encoder(batch_obs)
        h = torch.zeros(1, B, R, device=dev)
        post = torch.zeros(1, B, stoch, disc, device=dev)
        hs, posts, post_logits, prior_logits = [], [], [], []
        for i in range(T):
            h, post, _, pl, ql = wm.rssm.dynamic(post, h, data["actions"][i : i + 1], embedded[i : i + 1],
                                                 is_first[i : i + 1])
            hs.append(h)
            posts.append(post)
            post_logits.append(pl)
            prior_logits.append(ql)
        recurrent_states = torch.cat(hs)
        posteriors = torch.cat(posts)
        posteriors_logits = torch.cat(post_logits)
        priors_logits = torch.cat(prior_logits)
        latent = torch.cat((posteriors.view(T, B, -1), recurrent_states), -1)
        recon = wm.observation_model(latent)
        head_in = latent.detach() if self.detach_heads else latent
        reward_mean = wm.reward_model(head_in)
        cont_logits = cont_targets = None
        if wm_cfg.use_continues and wm.continue_model is not None:
            cont_logits = wm.continue_model(head_in)
            cont_targets = (1 - data["dones"]) * cfg.algo.gamma
        rec_loss, kl, state_loss, reward_loss, obs_loss, cont_loss = reconstruction_loss(
            recon, batch_obs, reward_mean, data["rewards"], priors_logits, posteriors_logits, stoch, disc,
            wm_cfg.kl_balancing_alpha, wm_cfg.kl_free_nats, wm_cfg.kl_free_avg, wm_cfg.kl_regularizer,
            cont_logits, cont_targets, wm_cfg.discount_scale_factor)
        self.world_optimizer.zero_grad()
        rec_loss.backward(inputs=self.wm_params)
        st["embedded"] = embedded.detach()
        with torch.no_grad():
            out = {
                "Loss/world_model_loss": rec_loss.detach(), "Loss/observation_loss": obs_loss.detach(),
                "Loss/reward_loss": reward_loss.detach(), "Loss/state_loss": state_loss.detach(),
                "Loss/continue_loss": cont_loss.detach(), "State/kl": kl.mean().detach(),
                "State/post_entropy": categorical_entropy(posteriors_logits.view(T, B, stoch, disc)).sum(-1).mean(),
                "State/prior_entropy": categorical_entropy(priors_logits.view(T, B, stoch, disc)).sum(-1).mean(),
            }
        st["out"] = out
        st["posteriors"] = posteriors.detach()
        st["recurrent_states"] = recurrent_states.detach()

    # ------------------------------------------------------------------ imagination + actor
    def _wm_step(self) -> None:
        st = self._st
        st["out"]["Grads/world_model"] = self._clip(self.world_model, self.world_optimizer,
                                                    self.cfg.algo.world_model.clip_gradients)
        self.world_optimizer.step()

    def _phase_behaviour(self, data: Dict[str, Tensor]) -> None:
        self._wm_step()
        mix = float(self.cfg.algo.actor.objective_mix)
        self._behaviour(data, self.actor, self.target_critic, self.actor_optimizer, self.actor_params, mix, "")

    def _behaviour(self, data, actor, target_critic, actor_optimizer, actor_params, mix: float, tag: str,
                   reward_fn=None) -> None:
        """Imagine with ``actor``, build lambda targets (``reward_fn(traj, acts)`` or the reward
        model), backprop the actor loss into ``actor_params``; results stashed under ``tag``."""
        cfg, st = self.cfg, self._st
        wm = self.world_model
        wm_cfg = cfg.algo.world_model
        ctx = torch.enable_grad() if mix < 1.0 else torch.no_grad()
        with ctx:
            trajectories, imagined_actions = imagine(wm, actor, st["posteriors"], st["recurrent_states"],
                                                     cfg.algo.horizon, self.actions_dim)
            target_values = target_critic(trajectories)
            rewards = reward_fn(trajectories, imagined_actions) if reward_fn is not None else wm.reward_model(trajectories)
            if wm_cfg.use_continues and wm.continue_model is not None:
                continues = torch.sigmoid(wm.continue_model(trajectories))
                true_done = (1 - data["dones"]).reshape(1, -1, 1) * cfg.algo.gamma
                continues = torch.cat((true_done, continues[1:]))
            else:
                continues = torch.ones_like(rewards.detach()) * cfg.algo.gamma
            lambda_values = compute_lambda_values(rewards[:-1], target_values[:-1], continues[:-1],
                                                  bootstrap=target_values[-1:], horizon=cfg.algo.horizon,
                                                  lmbda=cfg.algo.lmbda)
        with torch.no_grad():
            discount = torch.cumprod(torch.cat((torch.ones_like(continues[:1]), continues[:-1]), 0), 0)
        actor_optimizer.zero_grad()
        policies = actor(trajectories[:-2].detach())[1]
        advantage = (lambda_values[1:] - target_values[:-2]).detach()
        if mix > 0.0:
            reinforce = torch.stack(
                [p.log_prob(a[1:-1].detach()).unsqueeze(-1)
                 for p, a in zip(policies, torch.split(imagined_actions, self.actions_dim, -1))], -1).sum(-1) * advantage
        objective = reinforce if mix >= 1.0 else (lambda_values[1:] if mix <= 0.0 else
                                                   mix * reinforce + (1 - mix) * lambda_values[1:])
        try:
            entropy = cfg.algo.actor.ent_coef * torch.stack([p.entropy() for p in policies], -1).sum(-1)
        except NotImplementedError:
            entropy = torch.zeros_like(objective[..., 0])
        policy_loss = -torch.mean(discount[:-2].detach() * (objective + entropy.unsqueeze(-1)))
        policy_loss.backward(inputs=actor_params)
        st["out"]["Loss/policy_loss" + tag] = policy_loss.detach()
        st["trajectories" + tag] = trajectories.detach()
        st["lambda_values" + tag] = lambda_values.detach()
        st["target_values" + tag] = target_values.detach()
        st["discount" + tag] = discount

    # ------------------------------------------------------------------ critic
    def _critic_loss(self, critic, critic_params, tag: str) -> Tensor:
        st = self._st
        qv = critic(st["trajectories" + tag][:-1])
        # -log N(lambda | qv, 1) over the 1-dim event
        value_loss = torch.mean(st["discount" + tag][:-1, ..., 0] * normal_nll(qv, st["lambda_values" + tag], 1))
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


def imagine(wm, actor, posteriors: Tensor, recurrent_states: Tensor, horizon: int, actions_dim: Sequence[int]):
    """DreamerV2 imagination from every posterior state: ``[H+1, N, L]`` latents and ``[H+1, N, A]``
    actions (action 0 is zero), reference ``dreamer_v2.py:187-212``."""
    S = posteriors.shape[-2] * posteriors.shape[-1]
    R = recurrent_states.shape[-1]
    prior = posteriors.reshape(1, -1, S)
    h = recurrent_states.reshape(1, -1, R)
    latent = torch.cat((prior, h), -1)
    traj: List[Tensor] = [latent[0]]
    acts: List[Tensor] = [torch.zeros(latent.shape[1], int(sum(actions_dim)), device=latent.device)]
    for _ in range(horizon):
        actions = torch.cat(actor(latent.detach())[0], dim=-1)
        acts.append(actions[0])
        prior, h = wm.rssm.imagination(prior, h, actions)
        prior = prior.reshape(1, -1, S)
        latent = torch.cat((prior, h), -1)
        traj.append(latent[0])
    return torch.stack(traj), torch.stack(acts)


def make_aggregator(cfg, extra=()) -> MetricAggregator:
    names = ["Rewards/rew_avg", "Game/ep_len_avg", "Params/exploration_amout", *METRIC_KEYS, *extra]
    return MetricAggregator({n: MeanMetric(sync_on_compute=cfg.metric.sync_on_compute) for n in names})


def check_keys(cfg) -> None:
    if not set(cfg.cnn_keys.encoder) & set(cfg.cnn_keys.decoder) and not set(cfg.mlp_keys.encoder) & set(cfg.mlp_keys.decoder):
        raise RuntimeError("The CNN keys or the MLP keys of the encoder and decoder must not be disjointed")
    if set(cfg.cnn_keys.decoder) - set(cfg.cnn_keys.encoder):
        raise RuntimeError("The CNN keys of the decoder must be contained in the encoder ones. "
                           f"Those keys are decoded without being encoded: {list(set(cfg.cnn_keys.decoder))}")
    if set(cfg.mlp_keys.decoder) - set(cfg.mlp_keys.encoder):
        raise RuntimeError("The MLP keys of the decoder must be contained in the encoder ones. "
                           f"Those keys are decoded without being encoded: {list(set(cfg.mlp_keys.decoder))}")


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
    for name in ("Encoder CNN", "Encoder MLP", "Decoder CNN", "Decoder MLP"):
        part, kind = name.split()
        runner.print(f"{name} keys:", cfg[f"{kind.lower()}_keys"][part.lower()])

    world_model, actor, critic, target_critic = build_models(
        runner, actions_dim, is_continuous, cfg, obs_space, state["world_model"] if state else None,
        state["actor"] if state else None, state["critic"] if state else None,
        state["target_critic"] if state else None)
    player = PlayerDV2(world_model.encoder, world_model.rssm.recurrent_model, world_model.rssm.representation_model,
                       actor, actions_dim, cfg.algo.player.expl_amount, cfg.env.num_envs,
                       cfg.algo.world_model.stochastic_size, cfg.algo.world_model.recurrent_model.recurrent_state_size,
                       device, discrete_size=cfg.algo.world_model.discrete_size)
    world_optimizer = build_optimizer(cfg.algo.world_model.optimizer, world_model.parameters())
    actor_optimizer = build_optimizer(cfg.algo.actor.optimizer, actor.parameters())
    critic_optimizer = build_optimizer(cfg.algo.critic.optimizer, critic.parameters())
    if state:
        world_optimizer.load_state_dict(state["world_optimizer"])
        actor_optimizer.load_state_dict(state["actor_optimizer"])
        critic_optimizer.load_state_dict(state["critic_optimizer"])
    trainer = DreamerV2Trainer(runner, cfg, world_model, actor, critic, target_critic, world_optimizer,
                               actor_optimizer, critic_optimizer, is_continuous, actions_dim)
    aggregator = make_aggregator(cfg)
    buffer_size = cfg.buffer.size // int(cfg.env.num_envs * world_size) if not cfg.dry_run else 2
    rb, btype = build_replay(cfg, runner, log_dir, buffer_size)
    if state and cfg.buffer.checkpoint:
        restore_rb(rb, state, runner)

    spec = DreamerSpec(
        variant="dv2", player=player, train_step=trainer.train_step,
        update_target=lambda: trainer.update_target(1.0), target_every=cfg.algo.critic.target_network_update_freq,
        checkpoint_state=lambda: {
            "world_model": world_model.state_dict(), "actor": actor.state_dict(), "critic": critic.state_dict(),
            "target_critic": target_critic.state_dict(), "world_optimizer": world_optimizer.state_dict(),
            "actor_optimizer": actor_optimizer.state_dict(), "critic_optimizer": critic_optimizer.state_dict()},
        test=lambda: test(player, runner, cfg, log_dir), actor_cls_name=cfg.algo.actor.cls)
    run_dreamer_loop(runner, cfg, state, envs, spec, aggregator, rb, btype, actions_dim, is_continuous, log_dir,
                     expl_decay_steps=state["expl_decay_steps"] if state else 0)
