"""SAC-AE (reference: ``sheeprl/algos/sac_ae/sac_ae.py:47-569``).

Pixel SAC with an auto-encoder.  Per minibatch (``train``, ``sac_ae.py:47-129``):
  critic  : target Q, ensemble Q through the (trained) encoder          | all-reduce | Adam; EMA (gated)
  actor   : actor + Q on detached features, alpha loss (gated)           | all-reduce | Adam x2
  decoder : encoder -> decoder reconstruction of 5-bit dequantised obs   | all-reduce | Adam x2 (gated)
Each sub-update is a ``PhasedStep`` (hipGraph on one GPU, per-phase graphs + RCCL on N); the gates
are host-side and select which captured sub-update runs.

The critic and encoder optimisers share one flat slab (the encoder parameters are the leading run
of the critic's slab), exactly like the reference where both optimisers hold the encoder params.
"""
from __future__ import annotations

import copy
import os
from math import prod
from typing import Any, Dict, Optional

import numpy as np
import torch
import torch.nn.functional as F
from torch import Tensor

from sheeprl_prey_amd.algos.common import (
    build_envs,
    episode_stats,
    load_resume,
    log_throughput,
    restore_replay_buffer,
    setup_logger,
    warn_log_ckpt_every,
)
from sheeprl_prey_amd.algos.sac.loss import critic_loss, entropy_loss, policy_loss
from sheeprl_prey_amd.algos.sac.sac import gather_and_shard
from sheeprl_prey_amd.algos.sac_ae.agent import (
    CNNDecoder,
    CNNEncoder,
    MLPDecoder,
    MLPEncoder,
    SACAEAgent,
    SACAEContinuousActor,
    SACAECritic,
)
from sheeprl_prey_amd.algos.sac_ae.utils import preprocess_obs, test_sac_ae
from sheeprl_prey_amd.config.instantiate import get_class
from sheeprl_prey_amd.data.buffers import ReplayBuffer
from sheeprl_prey_amd.data.tensordict import TensorDict
from sheeprl_prey_amd.models.models import MultiDecoder, MultiEncoder
from sheeprl_prey_amd.parallel.flat_optim import build_optimizer
from sheeprl_prey_amd.parallel.graphs import PhasedStep
from sheeprl_prey_amd.utils.metric import MeanMetric, MetricAggregator
from sheeprl_prey_amd.utils.registry import register_algorithm
from sheeprl_prey_amd.utils.timer import timer


class SACAETrainer:
    def __init__(self, runner, cfg, agent: SACAEAgent, encoder, decoder, actor_optimizer, qf_optimizer,
                 alpha_optimizer, encoder_optimizer, decoder_optimizer):
        self.runner, self.cfg, self.agent = runner, cfg, agent
        self.encoder, self.decoder = encoder, decoder
        self.actor_optimizer, self.qf_optimizer, self.alpha_optimizer = actor_optimizer, qf_optimizer, alpha_optimizer
        self.encoder_optimizer, self.decoder_optimizer = encoder_optimizer, decoder_optimizer
        agent.bind_target_slab(qf_optimizer)
        self.gamma = float(cfg.algo.gamma)
        self.cnn_enc = list(cfg.cnn_keys.encoder)
        self.obs_keys = list(cfg.cnn_keys.encoder) + list(cfg.mlp_keys.encoder)
        self.dec_cnn = list(cfg.cnn_keys.decoder)
        self.dec_keys = list(cfg.cnn_keys.decoder) + list(cfg.mlp_keys.decoder)
        self.critic_params = list(agent.critic.parameters())
        self.actor_params = list(actor_optimizer.params)
        self.ae_params = list(encoder.parameters()) + list(decoder.parameters())
        self._st: Dict[str, Tensor] = {}
        g = bool(cfg.fabric.get("cuda_graphs", False))
        self.critic_step = PhasedStep(runner, [self._critic_fwd_bwd, self._critic_apply], [self._coll_critic], g,
                                      name="sac_ae_critic")
        self.actor_step = PhasedStep(runner, [self._actor_fwd_bwd, self._actor_apply], [self._coll_actor], g,
                                     name="sac_ae_actor")
        self.decoder_step = PhasedStep(runner, [self._ae_fwd_bwd, self._ae_apply], [self._coll_ae], g,
                                       name="sac_ae_decoder")

    def _norm(self, d: Dict[str, Tensor], prefix: str = "") -> Dict[str, Tensor]:
        return {k: d[prefix + k] / 255.0 if k in self.cnn_enc else d[prefix + k] for k in self.obs_keys}

    # ------------------------------------------------------------------ critic
    def _critic_fwd_bwd(self, d):
        a = self.agent
        target = a.get_next_target_q_values(self._norm(d, "next_"), d["rewards"], d["dones"], self.gamma)
        q = a.get_q_values(self._norm(d), d["actions"])
        loss = critic_loss(q, target, a.num_critics)
        self.qf_optimizer.zero_grad()
        loss.backward(inputs=self.critic_params)
        self._st["qf_loss"] = loss.detach()

    def _coll_critic(self, dry: bool = False):
        if not dry:
            self.runner.sync_gradients(self.qf_optimizer)

    def _critic_apply(self, d):
        self.qf_optimizer.step()
        self.agent.critic_target_ema(d["ema_q"])
        self.agent.critic_encoder_target_ema(d["ema_enc"])
        return {"Loss/value_loss": self._st["qf_loss"]}

    # ------------------------------------------------------------------ actor + alpha
    def _actor_fwd_bwd(self, d):
        a = self.agent
        obs = self._norm(d)
        actions, logp = a.get_actions_and_log_probs(obs, detach_encoder_features=True)
        q = a.get_q_values(obs, actions, detach_encoder_features=True)
        actor_loss = policy_loss(a.alpha_t, logp, q.min(-1, keepdim=True)[0])
        self.actor_optimizer.zero_grad()
        actor_loss.backward(inputs=self.actor_params)
        alpha_loss = entropy_loss(a.log_alpha, logp.detach(), a.target_entropy)
        self.alpha_optimizer.zero_grad()
        alpha_loss.backward(inputs=[a.log_alpha])
        self._st["actor_loss"], self._st["alpha_loss"] = actor_loss.detach(), alpha_loss.detach()

    def _coll_actor(self, dry: bool = False):
        if not dry:
            self.runner.sync_gradients(self.actor_optimizer)
            self.runner.sync_gradients(self.alpha_optimizer)

    def _actor_apply(self, d):
        self.actor_optimizer.step()
        self.alpha_optimizer.step()
        return {"Loss/policy_loss": self._st["actor_loss"], "Loss/alpha_loss": self._st["alpha_loss"]}

    # ------------------------------------------------------------------ auto-encoder
    def _ae_fwd_bwd(self, d):
        hidden = self.encoder(self._norm(d))
        rec = self.decoder(hidden)
        l2 = self.cfg.algo.decoder.l2_lambda * (0.5 * hidden.pow(2).sum(1)).mean()
        loss = 0.0
        for k in self.dec_keys:
            target = preprocess_obs(d[k], bits=5) if k in self.dec_cnn else d[k]
            loss = loss + F.mse_loss(target, rec[k]) + l2
        self.encoder_optimizer.zero_grad()
        self.decoder_optimizer.zero_grad()
        loss.backward(inputs=self.ae_params)
        self._st["rec_loss"] = loss.detach()

    def _coll_ae(self, dry: bool = False):
        if not dry:
            self.runner.sync_gradients(self.encoder_optimizer)
            self.runner.sync_gradients(self.decoder_optimizer)

    def _ae_apply(self, d):
        self.encoder_optimizer.step()
        self.decoder_optimizer.step()
        return {"Loss/reconstruction_loss": self._st["rec_loss"]}

    # ------------------------------------------------------------------ API
    def train(self, data: Dict[str, Tensor], update: int, policy_steps_per_update: int, aggregator=None,
              eager: bool = False) -> None:
        cfg = self.cfg
        critic_freq = cfg.algo.critic.target_network_frequency // policy_steps_per_update + 1
        actor_freq = cfg.algo.actor.network_frequency // policy_steps_per_update + 1
        decoder_freq = cfg.algo.decoder.update_freq // policy_steps_per_update + 1
        dev = data["rewards"].device
        do_ema = update % critic_freq == 0
        d = dict(data)
        # cached device scalars: a per-step torch.tensor(device=...) is a synchronous H2D copy
        cache = self.__dict__.setdefault("_ema_cache", {})
        key = (bool(do_ema), str(dev))
        if key not in cache:
            cache[key] = (torch.tensor([self.agent.tau if do_ema else 0.0], device=dev),
                          torch.tensor([self.agent.encoder_tau if do_ema else 0.0], device=dev))
        d["ema_q"], d["ema_enc"] = cache[key]
        out = {}
        out.update(self._run(self.critic_step, d, eager))
        if update % actor_freq == 0:
            out.update(self._run(self.actor_step, {k: data[k] for k in self.obs_keys}, eager))
        if update % decoder_freq == 0:
            out.update(self._run(self.decoder_step, {k: data[k] for k in set(self.obs_keys) | set(self.dec_keys)},
                                 eager))
        if aggregator is not None:
            for k, v in out.items():
                if k in aggregator:
                    aggregator.update(k, v)

    @staticmethod
    def _run(step: PhasedStep, d, eager: bool):
        if eager or not step.enabled:
            return step._run(d)
        return step(d)


def build_sac_ae(runner, cfg, envs, state: Optional[Dict[str, Any]] = None):
    obs_space = envs.single_observation_space
    act_dim = prod(envs.single_action_space.shape)
    cnn_channels = [prod(obs_space[k].shape[:-2]) for k in cfg.cnn_keys.encoder]
    mlp_dims = [obs_space[k].shape[0] for k in cfg.mlp_keys.encoder]
    enc_cfg, dec_cfg = cfg.algo.encoder, cfg.algo.decoder
    cnn_encoder = CNNEncoder(sum(cnn_channels), enc_cfg.features_dim, cfg.cnn_keys.encoder, cfg.env.screen_size,
                             enc_cfg.cnn_channels_multiplier) if cfg.cnn_keys.encoder else None
    mlp_encoder = MLPEncoder(sum(mlp_dims), cfg.mlp_keys.encoder, enc_cfg.dense_units, enc_cfg.mlp_layers,
                             get_class(enc_cfg.dense_act), enc_cfg.layer_norm) if cfg.mlp_keys.encoder else None
    encoder = MultiEncoder(cnn_encoder, mlp_encoder)
    cnn_decoder = CNNDecoder(cnn_encoder.conv_output_shape, encoder.output_dim, cfg.cnn_keys.decoder, cnn_channels,
                             cfg.env.screen_size, dec_cfg.cnn_channels_multiplier) if cfg.cnn_keys.decoder else None
    mlp_decoder = MLPDecoder(encoder.output_dim, mlp_dims, cfg.mlp_keys.decoder, dec_cfg.dense_units,
                             dec_cfg.mlp_layers, get_class(dec_cfg.dense_act),
                             dec_cfg.layer_norm) if cfg.mlp_keys.decoder else None
    decoder = MultiDecoder(cnn_decoder, mlp_decoder)
    actor = SACAEContinuousActor(copy.deepcopy(encoder), act_dim, cfg.distribution, cfg.algo.actor.hidden_size,
                                 envs.single_action_space.low, envs.single_action_space.high)
    critic = SACAECritic(encoder, act_dim, cfg.algo.critic.hidden_size, cfg.algo.critic.n)
    agent = SACAEAgent(actor, critic, -act_dim, alpha=cfg.algo.alpha.alpha, tau=cfg.algo.tau,
                       encoder_tau=cfg.algo.encoder.tau)
    if state is not None:
        agent.load_state_dict(state["agent"])
        encoder.load_state_dict(state["encoder"])
        decoder.load_state_dict(state["decoder"])
    agent = runner.setup_module(agent)
    decoder = runner.setup_module(decoder)
    return agent, agent.critic.encoder, decoder


@register_algorithm()
def main(runner, cfg: Dict[str, Any]):
    if "minedojo" in str(cfg.env.wrapper.get("_target_", "")).lower():
        raise ValueError("MineDojo is not currently supported by SAC-AE agent, since it does not take into "
                         "consideration the action masks provided by the environment, but needed in order to play "
                         "correctly the game. As an alternative you can use one of the Dreamers' agents.")
    cfg, state = load_resume(runner, cfg)
    device = runner.device
    rank, world_size = runner.global_rank, runner.world_size
    runner.seed_everything(cfg.seed)
    cfg.env.screen_size = 64

    logger, log_dir = setup_logger(runner, cfg)
    envs = build_envs(runner, cfg, log_dir)
    obs_space = envs.single_observation_space
    from sheeprl_prey_amd.envs import spaces

    if not isinstance(obs_space, spaces.Dict):
        raise RuntimeError(f"Unexpected observation type, should be of type Dict, got: {obs_space}")
    if cfg.cnn_keys.encoder == [] and cfg.mlp_keys.encoder == []:
        raise RuntimeError("You should specify at least one CNN keys or MLP keys from the cli: "
                           "`cnn_keys.encoder=[rgb]` or `mlp_keys.encoder=[state]`")
    if (len(set(cfg.cnn_keys.encoder) & set(cfg.cnn_keys.decoder)) == 0
            and len(set(cfg.mlp_keys.encoder) & set(cfg.mlp_keys.decoder)) == 0):
        raise RuntimeError("The CNN keys or the MLP keys of the encoder and decoder must not be disjoint")
    if len(set(cfg.cnn_keys.decoder) - set(cfg.cnn_keys.encoder)) > 0:
        raise RuntimeError("The CNN keys of the decoder must be contained in the encoder ones. "
                           f"Those keys are decoded without being encoded: {list(set(cfg.cnn_keys.decoder))}")
    if len(set(cfg.mlp_keys.decoder) - set(cfg.mlp_keys.encoder)) > 0:
        raise RuntimeError("The MLP keys of the decoder must be contained in the encoder ones. "
                           f"Those keys are decoded without being encoded: {list(set(cfg.mlp_keys.decoder))}")
    runner.print("Encoder CNN keys:", cfg.cnn_keys.encoder)
    runner.print("Encoder MLP keys:", cfg.mlp_keys.encoder)
    runner.print("Decoder CNN keys:", cfg.cnn_keys.decoder)
    runner.print("Decoder MLP keys:", cfg.mlp_keys.decoder)

    agent, encoder, decoder = build_sac_ae(runner, cfg, envs, state)
    # critic slab first: the encoder params are its leading run, shared by the encoder optimiser
    qf_optimizer = build_optimizer(cfg.algo.critic.optimizer, agent.critic.parameters())
    encoder_optimizer = build_optimizer(cfg.algo.encoder.optimizer, encoder.parameters())
    decoder_optimizer = build_optimizer(cfg.algo.decoder.optimizer, decoder.parameters())
    # the actor's tied conv/MLP trunk never receives actor gradients (detached features): the actor
    # optimiser owns only the actor's own parameters
    actor_optimizer = build_optimizer(cfg.algo.actor.optimizer,
                                      [p for p in agent.actor.parameters() if getattr(p, "_flat_slab", None) is None])
    alpha_optimizer = build_optimizer(cfg.algo.alpha.optimizer, [agent.log_alpha])
    if state:
        qf_optimizer.load_state_dict(state["qf_optimizer"])
        actor_optimizer.load_state_dict(state["actor_optimizer"])
        alpha_optimizer.load_state_dict(state["alpha_optimizer"])
        encoder_optimizer.load_state_dict(state["encoder_optimizer"])
        decoder_optimizer.load_state_dict(state["decoder_optimizer"])
    trainer = SACAETrainer(runner, cfg, agent, encoder, decoder, actor_optimizer, qf_optimizer, alpha_optimizer,
                           encoder_optimizer, decoder_optimizer)

    aggregator = MetricAggregator({k: MeanMetric(sync_on_compute=cfg.metric.sync_on_compute) for k in (
        "Rewards/rew_avg", "Game/ep_len_avg", "Loss/value_loss", "Loss/policy_loss", "Loss/alpha_loss",
        "Loss/reconstruction_loss")})

    obs_keys = list(cfg.cnn_keys.encoder) + list(cfg.mlp_keys.encoder)
    buffer_size = cfg.buffer.size // int(cfg.env.num_envs * world_size) if not cfg.dry_run else 1
    rb = ReplayBuffer(buffer_size, cfg.env.num_envs, device=device if cfg.buffer.memmap is False and
                      device.type == "cuda" else "cpu", memmap=cfg.buffer.memmap,
                      memmap_dir=os.path.join(log_dir, "memmap_buffer", f"rank_{rank}"), obs_keys=obs_keys)
    if state and cfg.buffer.checkpoint and "rb" in state:
        restore_replay_buffer(rb, state["rb"], runner)
    step_data = TensorDict({}, batch_size=[cfg.env.num_envs], device=rb.device)

    last_train = 0
    train_step = 0
    start_step = state["update"] // world_size if state else 1
    policy_step = state["update"] * cfg.env.num_envs if state else 0
    last_log = state["last_log"] if state else 0
    last_checkpoint = state["last_checkpoint"] if state else 0
    policy_steps_per_update = int(cfg.env.num_envs * world_size)
    num_updates = int(cfg.total_steps // policy_steps_per_update) if not cfg.dry_run else 1
    learning_starts = cfg.algo.learning_starts // policy_steps_per_update if not cfg.dry_run else 0
    if state and not cfg.buffer.checkpoint:
        learning_starts += start_step
    warn_log_ckpt_every(cfg, policy_steps_per_update)

    def to_obs(o):
        out = {}
        for k in obs_keys:
            t = torch.as_tensor(np.asarray(o[k])).to(device)
            if k in cfg.cnn_keys.encoder:
                t = t.view(cfg.env.num_envs, -1, *t.shape[-2:])
            else:
                t = t.float()
            out[k] = t
        return out

    obs = to_obs(envs.reset(seed=cfg.seed)[0])
    for update in range(start_step, num_updates + 1):
        policy_step += cfg.env.num_envs * world_size
        with timer("Time/env_interaction_time"):
            if update < learning_starts:
                actions = envs.action_space.sample()
            else:
                with torch.no_grad():
                    nobs = {k: v / 255 if k in cfg.cnn_keys.encoder else v for k, v in obs.items()}
                    actions = agent.actor(nobs)[0].cpu().numpy()
            o, rewards, dones, truncated, infos = envs.step(actions.reshape(envs.action_space.shape))
            dones = np.logical_or(dones, truncated)
        for i, ep_rew, ep_len in episode_stats(infos):
            aggregator.update("Rewards/rew_avg", ep_rew)
            aggregator.update("Game/ep_len_avg", ep_len)
            runner.print(f"Rank-0: policy_step={policy_step}, reward_env_{i}={ep_rew[-1]}")

        from sheeprl_prey_amd.algos.sac.sac import real_next_obs

        real_next = to_obs(real_next_obs(o, infos))
        next_obs = to_obs(o)
        for k in obs_keys:
            step_data[k] = obs[k].to(rb.device)
            if not cfg.buffer.sample_next_obs:
                step_data[f"next_{k}"] = real_next[k].to(rb.device)
        n = cfg.env.num_envs
        step_data["actions"] = torch.as_tensor(actions, dtype=torch.float32).view(n, -1).to(rb.device)
        step_data["rewards"] = torch.as_tensor(rewards, dtype=torch.float32).view(n, -1).to(rb.device)
        step_data["dones"] = torch.as_tensor(dones, dtype=torch.float32).view(n, -1).to(rb.device)
        rb.add(step_data.unsqueeze(0))
        obs = next_obs

        if update >= learning_starts - 1:
            training_steps = learning_starts if update == learning_starts - 1 else 1
            sample = rb.sample(max(training_steps, 1) * cfg.algo.per_rank_gradient_steps * cfg.per_rank_batch_size,
                               sample_next_obs=cfg.buffer.sample_next_obs)
            data = gather_and_shard(runner, sample, cfg).to(device)
            with timer("Time/train_time"):
                B = cfg.per_rank_batch_size
                for start in range(0, data.shape[0], B):
                    batch = data[start : start + B]
                    bd = {k: batch[k] for k in batch.keys()}
                    trainer.train(bd, update, policy_steps_per_update, aggregator,
                                  eager=bd["rewards"].shape[0] != B)
                train_step += world_size

        if policy_step - last_log >= cfg.metric.log_every or update == num_updates or cfg.dry_run:
            runner.log_dict(aggregator.compute(), policy_step)
            aggregator.reset()
            log_throughput(runner, timer.compute(), policy_step, last_log, train_step, last_train,
                           cfg.env.action_repeat)
            timer.reset()
            last_log = policy_step
            last_train = train_step

        if (cfg.checkpoint.every > 0 and policy_step - last_checkpoint >= cfg.checkpoint.every) or cfg.dry_run:
            last_checkpoint = policy_step
            ckpt_state = {
                "agent": agent.state_dict(),
                "encoder": encoder.state_dict(),
                "decoder": decoder.state_dict(),
                "qf_optimizer": qf_optimizer.state_dict(),
                "actor_optimizer": actor_optimizer.state_dict(),
                "alpha_optimizer": alpha_optimizer.state_dict(),
                "encoder_optimizer": encoder_optimizer.state_dict(),
                "decoder_optimizer": decoder_optimizer.state_dict(),
                "update": update * world_size,
                "batch_size": cfg.per_rank_batch_size * world_size,
                "last_log": last_log,
                "last_checkpoint": last_checkpoint,
            }
            runner.call("on_checkpoint_coupled", ckpt_path=os.path.join(log_dir, f"checkpoint/ckpt_{policy_step}_{rank}.ckpt"),
                        state=ckpt_state, replay_buffer=rb if cfg.buffer.checkpoint else None)

    envs.close()
    if runner.is_global_zero:
        test_sac_ae(agent.actor, runner, cfg, log_dir)
