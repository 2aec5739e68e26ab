"""SAC, coupled (reference: ``sheeprl/algos/sac/sac.py:34-406``).

Per env step every rank samples ``G*B`` transitions from its (device-resident) replay buffer, the
samples are all-gathered in ONE packed collective and re-sharded with ``DistributedSampler``
semantics, then each minibatch runs

    critic update  : target Q (actor + target ensemble), twin-Q ensemble fwd/bwd | all-reduce | Adam, EMA
    actor update   : squashed-Gaussian actor, ensemble Q, policy + alpha losses  | all-reduce | Adam x2

Each update is a ``PhasedStep``: one hipGraph per update on a single GPU, per-phase graphs with
RCCL between them on N GPUs.  The EMA's "every k updates" gate is a device scalar fed with the
batch (``ema_w = tau * do_update``), so the same graph serves every step.
"""
from __future__ import annotations

import os
from typing import Any, Dict, Optional

import numpy as np
import torch
from torch import Tensor

from sheeprl_prey_amd.algos.common import (
    episode_stats,
    load_resume,
    log_throughput,
    restore_replay_buffer,
    setup_logger,
    shard_indices,
    warn_log_ckpt_every,
)
from sheeprl_prey_amd import ops
from sheeprl_prey_amd.algos.sac.agent import SACAgent, SACCriticEnsemble, build_agent
from sheeprl_prey_amd.algos.sac.loss import critic_loss, entropy_loss, policy_loss
from sheeprl_prey_amd.algos.sac.utils import obs_to_tensor, test
from sheeprl_prey_amd.data.buffers import ReplayBuffer
from sheeprl_prey_amd.data.tensordict import TensorDict
from sheeprl_prey_amd.envs import spaces
from sheeprl_prey_amd.parallel.flat_optim import build_optimizer
from sheeprl_prey_amd.parallel.graphs import PhasedStep
from sheeprl_prey_amd.utils.metric import MeanMetric, MetricAggregator
from sheeprl_prey_amd.utils.registry import register_algorithm
from sheeprl_prey_amd.utils.timer import timer


class SACTrainer:
    """Critic / actor updates of SAC-style agents as captured phased steps.

    ``actor_q_reduce``: "min" (SAC, ``sac/sac.py:64``) or "mean" (DroQ, ``droq/droq.py:115``)."""

    def __init__(self, runner, cfg, agent: SACAgent, actor_optimizer, qf_optimizer, alpha_optimizer,
                 actor_q_reduce: str = "min", graphs: Optional[bool] = None):
        self.runner, self.cfg, self.agent = runner, cfg, agent
        self.actor_optimizer, self.qf_optimizer, self.alpha_optimizer = actor_optimizer, qf_optimizer, alpha_optimizer
        self.gamma = float(cfg.algo.gamma)
        self.actor_q_reduce = actor_q_reduce
        self.fused_critic = os.environ.get("SRL_SAC_FUSED", "1") != "0"
        agent.bind_target_slab(qf_optimizer)
        # the whole gradient step as seven fused launches (algos/sac/fused.py) when the agent fits its kernels
        from sheeprl_prey_amd.algos.sac.fused import SACFusedUpdate

        opts = (actor_optimizer, qf_optimizer, alpha_optimizer)
        self.fused = (SACFusedUpdate(agent, actor_optimizer, qf_optimizer, alpha_optimizer, self.gamma,
                                     reduce_min=actor_q_reduce == "min")
                      if self.fused_critic and SACFusedUpdate.supported(agent, opts) else None)
        self.critic_params = list(agent.critic.parameters())
        self.actor_params = [p for p in agent.actor.parameters() if p.requires_grad]
        self._st: Dict[str, Tensor] = {}
        self._ema_w: Dict[Any, Tensor] = {}
        use_graphs = bool(cfg.fabric.get("cuda_graphs", False)) if graphs is None else graphs
        if self.fused is not None:
            # the whole gradient step is one captured graph (one replay, one set of static inputs)
            self.step = PhasedStep(runner, [self._critic_fwd_bwd, self._critic_apply, self._actor_fwd_bwd,
                                            self._actor_apply], [self._coll_critic, _no_coll, self._coll_actor],
                                   graphs=use_graphs, name="sac_step")
            self.critic_step = self.actor_step = self.step
        else:
            self.critic_step = PhasedStep(runner, [self._critic_fwd_bwd, self._critic_apply], [self._coll_critic],
                                          graphs=use_graphs, name="sac_critic")
            self.actor_step = PhasedStep(runner, [self._actor_fwd_bwd, self._actor_apply], [self._coll_actor],
                                         graphs=use_graphs, name="sac_actor")
        self._ema_static: Optional[Tensor] = None

    # ------------------------------------------------------------------ critic
    def _critic_fwd_bwd(self, d: Dict[str, Tensor]) -> None:
        if self.fused is not None:
            self._st["qf_loss"] = self.fused.critic(d)
            return
        a = self.agent
        target = a.get_next_target_q_values(d["next_observations"], d["rewards"], d["dones"], self.gamma)
        # the twin-Q forward, loss and backward as two kernels (K15) when the critic layout allows
        res = (ops.sac_critic_loss(a.critic.model, d["observations"], d["actions"], target)
               if self.fused_critic and isinstance(a.critic, SACCriticEnsemble) else None)
        if res is not None:
            loss = res[0]
        else:
            q = a.get_q_values(d["observations"], d["actions"])
            loss = critic_loss(q, target, a.num_critics)
        self.qf_optimizer.zero_grad(set_to_none=True)
        loss.backward(inputs=self.critic_params)
        self._st["qf_loss"] = loss.detach()

    def _coll_critic(self, dry: bool = False) -> None:
        if not dry:
            self.runner.sync_gradients(self.qf_optimizer)

    def _critic_apply(self, d: Dict[str, Tensor]) -> Dict[str, Tensor]:
        if self.fused is not None:
            self.fused.critic_apply(d["ema_w"])
        else:
            self.qf_optimizer.step()
            self.agent.qfs_target_ema(d["ema_w"])
        return {"Loss/value_loss": self._st["qf_loss"]}

    # ------------------------------------------------------------------ actor + alpha
    def _actor_fwd_bwd(self, d: Dict[str, Tensor]) -> None:
        if self.fused is not None:
            losses = self.fused.actor(d["observations"])
            self._st["actor_loss"], self._st["alpha_loss"] = losses[0], losses[1]
            return
        a = self.agent
        obs = d["observations"]
        actions, logp = a.get_actions_and_log_probs(obs)
        q = a.get_q_values(obs, actions)
        q_red = q.min(-1, keepdim=True)[0] if self.actor_q_reduce == "min" else q.mean(-1, keepdim=True)
        actor_loss = policy_loss(a.alpha_t, logp, q_red)
        self.actor_optimizer.zero_grad(set_to_none=True)
        actor_loss.backward(inputs=self.actor_params)
        alpha_loss = entropy_loss(a.log_alpha, logp.detach(), a.target_entropy)
        self.alpha_optimizer.zero_grad(set_to_none=True)
        alpha_loss.backward(inputs=[a.log_alpha])
        self._st["actor_loss"] = actor_loss.detach()
        self._st["alpha_loss"] = alpha_loss.detach()

    def _coll_actor(self, dry: bool = False) -> None:
        if not dry:
            self.runner.sync_gradients(self.actor_optimizer)
            # log_alpha is not DDP-wrapped in the reference: its grad is all-reduced explicitly (sac.py:76)
            self.runner.sync_gradients(self.alpha_optimizer)

    def _actor_apply(self, d: Dict[str, Tensor]) -> Dict[str, Tensor]:
        if self.fused is not None:
            self.fused.actor_apply()
            return {"Loss/value_loss": self._st["qf_loss"], "Loss/policy_loss": self._st["actor_loss"],
                    "Loss/alpha_loss": self._st["alpha_loss"]}
        else:
            self.actor_optimizer.step()
            self.alpha_optimizer.step()
        return {"Loss/policy_loss": self._st["actor_loss"], "Loss/alpha_loss": self._st["alpha_loss"]}

    # ------------------------------------------------------------------ API
    def ema_weight(self, do_update: bool, device) -> Tensor:
        # two cached device scalars: no per-step host->device copy (a pageable copy syncs the stream)
        key = (bool(do_update), str(device))
        if key not in self._ema_w:
            self._ema_w[key] = torch.tensor([self.agent.tau if do_update else 0.0], device=device)
        return self._ema_w[key]

    def train(self, data: Dict[str, Tensor], do_ema: bool, aggregator: Optional[MetricAggregator] = None) -> None:
        """One SAC ``train`` call (reference ``sac/sac.py:34-78``) on a minibatch."""
        dev = data["rewards"].device
        d = dict(data)
        d["ema_w"] = self.ema_weight(do_ema, dev)
        self._ema_static = None  # the copy-in below rewrites the static EMA weight
        if self.fused is not None:
            self.fused.attach(aggregator)
            out = dict(self.step(d))
        else:
            out = dict(self.critic_step(d))
            out.update(self.actor_step({"observations": data["observations"]}))
        self.record(out, aggregator)

    TRAIN_KEYS = ("observations", "next_observations", "actions", "rewards", "dones")

    def buffer_draw_inputs(self, rb, batch_size: int) -> Optional[Dict[str, Tensor]]:
        """The captured fused step's static train inputs when ``train_from_buffer`` applies to ``rb`` (one GPU,
        fused update, captured step, device-resident replay holding exactly the train keys, static batch of
        ``batch_size``); None otherwise - the caller then takes the regular path.  Checked before any timing."""
        if self.fused is None or set(rb.keys()) != set(self.TRAIN_KEYS):
            return None
        dev = getattr(rb, "device", None)
        if dev is None or torch.device(dev).type != "cuda":
            return None
        st = self.critic_step.captured_inputs()
        if st is None:
            return None
        out = {k: st[k] for k in self.TRAIN_KEYS}
        if any(v.shape[0] != batch_size for v in out.values()):
            return None
        return out

    def train_from_buffer(self, rb, batch_size: int, n_batches: int, do_ema: bool,
                          aggregator: Optional[MetricAggregator] = None,
                          out: Optional[Dict[str, Tensor]] = None) -> bool:
        """``n_batches`` SAC updates on minibatches drawn by ONE device launch each straight into the captured
        step's static inputs (``ReplayBuffer.sample_rows_into``): per update one sampling kernel + one graph replay,
        no host-side index draw / gather / copy-in.  ``out``: ``buffer_draw_inputs(rb, batch_size)`` (looked up
        when omitted); False (nothing done) when the draw does not apply - the caller takes the regular path."""
        out = out if out is not None else self.buffer_draw_inputs(rb, batch_size)
        if out is None:
            return False
        st = self.critic_step.captured_inputs()
        ema = self.ema_weight(do_ema, st["ema_w"].device)
        if self._ema_static is not ema:
            st["ema_w"].copy_(ema)
            self._ema_static = ema
        self.fused.attach(aggregator)
        for i in range(n_batches):
            if not rb.sample_rows_into(out, batch_size):
                if i == 0:
                    return False
                raise RuntimeError("SAC: the device replay draw stopped applying mid-update")
            self.critic_step.replay()
        return True

    def record(self, out: Dict[str, Tensor], aggregator: Optional[MetricAggregator]) -> None:
        """Loss metrics into ``aggregator`` (the fused update accumulates its own on the device)."""
        if aggregator is None:
            return
        for k, v in out.items():
            if k in aggregator and not (self.fused is not None and k in self.fused.KEYS):
                aggregator.update(k, v)

    def policy(self):
        """The player's action function: the fused one-launch sampler when the update is fused, else None
        (``SACInteraction`` then runs ``agent.actor``)."""
        return self.fused.act if self.fused is not None else None


def _no_coll(dry: bool = False) -> None:
    pass


def make_aggregator(cfg) -> MetricAggregator:
    keys = ["Rewards/rew_avg", "Game/ep_len_avg", "Loss/value_loss", "Loss/policy_loss", "Loss/alpha_loss"]
    return MetricAggregator({k: MeanMetric(sync_on_compute=cfg.metric.sync_on_compute) for k in keys})


def check_sac_spaces(cfg, envs) -> None:
    if "minedojo" in str(cfg.env.wrapper.get("_target_", "")).lower():
        raise ValueError(
            "MineDojo is not currently supported by SAC agent, since it does not take into consideration the action "
            "masks provided by the environment, but needed in order to play correctly the game. As an alternative you "
            "can use one of the Dreamers' agents."
        )
    if not isinstance(envs.single_action_space, spaces.Box):
        raise ValueError("Only continuous action space is supported for the SAC agent")
    obs_space = envs.single_observation_space
    if not isinstance(obs_space, spaces.Dict):
        raise RuntimeError(f"Unexpected observation type, should be of type Dict, got: {obs_space}")
    if len(cfg.mlp_keys.encoder) == 0:
        raise RuntimeError("You should specify at least one MLP key for the encoder: `mlp_keys.encoder=[state]`")
    for k in cfg.mlp_keys.encoder:
        if len(obs_space[k].shape) > 1:
            raise ValueError("Only environments with vector-only observations are supported by the SAC agent. "
                             f"Provided environment: {cfg.env.id}")


def real_next_obs(next_obs: Dict[str, np.ndarray], infos: Dict[str, Any]) -> Dict[str, np.ndarray]:
    """Replace auto-reset observations with the true final observations (reference ``sac.py:292-297``)."""
    if "final_observation" not in infos:
        return next_obs
    out = {k: np.array(v, copy=True) for k, v in next_obs.items()}
    for idx, final in enumerate(infos["final_observation"]):
        if final is not None:
            for k, v in final.items():
                if k in out:
                    out[k][idx] = v
    return out


def gather_and_shard(runner, sample: TensorDict, cfg) -> TensorDict:
    """all_gather the per-rank samples (one packed collective) and take this rank's shard with
    ``DistributedSampler`` semantics (reference ``sac.py:310-331``)."""
    gathered = runner.all_gather(sample.to_dict())  # {k: [W, G*B, 1, ...]}
    flat = {k: v.reshape(-1, *v.shape[3:]) for k, v in gathered.items()}  # [W*G*B, ...]
    n = next(iter(flat.values())).shape[0]
    data = TensorDict(flat, batch_size=[n], device=next(iter(flat.values())).device)
    if runner.world_size > 1:
        idx = shard_indices(n, runner, True, cfg.seed, 0).to(data.device)
        data = data[idx]
    return data


@register_algorithm()
def main(runner, cfg: Dict[str, Any]):
    run_sac_family(runner, cfg, variant="sac")


def sac_train_update(trainer: SACTrainer, runner, cfg, rb, update: int, learning_starts: int, ema_every: int,
                     aggregator) -> bool:
    """SAC's per-env-step training (reference ``sac/sac.py:308-345``); returns whether it trained."""
    if update < learning_starts:
        return False
    training_steps = learning_starts if update == learning_starts else 1
    do_ema = update % ema_every == 0
    draw = (trainer.buffer_draw_inputs(rb, cfg.per_rank_batch_size)
            if runner.world_size == 1 and not cfg.buffer.sample_next_obs else None)
    if draw is not None:
        with timer("Time/train_time"):
            if trainer.train_from_buffer(rb, cfg.per_rank_batch_size,
                                         max(training_steps, 1) * cfg.algo.per_rank_gradient_steps, do_ema, aggregator,
                                         out=draw):
                return True
    sample = rb.sample(max(training_steps, 1) * cfg.algo.per_rank_gradient_steps * cfg.per_rank_batch_size,
                       sample_next_obs=cfg.buffer.sample_next_obs)
    data = gather_and_shard(runner, sample, cfg).to(runner.device)
    with timer("Time/train_time"):
        for start in range(0, data.shape[0], cfg.per_rank_batch_size):
            batch = data[start : start + cfg.per_rank_batch_size]
            bd = {k: batch[k] for k in ("observations", "next_observations", "actions", "rewards", "dones")}
            if bd["observations"].shape[0] != cfg.per_rank_batch_size and trainer.critic_step.enabled:
                # ragged tail batch: static graph shapes do not fit, run it eagerly
                _eager_train(trainer, bd, do_ema, aggregator)
            else:
                trainer.train(bd, do_ema, aggregator)
    return True


class SACInteraction:
    """One env-interaction step of the SAC family (reference ``sac/sac.py:270-305``), shared by
    ``run_sac_family`` and ``bench.py --algo sac``: act (random before ``learning_starts``, else the
    actor - one hipGraph replay on GPU), step the envs, and store the transition row.

    GPU: each env step's row (next obs, real next obs, actions, reward, done) goes to the device as ONE
    pinned copy sliced on the device (instead of five synchronous pageable copies); the staging buffer
    is rewritten only after an event recorded behind its last copy has completed."""

    def __init__(self, runner, cfg, envs, agent, rb, obs_dim: int, policy=None):
        self.runner, self.cfg, self.envs, self.agent, self.rb = runner, cfg, envs, agent, rb
        self.obs_dim = obs_dim
        self.n_env = int(cfg.env.num_envs)
        self.act_dim = int(np.prod(envs.single_action_space.shape))
        self.step_data = TensorDict({}, batch_size=[self.n_env], device=rb.device)
        self.gpu_row = rb.device.type == "cuda"
        if self.gpu_row:
            from sheeprl_prey_amd.parallel.graphs import GraphedStep

            self.stage = torch.empty((self.n_env, 2 * obs_dim + self.act_dim + 2), dtype=torch.float32).pin_memory()
            self.staged = torch.cuda.Event()  # the last copy out of `stage` (random-action steps have no readback)
            act = policy if policy is not None else (lambda o: agent.actor(o)[0])
            self.player = GraphedStep(lambda d: {"a": act(d["obs"])}, warmup=2, enabled=runner.cuda_graphs,
                                      name="sac_player")
        self._last = None

    def reset(self, seed: int) -> None:
        o = self.envs.reset(seed=seed)[0]
        self.obs = obs_to_tensor(o, self.cfg.mlp_keys.encoder, self.rb.device, self.n_env)

    def _host_rows(self, x: Dict[str, Any]) -> np.ndarray:
        return np.concatenate([np.asarray(x[k], dtype=np.float32).reshape(self.n_env, -1)
                               for k in self.cfg.mlp_keys.encoder], -1)

    def act_and_step(self, random_actions: bool):
        """Act and step the envs; returns the env ``infos`` (``store`` adds the row afterwards)."""
        if random_actions:
            actions = self.envs.action_space.sample()
        else:
            with torch.no_grad():
                if self.gpu_row:
                    actions = self.player({"obs": self.obs})["a"].cpu().numpy()
                else:
                    actions, _ = self.agent.actor(self.obs.to(self.runner.device))
                    actions = actions.cpu().numpy()
        next_o, rewards, dones, truncated, infos = self.envs.step(actions.reshape(self.envs.action_space.shape))
        self._last = (actions, next_o, rewards, np.logical_or(dones, truncated), infos)
        return infos

    def store(self) -> None:
        """Add the last step's transition to the replay buffer and advance the observation."""
        cfg, rb, n_env, obs_dim, act_dim = self.cfg, self.rb, self.n_env, self.obs_dim, self.act_dim
        actions, next_o, rewards, dones, infos = self._last
        sd = self.step_data
        if self.gpu_row:
            self.staged.synchronize()
            st = self.stage.numpy()
            st[:, :obs_dim] = self._host_rows(next_o)
            st[:, obs_dim:2 * obs_dim] = self._host_rows(real_next_obs(next_o, infos))
            st[:, 2 * obs_dim:2 * obs_dim + act_dim] = np.asarray(actions, dtype=np.float32).reshape(n_env, -1)
            st[:, -2] = np.asarray(rewards, dtype=np.float32).reshape(n_env)
            st[:, -1] = np.asarray(dones, dtype=np.float32).reshape(n_env)
            row = self.stage.to(rb.device, non_blocking=True)
            self.staged.record()
            next_obs = row[:, :obs_dim]
            step = {"observations": self.obs, "actions": row[:, 2 * obs_dim:2 * obs_dim + act_dim],
                    "rewards": row[:, -2:-1], "dones": row[:, -1:]}
            if not cfg.buffer.sample_next_obs:
                step["next_observations"] = row[:, obs_dim:2 * obs_dim]
            rb.add_step(step)  # one multi-tensor copy, no TensorDict round trip
            self.obs = next_obs
            return
        else:
            next_obs = obs_to_tensor(next_o, cfg.mlp_keys.encoder, rb.device, n_env)
            sd["dones"] = torch.as_tensor(dones, dtype=torch.float32).view(n_env, -1).to(rb.device)
            sd["actions"] = torch.as_tensor(actions, dtype=torch.float32).view(n_env, -1).to(rb.device)
            sd["observations"] = self.obs
            if not cfg.buffer.sample_next_obs:
                sd["next_observations"] = obs_to_tensor(real_next_obs(next_o, infos), cfg.mlp_keys.encoder,
                                                        rb.device, n_env)
            sd["rewards"] = torch.as_tensor(rewards, dtype=torch.float32).view(n_env, -1).to(rb.device)
        rb.add(sd.unsqueeze(0))
        self.obs = next_obs


def run_sac_family(runner, cfg: Dict[str, Any], variant: str = "sac"):
    """Shared coupled main loop of SAC (``sac/sac.py:81-406``) and DroQ (``droq/droq.py:128-416``)."""
    cfg, state = load_resume(runner, cfg)
    device = runner.device
    rank, world_size = runner.global_rank, runner.world_size
    runner.seed_everything(cfg.seed)

    if len(cfg.cnn_keys.encoder) > 0:
        import warnings

        warnings.warn("SAC algorithm cannot allow to use images as observations, the CNN keys will be ignored")
        cfg.cnn_keys.encoder = []

    logger, log_dir = setup_logger(runner, cfg)
    from sheeprl_prey_amd.algos.common import build_envs

    envs = build_envs(runner, cfg, log_dir)
    check_sac_spaces(cfg, envs)
    action_space = envs.single_action_space
    obs_space = envs.single_observation_space
    obs_dim = int(sum(int(np.prod(obs_space[k].shape)) for k in cfg.mlp_keys.encoder))

    droq = variant == "droq"
    if droq:
        from sheeprl_prey_amd.algos.droq.agent import build_agent as build_droq_agent

        agent = build_droq_agent(runner, cfg, obs_dim, action_space, state["agent"] if state else None)
    else:
        agent = build_agent(runner, cfg, obs_dim, action_space, state["agent"] if state else None)
    qf_optimizer = build_optimizer(cfg.algo.critic.optimizer, agent.critic.parameters())
    actor_optimizer = build_optimizer(cfg.algo.actor.optimizer, agent.actor.parameters())
    alpha_optimizer = build_optimizer(cfg.algo.alpha.optimizer, [agent.log_alpha])
    if state:
        qf_optimizer.load_state_dict(state["qf_optimizer"])
        actor_optimizer.load_state_dict(state["actor_optimizer"])
        alpha_optimizer.load_state_dict(state["alpha_optimizer"])
    trainer = SACTrainer(runner, cfg, agent, actor_optimizer, qf_optimizer, alpha_optimizer,
                         actor_q_reduce="mean" if droq else "min")
    aggregator = make_aggregator(cfg)

    buffer_size = cfg.buffer.size // int(cfg.env.num_envs * world_size) if not cfg.dry_run else 1
    rb = ReplayBuffer(buffer_size, cfg.env.num_envs, device=device if device.type == "cuda" else "cpu",
                      memmap=cfg.buffer.memmap and device.type == "cpu",
                      memmap_dir=os.path.join(log_dir, "memmap_buffer", f"rank_{rank}"))
    if state and cfg.buffer.checkpoint and "rb" in state:
        restore_replay_buffer(rb, state["rb"], runner)

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
    ema_every = cfg.algo.critic.target_network_frequency // policy_steps_per_update + 1

    loop = SACInteraction(runner, cfg, envs, agent, rb, obs_dim, policy=trainer.policy())
    loop.reset(cfg.seed)

    for update in range(start_step, num_updates + 1):
        policy_step += cfg.env.num_envs * world_size
        with timer("Time/env_interaction_time"):
            infos = loop.act_and_step(update <= learning_starts)

        for i, ep_rew, ep_len in episode_stats(infos):
            aggregator.update("Rewards/rew_avg", ep_rew)
            aggregator.update("Game/ep_len_avg", ep_len)
            runner.print(f"Rank-0: policy_step={policy_step}, reward_env_{i}={ep_rew[-1]}")

        loop.store()

        if droq:
            from sheeprl_prey_amd.algos.droq.droq import droq_train_update

            trained = droq_train_update(trainer, runner, cfg, rb, update, learning_starts, aggregator)
        else:
            trained = sac_train_update(trainer, runner, cfg, rb, update, learning_starts, ema_every, aggregator)
        if trained:
            train_step += world_size

        if policy_step - last_log >= cfg.metric.log_every or update == num_updates or cfg.dry_run:
            runner.log_dict(aggregator.compute(), policy_step)
            aggregator.reset()
            log_throughput(runner, timer.compute(), policy_step, last_log, train_step, last_train,
                           cfg.env.action_repeat)
            timer.reset()
            last_log = policy_step
            last_train = train_step

        if (cfg.checkpoint.every > 0 and policy_step - last_checkpoint >= cfg.checkpoint.every) or cfg.dry_run or \
                update == num_updates:
            last_checkpoint = policy_step
            ckpt_state = {
                "agent": agent.state_dict(),
                "qf_optimizer": qf_optimizer.state_dict(),
                "actor_optimizer": actor_optimizer.state_dict(),
                "alpha_optimizer": alpha_optimizer.state_dict(),
                "update": update * world_size,
                "batch_size": cfg.per_rank_batch_size * world_size,
                "last_log": last_log,
                "last_checkpoint": last_checkpoint,
            }
            ckpt_path = os.path.join(log_dir, f"checkpoint/ckpt_{policy_step}_{rank}.ckpt")
            runner.call("on_checkpoint_coupled", ckpt_path=ckpt_path, state=ckpt_state,
                        replay_buffer=rb if cfg.buffer.checkpoint else None)

    envs.close()
    if runner.is_global_zero:
        test(agent.actor, runner, cfg, log_dir)


def _eager_train(trainer: SACTrainer, bd, do_ema, aggregator) -> None:
    d = dict(bd)
    d["ema_w"] = trainer.ema_weight(do_ema, bd["rewards"].device)
    out = {}
    trainer._critic_fwd_bwd(d)
    trainer._coll_critic()
    out.update(trainer._critic_apply(d))
    trainer._actor_fwd_bwd(d)
    trainer._coll_actor()
    out.update(trainer._actor_apply(d))
    if trainer.fused is not None:
        trainer.fused.attach(aggregator)
    trainer.record(out, aggregator)
