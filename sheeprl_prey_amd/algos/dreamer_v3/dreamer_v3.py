"""DreamerV3 (reference: ``sheeprl/algos/dreamer_v3/dreamer_v3.py:51-807``).

``DreamerV3Trainer.train_step`` is one full gradient step - world model, behaviour (actor) and
critic - with the reference's math (``train`` at ``dreamer_v3.py:51-351``).  MI355X design:

* world-model, actor and critic each own a flat fp32 parameter/gradient slab (fused Adam,
  device-side clipping, one RCCL all-reduce per backward);
* the replay buffer lives in HBM, so a training batch is an on-device gather;
* the posterior scan hoists its step-invariant GEMMs (``RSSM.scan_dynamic``);
* for discrete actions the imagination rollout carries no autograd graph (the reference builds
  one that no loss uses: the discrete objective only back-propagates through ``log_prob`` of
  detached actions), halving the imagination cost;
* with ``fabric.cuda_graphs=True`` the whole step is captured once in a hipGraph and replayed
  (single-rank), removing ~3k kernel-launch gaps per step;
* the target critic is a flat slab too: its Polyak update is one ``lerp_`` kernel.
"""
from __future__ import annotations

import copy
import os
import time
import warnings
from typing import Any, Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F
from torch import Tensor

from sheeprl_prey_amd import ops
from sheeprl_prey_amd.ops import sidestream
from sheeprl_prey_amd.algos.common import (
    action_info,
    build_envs,
    check_obs_keys,
    episode_stats,
    episode_success,
    load_resume,
    log_throughput,
    setup_logger,
    warn_log_ckpt_every,
)
from sheeprl_prey_amd.algos.dreamer_v3 import imagine_cont
from sheeprl_prey_amd.algos.dreamer_v3.agent import PlayerDV3, build_models
from sheeprl_prey_amd.algos.dreamer_v3.interaction import InteractionLoop
from sheeprl_prey_amd.algos.dreamer_v3.loss import reconstruction_loss
from sheeprl_prey_amd.algos.dreamer_v3.utils import Moments, compute_lambda_values, test
from sheeprl_prey_amd.data.buffers import AsyncReplayBuffer
from sheeprl_prey_amd.data.tensordict import TensorDict
from sheeprl_prey_amd.ops.rssm import check_scan_health
from sheeprl_prey_amd.parallel.collectives import set_phase, step_boundary
from sheeprl_prey_amd.parallel.flat_optim import flatten_like, build_optimizer
from sheeprl_prey_amd.parallel.graphs import GraphedStep
from sheeprl_prey_amd.utils.distribution import OneHotCategoricalValidateArgs
from sheeprl_prey_amd.utils.metric import MeanMetric, MetricAggregator
from sheeprl_prey_amd.utils.registry import register_algorithm
from sheeprl_prey_amd.utils.timer import timer
from sheeprl_prey_amd.utils.utils import polynomial_decay

torch.distributions.Distribution.set_default_validate_args(False)

METRIC_KEYS = (
    "Loss/world_model_loss", "Loss/value_loss", "Loss/policy_loss", "Loss/observation_loss", "Loss/reward_loss",
    "Loss/state_loss", "Loss/continue_loss", "State/kl", "State/post_entropy", "State/prior_entropy",
    "Grads/world_model", "Grads/actor", "Grads/critic",
)


class DreamerV3Trainer:
    """One DreamerV3 gradient step as five phases separated by the collectives they need:

    ``wm`` (world-model fwd/bwd) | all-reduce(wm grads) | ``imagine`` (wm step, imagination, lambda) |
    all-gather(lambda) | ``actor`` (Moments, actor fwd/bwd) | all-reduce(actor grads) | ``critic`` (critic
    fwd/bwd) | all-reduce(critic grads) | ``final`` (actor step, critic step).

    The critic loss reads neither the actor's weights nor its gradients, so the actor's all-reduce is
    left in flight across the critic phase and joined by the actor's clip/step in ``final`` (the
    reference steps the actor before the critic forward, ``dreamer_v3.py:319-327``: same values).

    Execution:
    * one rank, graphs: ONE hipGraph for the whole step;
    * N ranks, graphs: one hipGraph per phase with the collectives issued eagerly between replays (no
      collective is ever captured: a capture holding RCCL work launched from the autograd thread aborted
      the process on ROCm, profiles/r6_rccl_abort.md) (for continuous actors the actor phase's backward
      then runs through the imagination graph the previous capture recorded; both captures share one
      memory pool);
    * no graphs: eager."""

    # the segmented (multi-rank) form's graphs: the actor all-reduce is issued (async) between the actor and critic
    # graphs and runs on the RCCL stream while the critic graph replays; the critic collective joins it before the
    # final graph (round 5 merged actor+critic into one graph and lost that overlap)
    PHASES = ("wm", "imagine", "actor", "critic", "final")

    def __init__(self, runner, cfg, world_model, actor, critic, target_critic, world_optimizer, actor_optimizer,
                 critic_optimizer, moments: Moments, is_continuous: bool, actions_dim: Sequence[int],
                 force_segmented: bool = False):
        self.runner, self.cfg = runner, cfg
        self.world_model, self.actor, self.critic, self.target_critic = world_model, actor, critic, target_critic
        self.world_optimizer, self.actor_optimizer, self.critic_optimizer = world_optimizer, actor_optimizer, critic_optimizer
        self.moments = moments
        self.is_continuous = is_continuous
        self.actions_dim = list(actions_dim)
        self.target_flat = flatten_like(target_critic, critic_optimizer)
        # discrete fast path: record the rollout's actor forward and keep the imagination critic forward's
        # graph, so the actor / critic losses skip their second forwards (attribute: tests toggle it)
        self.reuse_forwards = True
        # first layers over the one-hot posteriors / priors as row gathers (ops/onehot.py)
        self.onehot_heads = True
        # continuous actors: the imagined rollout + its backward as one hand-written autograd node
        # (algos/dreamer_v3/imagine_cont.py); False = the reference-shaped eager loop
        self.cont_fast = True
        self._st: Dict[str, Any] = {}
        self._consts: Dict[Any, Tensor] = {}
        self._gather_buf = None
        # teacher forcing of the eager oracle (tests/test_dv3_step_oracle_gpu.py): {"posteriors" [T,B,S],
        # "priors" [H+1,M,S], "actions" [H+1,M,A]} one-hot samples of a fused run, taken instead of drawing
        # (eager discrete path only) so both runs see the same discrete latents / actions
        self.teacher: Dict[str, Tensor] = None
        ws = runner.world_size
        graphs = bool(runner.cuda_graphs)
        self.segmented = graphs and (force_segmented or ws > 1)
        single = graphs and not self.segmented
        self.graph_mode = "segmented" if self.segmented else ("single" if single else "eager")
        # the actor all-reduce overlaps the critic phase: inside the single graph as a deferred join, in the
        # segmented form as an async collective between the actor and critic replays (joined by ``_coll_critic``)
        self.defer_actor_sync = True
        # discrete single-graph step on one rank: the actor phase on a side stream beside the critic phase, joined
        # before the final phase (dense <= 512, see below).  A backward runs on the stream its forward ran on: the actor's loss graph is built
        # inside its phase (side stream), the critic reuses the imagination's forward graph (main stream).  Measured
        # +0.4 % (the two phases' GEMMs slow each other, profiles/r5_ac_overlap.md); the continuous step (critic on
        # the side beside the rollout backward) measured 1.4 % slower and stays in line.  SRL_DV3_AC_OVERLAP=0: in line
        # Wider models fill the chip with either phase alone: XL (dense 1024, 5 layers) measured 47.0-47.3 overlapped
        # vs 48.2-48.4 in line, so the overlap is kept to dense <= 512 (the Atari-100k recipe)
        self.overlap_ac = (not self.segmented and ws == 1 and not is_continuous
                           and int(cfg.algo.get("dense_units", 512)) <= 512
                           and os.environ.get("SRL_DV3_AC_OVERLAP", "1") != "0")
        self.graphed = GraphedStep(self._full_step, warmup=2, enabled=single, name="dreamer_v3_train")
        if self.segmented:
            from sheeprl_prey_amd.parallel.graphs import SegmentedGraph

            self.seg = SegmentedGraph(
                [self._phase_wm, self._phase_imagine, self._phase_actor, self._phase_critic, self._phase_final],
                [self._coll_wm, self._coll_lambda, self._coll_actor, self._coll_critic],
                warmup=2,
            )

    def _const(self, like: Tensor, value: float) -> Tensor:
        """A cached tensor shaped like ``like`` filled with ``value`` (backward seeds, constant rows): made once,
        outside the captured replays, instead of a fill launch per step."""
        key = (tuple(like.shape), like.dtype, str(like.device), float(value))
        t = self._consts.get(key)
        if t is None:
            t = self._consts[key] = torch.full(like.shape, float(value), dtype=like.dtype, device=like.device)
        return t

    @property
    def uses_graphs(self) -> bool:
        return bool(self.graphed.enabled or self.segmented)

    @torch.no_grad()
    def update_target(self, tau: float) -> None:
        """theta' <- tau*theta + (1-tau)*theta' as one lerp over the flat slab (reference ``dreamer_v3.py:713-716``)."""
        self.target_flat.lerp_(self.critic_optimizer.flat_param, float(tau))

    def train_step(self, data: Dict[str, Tensor]) -> Dict[str, Tensor]:
        step_boundary()
        if self.segmented:
            return self.seg(data)
        return self.graphed(data)

    def train_step_sampled(self, rb, batch_size: int, sequence_length: int):
        """Once the step is captured (single graph, or the per-phase graphs of the segmented mode): the
        replay sample is drawn straight into the graphs' static inputs by one device launch
        (``sample_into``) and the step replayed - None (caller samples + calls ``train_step``) otherwise."""
        g = self.seg if self.segmented else self.graphed
        ready = g.graphs is not None if self.segmented else g.graph is not None
        if not ready or g.static_in is None or not hasattr(rb, "sample_into"):
            return None
        if not rb.sample_into(g.static_in, batch_size, sequence_length):
            return None
        step_boundary()
        return g.replay_static()

    def _full_step(self, data: Dict[str, Tensor]) -> Dict[str, Tensor]:
        self._phase_wm(data)
        self._coll_wm()
        self._phase_imagine(data)
        self._coll_lambda()
        dev = data["rewards"].device
        if self.overlap_ac and dev.type == "cuda" and self.runner.world_size == 1:
            main = torch.cuda.current_stream(dev)
            side = sidestream._stream(sidestream._index(dev))  # its own half of the column-sum tickets
            side.wait_stream(main)
            # the recorded rollout activations (allocated on the main stream) stay referenced until the join: the
            # actor phase drops them while its backward may still be reading them on the side stream
            keep = self._st.get("actor_rec")
            with torch.cuda.stream(side):
                self._phase_actor(data)
                self._coll_actor()  # (one rank: no communication; kept so the phase contract holds)
            self._phase_critic(data)
            self._coll_critic()
            main.wait_stream(side)
            del keep
            return self._phase_final(data)
        self._phase_actor(data)
        self._coll_actor()
        self._phase_critic(data)
        self._coll_critic()
        return self._phase_final(data)

    # ------------------------------------------------------------------ collectives (eager)
    # ``dry=True``: bind buffers only (called between phase captures, no communication)
    def _coll_wm(self, dry: bool = False) -> None:
        set_phase("coll_wm")
        if not dry:
            self.runner.sync_gradients(self.world_optimizer, faults=True)

    def _coll_actor(self, dry: bool = False) -> None:
        set_phase("coll_actor")
        if not dry:
            self.runner.sync_gradients(self.actor_optimizer, wait=not self.defer_actor_sync)

    def _coll_critic(self, dry: bool = False) -> None:
        set_phase("coll_critic")
        if not dry:
            self.runner.sync_gradients(self.critic_optimizer)
            if self.segmented:
                # the final graph's clip/step read the actor slab: its in-flight all-reduce is joined here, eagerly
                # (a stream dependency on the RCCL stream, no host wait) - the captured join saw no pending work
                self.actor_optimizer.wait_grads()

    def _coll_lambda(self, dry: bool = False) -> None:
        set_phase("coll_lambda")
        lam = self._st["lambda_values"]
        ws = self.runner.world_size
        if ws <= 1:
            self._st["gathered"] = lam
            return
        import torch.distributed as dist

        if self._gather_buf is None or self._gather_buf.shape[1:] != lam.shape:
            self._gather_buf = torch.empty((ws,) + tuple(lam.shape), device=lam.device, dtype=lam.dtype)
        self._st["gathered"] = self._gather_buf
        if dry:
            return
        if lam.is_cuda and self.runner.backend == "nccl":
            dist.all_gather_into_tensor(self._gather_buf, lam.detach().contiguous(), group=self.runner.group)
        else:
            dist.all_gather(list(self._gather_buf.unbind(0)), lam.detach().contiguous(), group=self.runner.group)
        self._st["gathered"] = self._gather_buf

    @staticmethod
    def _head(mlp, x: Tensor, onehot, table: Optional[Tensor] = None) -> Tensor:
        """``mlp(x)``; with ``onehot = (idx, G, off, S)`` the first layer's one-hot prior columns are row
        gathers (``ops/onehot.py``) instead of GEMM columns (``table``: their transposed weight, if made already)."""
        if onehot is not None:
            from sheeprl_prey_amd.ops.onehot import mlp_forward

            idx, G, off, S = onehot
            y = mlp_forward(mlp, x, idx, G, off, S, table=table)
            if y is not None:
                return y
        return mlp(x)

    def _head_tables(self, oh) -> Dict[str, Tensor]:
        """The transposed one-hot columns of the imagination heads' first layers (critic, reward, continue and the
        target critic of the critic phase) in ONE transpose launch instead of one per head."""
        if not (ops.fused_enabled() and self.onehot_heads):
            return {}
        from sheeprl_prey_amd.ops.onehot import head_table

        S = oh[3]
        heads = {"critic": self.critic, "reward": self.world_model.reward_model,
                 "continue": self.world_model.continue_model, "target": self.target_critic}
        srcs = {k: head_table(m, S) for k, m in heads.items()}
        srcs = {k: v for k, v in srcs.items() if v is not None and v.is_cuda}
        if not srcs:
            return {}
        with torch.no_grad():
            outs = dict(zip(srcs, ops.transpose_many(list(srcs.values()))))
        for k in ("target", "critic"):  # read again by the critic phase (same weights until the final phase)
            if k in outs:
                self._st[k + "_table"] = outs[k]
        return outs

    # ------------------------------------------------------------------ phases
    def _phase_wm(self, data: Dict[str, Tensor]) -> None:
        set_phase("wm")
        cfg = self.cfg
        wm = self.world_model
        st = self._st
        T, B = data["rewards"].shape[:2]
        wm_cfg = cfg.algo.world_model
        stoch, disc = wm_cfg.stochastic_size, wm_cfg.discrete_size
        out: Dict[str, Tensor] = {}
        # image keys go to the encoder as the raw uint8 frames: it scales them by 1/255 itself (inside the
        # fused conv stack's NHWC conversion), the reference divides here (dreamer_v3.py:169)
        batch_obs = {k: data[k] if data[k].dtype == torch.uint8 else data[k] / 255.0 for k in cfg.cnn_keys.encoder}
        batch_obs.update({k: data[k] for k in cfg.mlp_keys.encoder})
        # first row forced to a reset, actions shifted by one step: one concatenation each with a cached constant row
        is_first = torch.cat((self._const(data["is_first"][:1], 1.0), data["is_first"][1:]), dim=0)
        batch_actions = torch.cat((self._const(data["actions"][:1], 0.0), data["actions"][:-1]), dim=0)
        embedded_obs = wm.encoder(batch_obs)
        forced = self.teacher["posteriors"] if self.teacher is not None else None
        recurrent_states, posteriors, posteriors_logits, priors_logits = wm.rssm.scan_dynamic(
            embedded_obs, batch_actions, is_first, forced=forced)
        latent_states = torch.cat((posteriors.view(T, B, -1), recurrent_states), -1)
        # the posteriors are exact one-hots: the heads' first layers gather those columns (ops/onehot.py)
        oh = None
        if latent_states.is_cuda and ops.fused_enabled() and self.onehot_heads:
            from sheeprl_prey_amd.ops.onehot import onehot_index

            G = stoch
            idx = onehot_index(posteriors.reshape(T * B, stoch * disc), disc,
                               torch.empty(T * B, G, dtype=torch.int32, device=latent_states.device))
            oh = (idx.view(T, B, G), G, 0, stoch * disc)
        reconstructed = wm.observation_model(latent_states, onehot=oh) if oh is not None else wm.observation_model(latent_states)
        # image MSE against the raw uint8 frames and vector symlog MSE, one fused kernel each way (K6)
        terms = [ops.obs_mse(reconstructed[k], data[k] if data[k].dtype == torch.uint8 else batch_obs[k],
                             1.0 / 255.0 if data[k].dtype == torch.uint8 else 1.0) for k in cfg.cnn_keys.decoder]
        terms += [ops.obs_mse(reconstructed[k], batch_obs[k], symlog=True) for k in cfg.mlp_keys.decoder]
        obs_loss = terms[0] if terms else 0  # no "0 + term" launch for the single-key case
        for t_ in terms[1:]:
            obs_loss = obs_loss + t_
        reward_logits = self._head(wm.reward_model, latent_states, oh)
        continue_logits = self._head(wm.continue_model, latent_states, oh)
        ents: List[Tensor] = []  # posterior / prior entropies: a by-product of the KL kernel
        rec_loss, kl, state_loss, reward_loss, observation_loss, continue_loss = reconstruction_loss(
            obs_loss, reward_logits, data["rewards"], priors_logits, posteriors_logits, stoch, disc,
            wm_cfg.kl_dynamic, wm_cfg.kl_representation, wm_cfg.kl_free_nats, wm_cfg.kl_regularizer,
            continue_logits, None, wm_cfg.continue_scale_factor, entropies=ents, dones=data["dones"],
        )
        self.world_optimizer.zero_grad(set_to_none=True)
        with sidestream.scope():  # decoder weight gradients beside the scan backward (ops/sidestream.py)
            rec_loss.backward(self._const(rec_loss, 1.0))
        out["Loss/world_model_loss"] = rec_loss.detach()
        out["Loss/observation_loss"] = observation_loss.detach()
        out["Loss/reward_loss"] = reward_loss.detach()
        out["Loss/state_loss"] = state_loss.detach()
        out["Loss/continue_loss"] = continue_loss.detach()
        out["State/kl"] = kl.detach()
        with torch.no_grad():
            out["State/post_entropy"] = ents[0].mean()
            out["State/prior_entropy"] = ents[1].mean()
        st["out"] = out
        st["posteriors"] = posteriors.detach()
        st["recurrent_states"] = recurrent_states.detach()

    def _phase_imagine(self, data: Dict[str, Tensor]) -> None:
        set_phase("imagine")
        cfg, st = self.cfg, self._st
        wm, actor, critic = self.world_model, self.actor, self.critic
        wm_cfg = cfg.algo.world_model
        S = wm_cfg.stochastic_size * wm_cfg.discrete_size
        H = wm_cfg.recurrent_model.recurrent_state_size
        clip = wm_cfg.clip_gradients
        if clip is not None and clip > 0:
            st["out"]["Grads/world_model"] = self.runner.clip_gradients(wm, self.world_optimizer, max_norm=clip).detach()
        else:
            st["out"]["Grads/world_model"] = torch.zeros((), device=data["rewards"].device)
        self.world_optimizer.step()
        grad_ctx = torch.enable_grad() if self.is_continuous else torch.no_grad()
        # continuous actors back-propagate the policy loss through the imagined dynamics and the critic: only
        # the DATA gradients through the world model and the critic are needed - their parameter gradients
        # from that loss are discarded (the reference zeroes them before the next world-model / critic
        # backward, dreamer_v3.py:179 / :336) - so the rollout's graph is built with those parameters frozen:
        # no weight-gradient GEMMs for them in the actor backward
        frozen = [p for m in (wm, critic) for p in m.parameters() if p.requires_grad] if self.is_continuous else []
        for p in frozen:
            p.requires_grad_(False)
        try:
            self._imagine(data, grad_ctx)
        finally:
            for p in frozen:
                p.requires_grad_(True)

    def _imagine(self, data: Dict[str, Tensor], grad_ctx) -> None:
        cfg, st = self.cfg, self._st
        wm, actor, critic = self.world_model, self.actor, self.critic
        wm_cfg = cfg.algo.world_model
        S = wm_cfg.stochastic_size * wm_cfg.discrete_size
        H = wm_cfg.recurrent_model.recurrent_state_size
        st.pop("traj_onehot", None)  # set again below by this step's rollout (never a previous step's indices)
        with grad_ctx:
            prior = st["posteriors"].reshape(-1, S)
            h = st["recurrent_states"].reshape(-1, H)
            fast = (not self.is_continuous and prior.is_cuda and wm.rssm.imagine_fast_ok(actor) and self.teacher is None)
            fast_c = (self.is_continuous and self.cont_fast and prior.is_cuda and imagine_cont.supported(wm.rssm, actor))
            if fast_c:
                imagined_trajectories, imagined_actions_t, pre, roll = imagine_cont.imagine_continuous(
                    wm.rssm, actor, prior, h, cfg.algo.horizon)
                st["actor_pre"] = pre  # the policies of the actor loss (entropy) come from these head outputs
                if self.onehot_heads:
                    st["traj_onehot"] = (roll.IDX, roll.G, 0, S)
            elif fast:
                res = wm.rssm.imagine_discrete(prior, h, actor, cfg.algo.horizon, record=self.reuse_forwards,
                                               indices=True, gather=self.onehot_heads)
                imagined_trajectories, imagined_actions_t = res[0], res[1]
                if self.reuse_forwards and res[2] is not None:
                    st["actor_rec"] = res[2]
                # hot columns of the trajectories' one-hot priors (offset: the actions' columns), for the
                # heads' first layers as row gathers (ops/onehot.py)
                A = imagined_actions_t.shape[-1]
                if self.onehot_heads:
                    st["traj_onehot"] = (res[-1][:, :, len(self.actions_dim):], S // wm_cfg.discrete_size, A, S)
            else:
                tf = self.teacher if not self.is_continuous else None

                def act(x, t):
                    if tf is None:
                        return actor(x)
                    return actor(x, forced=torch.split(tf["actions"][t], self.actions_dim, -1))

                latent = torch.cat((prior, h), -1)
                trajectories: List[Tensor] = [latent]
                actions = torch.cat(act(latent.detach(), 0)[0], dim=-1)
                imagined_actions: List[Tensor] = [actions]
                for t in range(cfg.algo.horizon):
                    prior, h = wm.rssm.imagination(prior, h, actions, forced=tf["priors"][t + 1] if tf is not None else None)
                    prior = prior.reshape(-1, S)
                    latent = torch.cat((prior, h), -1)
                    trajectories.append(latent)
                    actions = torch.cat(act(latent.detach(), t + 1)[0], dim=-1)
                    imagined_actions.append(actions)
                imagined_trajectories = torch.stack(trajectories)
                imagined_actions_t = torch.stack(imagined_actions)
            oh = st.get("traj_onehot")
            tabs = self._head_tables(oh) if oh is not None else {}
            if fast and self.reuse_forwards:
                # the critic's forward over the trajectories, WITH its graph: the critic loss of this step
                # (same weights - the critic steps in the final phase - same detached inputs) reuses it
                # instead of running the critic forward a second time (reference dreamer_v3.py:260, :327)
                with torch.enable_grad():
                    st["critic_logits"] = self._head(critic, imagined_trajectories, oh, tabs.get("critic"))
                predicted_values = ops.twohot_mean(st["critic_logits"].detach())
            else:
                predicted_values = ops.twohot_mean(self._head(critic, imagined_trajectories, oh, tabs.get("critic")))
            # the reward and continue heads only on the imagined steps 1..H: the losses never read row 0 (reference
            # dreamer_v3.py:261-276 uses rewards[1:] and replaces continues[0] by 1 - done)
            traj1 = imagined_trajectories[1:]
            oh1 = (oh[0][1:],) + tuple(oh[1:]) if oh is not None else None
            predicted_rewards = ops.twohot_mean(self._head(wm.reward_model, traj1, oh1, tabs.get("reward")))
            # continuation flags, their gamma-discounts and the cumulative discount: one kernel (K11)
            cont_g, discount = ops.imag_discount(self._head(wm.continue_model, traj1, oh1, tabs.get("continue")),
                                                 data["dones"], cfg.algo.gamma, skip_first=True)
            lambda_values = compute_lambda_values(predicted_rewards, predicted_values[1:], cont_g,
                                                  lmbda=cfg.algo.lmbda)
        st["discount"] = discount.detach()
        st["imagined_trajectories"] = imagined_trajectories
        st["imagined_actions"] = imagined_actions_t
        st["predicted_values"] = predicted_values
        st["lambda_values"] = lambda_values

    def _phase_actor(self, data: Dict[str, Tensor]) -> None:
        set_phase("actor")
        cfg, st = self.cfg, self._st
        self.actor_optimizer.zero_grad(set_to_none=True)
        rec = st.pop("actor_rec", None)
        pre = st.pop("actor_pre", None)
        if pre is not None:
            # continuous fast rollout: its head outputs carry the actor's graph (imagine_cont.py)
            policies = (self.actor._continuous_dist(pre),)
            mixed = None
        elif rec is not None:
            # the rollout recorded the actor trunk: heads + unimix over its output, backward through the
            # recorded activations (ops/mlp_trunk.py) - no second actor forward
            trunk = rec.output(st["imagined_trajectories"].detach())
            mixed = [ops.unimix_sample(head(trunk), int(a), float(self.actor._unimix), sample=False)[0]
                     for head, a in zip(self.actor.mlp_heads, self.actions_dim)]
            policies = None  # built from ``mixed`` only if the eager objective below is needed
        else:
            policies = self.actor(st["imagined_trajectories"].detach())[1]
            mixed = None if self.is_continuous else [p.logits for p in policies]
        lambda_values = st["lambda_values"]
        baseline = st["predicted_values"][:-1]
        offset, invscale = self.moments.update(st["gathered"])
        if pre is not None and self.actor.distribution == "trunc_normal":
            # advantage, closed-form truncated-normal entropies, discounting and the mean in one kernel
            T = pre.shape[0]
            policy_loss = ops.actor_loss_cont(pre, lambda_values.reshape(T - 1, -1), baseline.reshape(T - 1, -1),
                                              st["discount"].detach().reshape(T, -1), offset, invscale,
                                              cfg.algo.actor.ent_coef, self.actor.init_std, self.actor.min_std)
            if policy_loss is not None:
                policy_loss.backward(self._const(policy_loss, 1.0))
                st["out"]["Loss/policy_loss"] = policy_loss.detach()
                return
        if not self.is_continuous:
            # advantage, log-probs, entropies, discounting and the mean in one kernel (actor_loss.hip)
            z = torch.cat(mixed, -1) if len(mixed) > 1 else mixed[0]
            T = z.shape[0]
            policy_loss = ops.actor_loss_discrete(
                z, st["imagined_actions"], lambda_values.reshape(T - 1, -1), baseline.reshape(T - 1, -1),
                st["discount"].detach().reshape(T, -1), offset, invscale, self.actions_dim, cfg.algo.actor.ent_coef)
            if policy_loss is not None:
                policy_loss.backward(self._const(policy_loss, 1.0))
                st["out"]["Loss/policy_loss"] = policy_loss.detach()
                return
        if policies is None:
            policies = [OneHotCategoricalValidateArgs(logits=m, validate_args=False) for m in mixed]
        advantage = (lambda_values - offset) / invscale - (baseline - offset) / invscale
        if self.is_continuous:
            objective = advantage
        else:
            objective = torch.stack(
                [p.log_prob(a.detach()).unsqueeze(-1)[:-1]
                 for p, a in zip(policies, torch.split(st["imagined_actions"], self.actions_dim, dim=-1))], dim=-1,
            ).sum(dim=-1) * advantage.detach()
        try:
            entropy = cfg.algo.actor.ent_coef * torch.stack([p.entropy() for p in policies], -1).sum(dim=-1)
        except NotImplementedError:
            entropy = torch.zeros_like(objective[..., 0])
        policy_loss = -torch.mean(st["discount"][:-1].detach() * (objective + entropy.unsqueeze(-1)[:-1]))
        policy_loss.backward(self._const(policy_loss, 1.0))
        st["out"]["Loss/policy_loss"] = policy_loss.detach()

    def _phase_critic(self, data: Dict[str, Tensor]) -> None:
        set_phase("critic")
        cfg, st = self.cfg, self._st
        traj = st["imagined_trajectories"].detach()[:-1]
        qv_full = st.pop("critic_logits", None)
        oh = st.get("traj_onehot")
        ctab = st.pop("critic_table", None)
        if qv_full is not None:
            qv_logits = qv_full[:-1]
        else:  # (continuous) the critic's first layer gathers the one-hot prior columns too
            qv_logits = self._head(self.critic, traj, (oh[0][:-1],) + oh[1:] if oh else None, ctab)
        with torch.no_grad():
            target_values = ops.twohot_mean(self._head(self.target_critic, traj, (oh[0][:-1],) + oh[1:] if oh else None,
                                                        st.pop("target_table", None)))
        self.critic_optimizer.zero_grad(set_to_none=True)
        # mean(discount * (nll(lambda returns) + nll(target values))): one kernel writing the loss and its logits gradient
        value_loss = ops.twohot_value_loss(qv_logits, st["lambda_values"].detach(), target_values, st["discount"][:-1].detach())
        value_loss.backward(self._const(value_loss, 1.0))
        st["out"]["Loss/value_loss"] = value_loss.detach()

    def _phase_final(self, data: Dict[str, Tensor]) -> Dict[str, Tensor]:
        set_phase("final")
        cfg, st = self.cfg, self._st
        clip = cfg.algo.actor.clip_gradients
        # joins the actor all-reduce left in flight across the critic phase
        if clip is not None and clip > 0:
            st["out"]["Grads/actor"] = self.runner.clip_gradients(self.actor, self.actor_optimizer, max_norm=clip).detach()
        else:
            st["out"]["Grads/actor"] = torch.zeros((), device=data["rewards"].device)
        self.actor_optimizer.step()
        clip = cfg.algo.critic.clip_gradients
        if clip is not None and clip > 0:
            st["out"]["Grads/critic"] = self.runner.clip_gradients(self.critic, self.critic_optimizer, max_norm=clip).detach()
        else:
            st["out"]["Grads/critic"] = torch.zeros((), device=data["rewards"].device)
        self.critic_optimizer.step()
        # clean-up zeros (not armed: the next backward reaching these parameters may belong to another
        # loss, e.g. the continuous actor loss flowing into the critic), and drop every autograd-carrying
        # hand-off so no graph of this step outlives it
        self.actor_optimizer.zero_grad(set_to_none=True, arm=False)
        self.critic_optimizer.zero_grad(set_to_none=True, arm=False)
        self.world_optimizer.zero_grad(set_to_none=True, arm=False)
        st.pop("traj_onehot", None)
        for k, v in list(st.items()):
            if torch.is_tensor(v) and v.grad_fn is not None:
                st[k] = v.detach()  # same storage (the segmented collectives re-read it), no graph
        return dict(st["out"])


def make_aggregator(cfg) -> MetricAggregator:
    sync = cfg.metric.sync_on_compute
    names = ["Rewards/rew_avg", "Game/ep_len_avg", "Game/success_rate", "Params/exploration_amout", *METRIC_KEYS]
    return MetricAggregator({n: MeanMetric(sync_on_compute=sync) for n in names})


@register_algorithm()
def main(runner, cfg: Dict[str, Any]):
    cfg, state = load_resume(runner, cfg)
    device = runner.device
    rank, world_size = runner.global_rank, runner.world_size
    # the fork does not seed everything (reference dreamer_v3.py:359-360); we seed for reproducibility
    runner.seed_everything(cfg.seed + rank)
    torch.backends.cudnn.deterministic = cfg.torch_deterministic

    cfg.env.frame_stack = -1
    if 2 ** int(np.log2(cfg.env.screen_size)) != cfg.env.screen_size:
        raise ValueError(f"The screen size must be a power of 2, got: {cfg.env.screen_size}")

    logger, log_dir = setup_logger(runner, cfg)
    envs = build_envs(runner, cfg, log_dir, restart_on_exception=True)
    action_space = envs.single_action_space
    observation_space = envs.single_observation_space
    is_continuous, is_multidiscrete, actions_dim = action_info(action_space)
    clip_rewards_fn = (lambda r: torch.tanh(r)) if cfg.env.clip_rewards else (lambda r: r)
    check_obs_keys(cfg, observation_space)
    if not set(cfg.cnn_keys.encoder) & set(cfg.cnn_keys.decoder) and not set(cfg.mlp_keys.encoder) & set(cfg.mlp_keys.decoder):
        raise RuntimeError("The CNN keys or the MLP keys of the encoder and decoder must not be disjointed")
    if set(cfg.cnn_keys.decoder) - set(cfg.cnn_keys.encoder):
        raise RuntimeError("The CNN keys of the decoder must be contained in the encoder ones. "
                           f"Those keys are decoded without being encoded: {list(set(cfg.cnn_keys.decoder))}")
    if set(cfg.mlp_keys.decoder) - set(cfg.mlp_keys.encoder):
        raise RuntimeError("The MLP keys of the decoder must be contained in the encoder ones. "
                           f"Those keys are decoded without being encoded: {list(set(cfg.mlp_keys.decoder))}")
    runner.print("Encoder CNN keys:", cfg.cnn_keys.encoder)
    runner.print("Encoder MLP keys:", cfg.mlp_keys.encoder)
    runner.print("Decoder CNN keys:", cfg.cnn_keys.decoder)
    runner.print("Decoder MLP keys:", cfg.mlp_keys.decoder)
    obs_keys = list(cfg.cnn_keys.encoder) + list(cfg.mlp_keys.encoder)

    world_model, actor, critic, target_critic = build_models(
        runner, actions_dim, is_continuous, cfg, observation_space,
        state["world_model"] if state else None, state["actor"] if state else None,
        state["critic"] if state else None, state["target_critic"] if state else None,
    )
    player = PlayerDV3(world_model.encoder, world_model.rssm, actor, actions_dim, cfg.algo.player.expl_amount,
                       cfg.env.num_envs, cfg.algo.world_model.stochastic_size,
                       cfg.algo.world_model.recurrent_model.recurrent_state_size, device,
                       discrete_size=cfg.algo.world_model.discrete_size)

    world_optimizer = build_optimizer(cfg.algo.world_model.optimizer, world_model.parameters())
    actor_optimizer = build_optimizer(cfg.algo.actor.optimizer, actor.parameters())
    critic_optimizer = build_optimizer(cfg.algo.critic.optimizer, critic.parameters())
    if state:
        world_optimizer.load_state_dict(state["world_optimizer"])
        actor_optimizer.load_state_dict(state["actor_optimizer"])
        critic_optimizer.load_state_dict(state["critic_optimizer"])
    moments = Moments(runner, cfg.algo.actor.moments.decay, cfg.algo.actor.moments.max,
                      cfg.algo.actor.moments.percentile.low, cfg.algo.actor.moments.percentile.high).to(device)
    if state:
        moments.load_state_dict(state["moments"])
    trainer = DreamerV3Trainer(runner, cfg, world_model, actor, critic, target_critic, world_optimizer,
                               actor_optimizer, critic_optimizer, moments, is_continuous, actions_dim)
    aggregator = make_aggregator(cfg)

    buffer_size = cfg.buffer.size // int(cfg.env.num_envs * world_size) if not cfg.dry_run else 2
    buf_device = device if str(cfg.buffer.get("device", "auto")) in ("auto", "cuda") and device.type == "cuda" else torch.device("cpu")
    rb = AsyncReplayBuffer(buffer_size, cfg.env.num_envs, device=buf_device,
                           memmap=cfg.buffer.memmap and buf_device.type == "cpu",
                           memmap_dir=os.path.join(log_dir, "memmap_buffer", f"rank_{rank}"), sequential=True)
    if state and cfg.buffer.checkpoint and state.get("rb") is not None:
        if isinstance(state["rb"], list) and world_size == len(state["rb"]):
            rb.load_state_dict(state["rb"][rank])
        elif isinstance(state["rb"], dict):
            rb.load_state_dict(state["rb"])
        else:
            raise RuntimeError(f"Given {len(state['rb'])}, but {world_size} processes are instantiated")
    expl_decay_steps = state["expl_decay_steps"] if state else 0

    train_step = 0
    last_train = 0
    start_step = state["update"] // world_size if state else 1
    policy_step = state["update"] * cfg.env.num_envs if state else 0
    last_log = state["last_log"] if state else 0
    last_checkpoint = state["last_checkpoint"] if state else 0
    policy_steps_per_update = int(cfg.env.num_envs * world_size)
    updates_before_training = cfg.algo.train_every // policy_steps_per_update
    num_updates = int(cfg.total_steps // policy_steps_per_update) if not cfg.dry_run else 1
    learning_starts = cfg.algo.learning_starts // policy_steps_per_update if not cfg.dry_run else 0
    if state and not cfg.buffer.checkpoint:
        learning_starts += start_step
    max_step_expl_decay = cfg.algo.player.max_step_expl_decay // (cfg.algo.per_rank_gradient_steps * world_size)
    if state:
        player.expl_amount = polynomial_decay(expl_decay_steps, initial=cfg.algo.player.expl_amount,
                                              final=cfg.algo.player.expl_min, max_decay_steps=max_step_expl_decay)
    warn_log_ckpt_every(cfg, policy_steps_per_update)

    # env interaction shared with bench.py (interaction.py): pinned staging ring, H2D on a side stream,
    # the gradient steps launched before the CPU env step so the two overlap
    player.use_graphs = bool(runner.cuda_graphs) and cfg.algo.actor.cls.endswith(".Actor")
    loop = InteractionLoop(runner, cfg, envs, player, rb, actions_dim, is_continuous, clip_rewards_fn)
    loop.reset(cfg.seed)
    train_events = []  # (start, end) GPU events of launched gradient bursts, charged to Time/train_time at log

    per_rank_gradient_steps = 0

    def train_burst(n_samples: int) -> None:
        nonlocal per_rank_gradient_steps
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) if device.type == "cuda" else None
        t0 = time.perf_counter()
        if ev:
            ev[0].record()
        if n_samples == 1 and device.type == "cuda":
            if per_rank_gradient_steps % cfg.algo.critic.target_network_update_freq == 0:
                trainer.update_target(1.0 if per_rank_gradient_steps == 0 else cfg.algo.critic.tau)
            metrics = trainer.train_step_sampled(rb, cfg.per_rank_batch_size, cfg.per_rank_sequence_length)
            if metrics is not None:
                for k, v in metrics.items():
                    aggregator.update(k, v)
                per_rank_gradient_steps += 1
                if ev:
                    ev[1].record()
                    train_events.append(ev)
                return
            # not captured yet: the target update above already ran for this step
            n_target_done = 1
        else:
            n_target_done = 0
        local_data = rb.sample(cfg.per_rank_batch_size, sequence_length=cfg.per_rank_sequence_length, n_samples=n_samples)
        local_data = local_data.to(device)
        for i in range(n_samples):
            if per_rank_gradient_steps % cfg.algo.critic.target_network_update_freq == 0 and not (i == 0 and n_target_done):
                trainer.update_target(1.0 if per_rank_gradient_steps == 0 else cfg.algo.critic.tau)
            batch = {k: v[i].float() if v.dtype != torch.uint8 else v[i] for k, v in local_data.items()}
            metrics = trainer.train_step(batch)
            for k, v in metrics.items():
                aggregator.update(k, v)
            per_rank_gradient_steps += 1
        if ev:
            ev[1].record()
            train_events.append(ev)
        else:
            timer.add("Time/train_time", time.perf_counter() - t0)

    for update in range(start_step, num_updates + 1):
        policy_step += cfg.env.num_envs * world_size
        random_actions = update <= learning_starts and state is None and "minedojo" not in cfg.algo.actor.cls.lower()
        train_now = update >= learning_starts and updates_before_training - 1 <= 0
        n_samples = (cfg.algo.per_rank_pretrain_steps if update == learning_starts else cfg.algo.per_rank_gradient_steps)
        t_int = time.perf_counter()
        infos = loop.step(random_actions, (lambda: train_burst(n_samples)) if train_now else None)
        # the gradient steps launched inside the interaction step are charged to Time/train_time only
        timer.add("Time/env_interaction_time", time.perf_counter() - t_int - loop.last_train_host_s)

        for i, ep_rew, ep_len in episode_stats(infos):
            aggregator.update("Rewards/rew_avg", ep_rew)
            aggregator.update("Game/ep_len_avg", ep_len)
            runner.print(f"Rank-0: policy_step={policy_step}, reward_env_{i}={ep_rew[-1]}")
        for _, ok in episode_success(infos):
            aggregator.update("Game/success_rate", ok)  # goal reached (prey env ``is success``), not in the reference

        updates_before_training -= 1
        if train_now:
            train_step += world_size
            updates_before_training = cfg.algo.train_every // policy_steps_per_update
            if cfg.algo.player.expl_decay:
                expl_decay_steps += 1
                player.expl_amount = polynomial_decay(expl_decay_steps, initial=cfg.algo.player.expl_amount,
                                                      final=cfg.algo.player.expl_min, max_decay_steps=max_step_expl_decay)
            aggregator.update("Params/exploration_amout", player.expl_amount)

        if policy_step - last_log >= cfg.metric.log_every or update == num_updates or cfg.dry_run:
            for e0, e1 in train_events:
                e1.synchronize()
                timer.add("Time/train_time", e0.elapsed_time(e1) / 1e3)
            train_events.clear()
            if device.type == "cuda":
                # optimiser updates the device skipped since the last log because a kernel recorded a fault
                runner.log_dict({"Health/skipped_updates": float(ops.skipped_updates(reset=True))}, policy_step)
            rb.check_gather_error()
            check_scan_health()
            runner.log_dict(aggregator.compute(), policy_step)
            aggregator.reset()
            log_throughput(runner, timer.compute(), policy_step, last_log, train_step, last_train, cfg.env.action_repeat)
            timer.reset()
            last_log = policy_step
            last_train = train_step

        if (cfg.checkpoint.every > 0 and policy_step - last_checkpoint >= cfg.checkpoint.every) or cfg.dry_run or update == num_updates:
            last_checkpoint = policy_step
            ckpt_state = {
                "world_model": world_model.state_dict(),
                "actor": actor.state_dict(),
                "critic": critic.state_dict(),
                "target_critic": target_critic.state_dict(),
                "world_optimizer": world_optimizer.state_dict(),
                "actor_optimizer": actor_optimizer.state_dict(),
                "critic_optimizer": critic_optimizer.state_dict(),
                "expl_decay_steps": expl_decay_steps,
                "moments": moments.state_dict(),
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
        test(player, runner, cfg, log_dir, sample_actions=True)
