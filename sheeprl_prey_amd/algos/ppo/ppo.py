"""PPO, coupled (reference: ``sheeprl/algos/ppo/ppo.py:32-459``).

Every rank runs ``env.num_envs`` envs, fills a device-resident rollout buffer, computes GAE
with the HIP reverse-scan kernel, optionally all-gathers the rollouts (``buffer.share_data``),
and runs ``update_epochs`` x minibatch SGD; gradients are averaged with one RCCL all-reduce of
the optimiser's flat slab per step.
"""
from __future__ import annotations

import copy
import os
from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch
from torch import Tensor, nn

from sheeprl_prey_amd.algos.common import (
    PolynomialLR,
    action_info,
    build_envs,
    check_obs_keys,
    episode_stats,
    load_resume,
    log_throughput,
    setup_logger,
    shard_indices,
    warn_log_ckpt_every,
)
from sheeprl_prey_amd.algos.ppo.agent import PPOAgent
from sheeprl_prey_amd.algos.ppo.loss import entropy_loss, policy_loss, value_loss
from sheeprl_prey_amd.algos.ppo.utils import test
from sheeprl_prey_amd.data.buffers import ReplayBuffer
from sheeprl_prey_amd.data.tensordict import TensorDict
from sheeprl_prey_amd.parallel.flat_optim import build_optimizer
from sheeprl_prey_amd.utils.metric import MeanMetric, MetricAggregator
from sheeprl_prey_amd.utils.registry import register_algorithm
from sheeprl_prey_amd.utils.timer import timer
from sheeprl_prey_amd.utils.utils import gae, normalize_tensor, polynomial_decay


def train(runner, agent, optimizer, data: TensorDict, aggregator: MetricAggregator, cfg: Dict[str, Any]) -> None:
    """Eager update_epochs x minibatch SGD (reference ``ppo.py:32-104``); see ``PPOTrainer`` for the
    captured single-rank form used on GPU."""
    n = data.shape[0]
    obs_keys = list(cfg.mlp_keys.encoder) + list(cfg.cnn_keys.encoder)
    for epoch in range(cfg.algo.update_epochs):
        if cfg.buffer.share_data and runner.world_size > 1:
            idx = shard_indices(n, runner, True, cfg.seed, epoch)
        else:
            idx = torch.randperm(n)
        idx = idx.to(data["rewards"].device)
        for start in range(0, len(idx), cfg.per_rank_batch_size):
            batch = data[idx[start : start + cfg.per_rank_batch_size]]
            pg_loss, v_loss, ent_loss = _minibatch_step(runner, agent, optimizer, batch, obs_keys, cfg, cfg.algo.clip_coef,
                                                        cfg.algo.ent_coef)
            if aggregator is not None:
                aggregator.update("Loss/policy_loss", pg_loss.detach())
                aggregator.update("Loss/value_loss", v_loss.detach())
                aggregator.update("Loss/entropy_loss", ent_loss.detach())


def _minibatch_step(runner, agent, optimizer, batch, obs_keys, cfg, clip_coef, ent_coef):
    obs = {k: batch[k] / 255 - 0.5 if k in cfg.cnn_keys.encoder else batch[k] for k in obs_keys}
    _, logprobs, entropy, new_values = agent(obs, torch.split(batch["actions"], agent.actions_dim, dim=-1))
    adv = batch["advantages"]
    if cfg.algo.normalize_advantages:
        adv = normalize_tensor(adv)
    pg_loss = policy_loss(logprobs, batch["logprobs"], adv, clip_coef, cfg.algo.loss_reduction)
    v_loss = value_loss(new_values, batch["values"], batch["returns"], clip_coef, cfg.algo.clip_vloss, cfg.algo.loss_reduction)
    ent_loss = entropy_loss(entropy, cfg.algo.loss_reduction)
    loss = pg_loss + cfg.algo.vf_coef * v_loss + ent_coef * ent_loss
    optimizer.zero_grad(set_to_none=True)
    runner.backward(loss, optimizer)
    if cfg.algo.max_grad_norm > 0.0:
        runner.clip_gradients(agent, optimizer, max_norm=cfg.algo.max_grad_norm)
    optimizer.step()
    return pg_loss, v_loss, ent_loss


class FusedPPOTrainer:
    """The whole PPO update (``update_epochs`` x minibatch steps: forward, clipped-surrogate / value /
    entropy losses, backward, optional global-norm clip, Adam) as ONE kernel launch
    (``ops/csrc/ppo_train.hip``) for discrete MLP agents whose weights fit one CU's LDS (the
    ``exp=ppo`` CartPole agent does).  Semantics follow ``train`` / ``_minibatch_step`` (reference
    ``ppo.py:32-104``): same minibatch order source (a uniform permutation per epoch), the loss
    means are reported like ``PPOTrainer``'s graph outputs, and the optimiser's flat slabs
    (weights, Adam moments, step counter, last gradients) are updated in place."""

    def __init__(self, runner, agent, optimizer, cfg, n: int, plan):
        self.runner, self.agent, self.optimizer, self.cfg, self.n = runner, agent, optimizer, cfg, n
        self.layers, self.counts = plan
        dev = runner.device
        self.key = list(cfg.mlp_keys.encoder)[0]
        self.coefs = [torch.tensor([float(cfg.algo.clip_coef)], device=dev), torch.tensor([float(cfg.algo.ent_coef)], device=dev)]
        self.out = torch.zeros(3, device=dev)
        self.err = torch.zeros(1, device=dev)  # > 0: a grid-barrier wait of the multi-workgroup kernel timed out
        self.prof = torch.empty(0, dtype=torch.int64, device=dev)  # set to int64 [4] for phase cycle totals
        # workgroups per launch: one 16-row chunk of every minibatch each (grid barriers between steps)
        self.nwg = int(cfg.algo.get("fused_update_workgroups", 8))

    @staticmethod
    def plan(runner, agent, optimizer, cfg):
        """(layers, counts) for the kernel, or None when this setup is not covered."""
        from sheeprl_prey_amd import ops
        from sheeprl_prey_amd.parallel.flat_optim import FlatAdam

        if (runner.device.type != "cuda" or runner.world_size != 1 or not isinstance(optimizer, FlatAdam)
                or len(cfg.mlp_keys.encoder) != 1 or len(cfg.cnn_keys.encoder) != 0 or agent.is_continuous
                or str(cfg.algo.loss_reduction).lower() != "mean" or not ops.native_available()
                or getattr(runner, "_amp_dtype", None) is not None):
            return None
        chains = FusedCartPoleRollout.chains_of(agent)
        if chains is None:
            return None
        offs = {id(p): off for p, off in zip(optimizer.params, optimizer.offsets)}
        layers = []
        for W, B, A in chains:
            for w, b, a in zip(W, B, A):
                if id(w) not in offs or (b is not None and id(b) not in offs):
                    return None
                layers.append([w.shape[1], w.shape[0], a, offs[id(w)], offs[id(b)] if b is not None else -1])
        counts = [len(c[0]) for c in chains]
        D0 = layers[0][0]
        A = int(sum(agent.actions_dim))
        if not ops._ext().ppo_mlp_train_fits(layers, counts, D0, A):
            return None
        n_chain = sum(len(c[0]) + sum(b is not None for b in c[1]) for c in chains)
        if n_chain != sum(1 for _ in agent.parameters()):
            return None  # every trainable tensor of the agent must be a chain weight / bias
        return layers, counts

    def __call__(self, data: TensorDict, aggregator: Optional[MetricAggregator] = None,
                 perm: Optional[torch.Tensor] = None) -> None:
        from sheeprl_prey_amd import ops

        cfg, opt, n = self.cfg, self.optimizer, self.n
        dev = self.out.device
        if perm is None:  # one uniform permutation per epoch (minibatch order)
            perm = torch.argsort(torch.rand(int(cfg.algo.update_epochs), n, device=dev), dim=1)
        f = lambda k: data[k].reshape(n, -1).float().contiguous()  # noqa: E731
        cols = [f(self.key), f("actions"), f("logprobs").reshape(-1), f("values").reshape(-1), f("returns").reshape(-1),
                f("advantages").reshape(-1)]
        self.coefs[0].fill_(float(cfg.algo.clip_coef))
        self.coefs[1].fill_(float(cfg.algo.ent_coef))
        opt._gather()
        g = opt.param_groups[0]
        b1, b2 = g["betas"]
        ops._ext().ppo_mlp_train(self.layers, self.counts, cols, perm,
                                 [opt.flat_param, opt.flat_grad, opt.exp_avg, opt.exp_avg_sq, opt.scalars], self.coefs,
                                 self.out, int(cfg.per_rank_batch_size), float(cfg.algo.vf_coef),
                                 float(cfg.algo.max_grad_norm), bool(cfg.algo.clip_vloss),
                                 bool(cfg.algo.normalize_advantages), float(g["lr"]), float(b1), float(b2), float(g["eps"]),
                                 float(g["weight_decay"]), bool(opt.decoupled), self.nwg, self.err, self.prof)
        if aggregator is not None:
            for i, k in enumerate(("Loss/policy_loss", "Loss/value_loss", "Loss/entropy_loss")):
                aggregator.update(k, self.out[i].clone())


class SegmentedPPOUpdate:
    """The update as hipGraph replays with the gradient all-reduce between them (N ranks, GPU,
    ``fabric.cuda_graphs``): per minibatch ``fwd+bwd`` graph -> RCCL all-reduce of the flat gradient
    slab (eager, the reference's DDP averaging, ``ppo.py:41-52``) -> ``clip + Adam`` graph.  The
    minibatch rows come from a static index buffer refreshed by one device copy per minibatch, so
    one forward/backward graph serves every minibatch of a size (a ragged tail gets its own)."""

    def __init__(self, trainer: "PPOTrainer", warmup: int = 2):
        self.tr = trainer
        self.warmup = warmup
        self.calls = 0
        self.static = None
        self.g_fb: Dict[int, torch.cuda.CUDAGraph] = {}
        self.g_opt = None
        self.pool = None
        dev = trainer.runner.device
        self.sums = torch.zeros(3, device=dev)
        self.idx_cur = torch.zeros(max(1, int(trainer.cfg.per_rank_batch_size)), dtype=torch.long, device=dev)

    def _fb(self, m: int) -> None:
        tr, cfg = self.tr, self.tr.cfg
        sel = self.idx_cur[:m]
        batch = {k: v.index_select(0, sel) for k, v in self.static.items()}
        obs = {k: batch[k] / 255 - 0.5 if k in cfg.cnn_keys.encoder else batch[k] for k in tr.obs_keys}
        _, logprobs, entropy, new_values = tr.agent(obs, torch.split(batch["actions"], tr.agent.actions_dim, dim=-1))
        adv = batch["advantages"]
        if cfg.algo.normalize_advantages:
            adv = normalize_tensor(adv)
        pg = policy_loss(logprobs, batch["logprobs"], adv, tr.clip_t, cfg.algo.loss_reduction)
        vl = value_loss(new_values, batch["values"], batch["returns"], tr.clip_t, cfg.algo.clip_vloss, cfg.algo.loss_reduction)
        el = entropy_loss(entropy, cfg.algo.loss_reduction)
        loss = pg + cfg.algo.vf_coef * vl + tr.ent_t * el
        tr.optimizer.zero_grad(set_to_none=True)
        loss.backward()
        tr.optimizer._gather()  # the grads reach the flat slab inside this graph, before the all-reduce
        self.sums.add_(torch.stack((pg.detach(), vl.detach(), el.detach())))

    def _opt(self) -> None:
        tr, cfg = self.tr, self.tr.cfg
        if cfg.algo.max_grad_norm > 0.0:
            tr.runner.clip_gradients(tr.agent, tr.optimizer, max_norm=cfg.algo.max_grad_norm)
        tr.optimizer.step()

    def _run(self, key, fn) -> None:
        """Eager on a side stream while warming up, then capture once and replay."""
        graphs = self.g_fb if key != "opt" else None
        g = graphs.get(key) if graphs is not None else self.g_opt
        if g is not None:
            g.replay()
            return
        if self.calls < self.warmup:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                fn()
            torch.cuda.current_stream().wait_stream(s)
            return
        g = torch.cuda.CUDAGraph()
        from sheeprl_prey_amd.parallel.graphs import capture_error_mode, quiesce_for_capture

        quiesce_for_capture()
        with torch.cuda.graph(g, pool=self.pool, capture_error_mode=capture_error_mode()):
            fn()
        self.pool = g.pool()
        if graphs is not None:
            graphs[key] = g
        else:
            self.g_opt = g
        g.replay()  # capture recorded without running

    def __call__(self, data: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        tr, cfg = self.tr, self.tr.cfg
        n, bs = tr.n, int(cfg.per_rank_batch_size)
        if self.static is None:
            self.static = {k: v.detach().clone() for k, v in data.items()}
        for k, v in data.items():
            self.static[k].copy_(v, non_blocking=True)
        dev = self.sums.device
        self.sums.zero_()
        steps = 0
        share = bool(cfg.buffer.share_data) and tr.runner.world_size > 1
        for epoch in range(cfg.algo.update_epochs):
            if share:  # DistributedSampler semantics over the gathered rollout (reference ppo.py:41-52)
                perm = shard_indices(n, tr.runner, True, cfg.seed, epoch).to(dev, non_blocking=True)
            else:
                perm = torch.argsort(torch.rand(n, device=dev))
            for start in range(0, perm.numel(), bs):
                m = min(bs, perm.numel() - start)
                self.idx_cur[:m].copy_(perm[start:start + m])
                self._run(m, lambda m=m: self._fb(m))
                tr.runner.sync_gradients(tr.optimizer)
                self._run("opt", self._opt)
                steps += 1
        self.calls += 1
        out = self.sums / max(1, steps)
        return {"Loss/policy_loss": out[0], "Loss/value_loss": out[1], "Loss/entropy_loss": out[2]}


class PPOTrainer:
    """All ``update_epochs`` x minibatch steps of one PPO update:

    * one rank, GPU, ``fabric.cuda_graphs``: the fused one-launch kernel when the agent fits it
      (``FusedPPOTrainer``), else ONE hipGraph for the whole update - permutations drawn on device
      (``argsort`` of uniform keys), clip / entropy coefficients as device scalars refreshed before
      each replay (annealing works), the loss means as graph outputs;
    * N ranks (or ``force_segmented``): ``SegmentedPPOUpdate`` - graph replays with the per-minibatch
      RCCL all-reduce between them;
    * ``anneal_lr`` (the flat Adam takes its lr as a launch argument) or CPU: eager ``train``."""

    def __init__(self, runner, agent, optimizer, cfg, n: int, force_segmented: bool = False):
        from sheeprl_prey_amd.parallel.graphs import GraphedStep

        self.runner, self.agent, self.optimizer, self.cfg, self.n = runner, agent, optimizer, cfg, n
        dev = runner.device
        self.obs_keys = list(cfg.mlp_keys.encoder) + list(cfg.cnn_keys.encoder)
        self.clip_t = torch.tensor(float(cfg.algo.clip_coef), device=dev)
        self.ent_t = torch.tensor(float(cfg.algo.ent_coef), device=dev)
        graphs = dev.type == "cuda" and bool(getattr(runner, "cuda_graphs", False)) and not cfg.algo.anneal_lr
        ws = runner.world_size
        self.segmented = SegmentedPPOUpdate(self) if graphs and (ws > 1 or force_segmented) else None
        self.graphed = GraphedStep(self._train, warmup=2, enabled=graphs and self.segmented is None, name="ppo_train")
        # DistributedSampler permutations of the shared rollout (seeded per epoch, the same every update as in
        # the reference's sampler.set_epoch(epoch) loop): built once, static inputs of the captured update
        self._share_perms = None
        if bool(cfg.buffer.share_data) and ws > 1:
            self._share_perms = [shard_indices(n, runner, True, cfg.seed, e).to(dev) for e in range(cfg.algo.update_epochs)]
        from sheeprl_prey_amd import ops

        plan = (FusedPPOTrainer.plan(runner, agent, optimizer, cfg)
                if cfg.algo.get("fused_update", True) and ops._FUSED and self.segmented is None else None)
        self.fused = FusedPPOTrainer(runner, agent, optimizer, cfg, n, plan) if plan is not None else None

    @property
    def mode(self) -> str:
        if self.fused is not None:
            return "fused"
        if self.segmented is not None:
            return "segmented"
        if self.graphed.enabled:
            return "graph"
        return "eager"

    def _train(self, data: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        cfg = self.cfg
        n, bs = self.n, cfg.per_rank_batch_size
        dev = data["rewards"].device
        sums = torch.zeros(3, device=dev)
        steps = 0
        for epoch in range(cfg.algo.update_epochs):
            idx = self._share_perms[epoch] if self._share_perms is not None else torch.argsort(torch.rand(n, device=dev))
            for start in range(0, idx.numel(), bs):
                sel = idx[start : start + bs]
                batch = {k: v.index_select(0, sel) for k, v in data.items()}
                pg, vl, el = _minibatch_step(self.runner, self.agent, self.optimizer, batch, self.obs_keys, cfg,
                                             self.clip_t, self.ent_t)
                sums = sums + torch.stack((pg.detach(), vl.detach(), el.detach()))
                steps += 1
        sums = sums / steps
        return {"Loss/policy_loss": sums[0], "Loss/value_loss": sums[1], "Loss/entropy_loss": sums[2]}

    def __call__(self, data: TensorDict, aggregator: Optional[MetricAggregator] = None) -> None:
        if self.fused is not None:
            self.fused(data, aggregator)
            return
        if self.segmented is None and not self.graphed.enabled:
            train(self.runner, self.agent, self.optimizer, data, aggregator, self.cfg)
            return
        self.clip_t.fill_(float(self.cfg.algo.clip_coef))
        self.ent_t.fill_(float(self.cfg.algo.ent_coef))
        inputs = {k: data[k] for k in data.keys()}
        out = self.segmented(inputs) if self.segmented is not None else self.graphed(inputs)
        if aggregator is not None:
            for k, v in out.items():
                aggregator.update(k, v.clone())


class PPOPlayer:
    """Rollout policy step (reference ``ppo.py:289-300``): forward + sampling, returning the one-hot
    actions, env actions, log-probs and values.  With ``fabric.cuda_graphs`` on GPU the whole step
    is one hipGraph replay (sampling via Philox, graph-safe); outputs are static buffers the caller
    copies (``ReplayBuffer.add``) before the next call."""

    def __init__(self, agent, cfg, is_continuous: bool, enabled: bool):
        from sheeprl_prey_amd.parallel.graphs import GraphedStep

        self.agent, self.cfg, self.is_continuous = agent, cfg, is_continuous
        self.graphed = GraphedStep(self._step, warmup=2, enabled=enabled, name="ppo_player")

    @torch.no_grad()
    def _step(self, obs: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        nobs = {k: v / 255 - 0.5 if k in self.cfg.cnn_keys.encoder else v for k, v in obs.items()}
        actions, logprobs, _, values = self.agent(nobs)
        if self.is_continuous:
            real = torch.cat(actions, -1)
        else:
            real = torch.stack([a.argmax(dim=-1) for a in actions], dim=-1)
        return {"actions": torch.cat(actions, -1), "real": real, "logprobs": logprobs, "values": values}

    def __call__(self, obs: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        return self.graphed(obs)


class HostRollout:
    """The rollout loop (reference ``ppo.py:281-356``, decoupled actor ``ppo_decoupled.py:115-190``) against
    host (CPU) vector envs, with every rollout tensor device-resident ``[T, N, ...]``:

        per env step: next obs -> pinned staging -> (H2D inside the player's copy-in) -> ONE graphed
        policy replay (``PPOPlayer``) -> obs / actions / log-probs / values copied into slot t on the
        device -> env actions read back into pinned memory (the only sync) -> env.step on the CPU;
        rewards / dones land in host arrays, moved H2D once per rollout.

    Image observations stay uint8 end to end (the player normalises on the device).  A truncated
    episode's reward is bootstrapped with V(final obs) as in the reference (eager, rare).  ``obs``
    holds the device observation after the last step (the GAE bootstrap input)."""

    def __init__(self, agent, envs, cfg, player: "PPOPlayer", device, obs_keys, first_obs) -> None:
        self.agent, self.envs, self.cfg, self.player, self.device = agent, envs, cfg, player, device
        self.obs_keys = list(obs_keys)
        self.cnn = set(cfg.cnn_keys.encoder)
        self.T, self.N = int(cfg.algo.rollout_steps), int(cfg.env.num_envs)
        T, N = self.T, self.N
        A = int(sum(agent.actions_dim))
        cur = self._prep(first_obs)
        pin = device.type == "cuda"
        self.pinned = {k: torch.from_numpy(v.copy()) for k, v in cur.items()}
        if pin:
            self.pinned = {k: v.pin_memory() for k, v in self.pinned.items()}
        self.obs = {k: v.to(device) for k, v in self.pinned.items()}
        self.buf = {k: torch.zeros((T, N) + tuple(v.shape[1:]), dtype=v.dtype, device=device) for k, v in self.obs.items()}
        self.buf.update({"actions": torch.zeros(T, N, A, device=device), "logprobs": torch.zeros(T, N, 1, device=device),
                         "values": torch.zeros(T, N, 1, device=device)})
        self.rew_host = torch.zeros(T, N, 1)
        self.done_host = torch.zeros(T, N, 1)
        if pin:  # (re-written only after the next rollout's first sync: the previous H2D has finished)
            self.rew_host, self.done_host = self.rew_host.pin_memory(), self.done_host.pin_memory()
        self.real_pin = None
        self.episodes: List[Tuple[float, float]] = []

    def _prep(self, o) -> Dict[str, np.ndarray]:
        out = {}
        for k in self.obs_keys:
            a = np.asarray(o[k])
            out[k] = a.reshape(self.N, -1, *a.shape[-2:]) if k in self.cnn else a.astype(np.float32, copy=False)
        return out

    @torch.no_grad()
    def __call__(self) -> Dict[str, Tensor]:
        envs, buf, graphed = self.envs, self.buf, self.player.graphed
        self.episodes = []
        for t in range(self.T):
            use_pinned = graphed.enabled and graphed.graph is not None
            pout = self.player(self.pinned if use_pinned else self.obs)
            src = graphed.static_in if use_pinned else self.obs
            for k in self.obs_keys:
                buf[k][t].copy_(src[k])
            for n in ("actions", "logprobs", "values"):
                buf[n][t].copy_(pout[n])
            real = pout["real"]
            if real.is_cuda:
                if self.real_pin is None:
                    self.real_pin = torch.empty(real.shape, dtype=real.dtype).pin_memory()
                self.real_pin.copy_(real, non_blocking=True)
                torch.cuda.current_stream().synchronize()
                real_np = self.real_pin.numpy()
            else:
                real_np = real.numpy()
            o, rewards, dones, truncated, info = envs.step(real_np.reshape(envs.action_space.shape))
            trunc = np.nonzero(truncated)[0]
            if len(trunc) > 0:  # truncation bootstrap r += V(final obs), as the reference
                final = {}
                for k in self.obs_keys:
                    v = torch.as_tensor(np.stack([np.asarray(info["final_observation"][e][k]) for e in trunc]),
                                        dtype=torch.float32, device=self.device)
                    final[k] = v.view(len(trunc), -1, *v.shape[-2:]) / 255.0 - 0.5 if k in self.cnn else v
                rewards = np.asarray(rewards, dtype=np.float32).copy()
                rewards[trunc] += self.agent.get_value(final).cpu().numpy().reshape(rewards[trunc].shape)
            self.rew_host[t, :, 0] = torch.from_numpy(np.asarray(rewards, dtype=np.float32).reshape(self.N))
            self.done_host[t, :, 0] = torch.from_numpy(np.logical_or(dones, truncated).astype(np.float32).reshape(self.N))
            cur = self._prep(o)
            for k in self.obs_keys:
                self.pinned[k].numpy()[...] = cur[k]
                if not use_pinned or t == self.T - 1:
                    self.obs[k].copy_(self.pinned[k], non_blocking=self.pinned[k].is_pinned())
            for _, ep_rew, ep_len in episode_stats(info):
                for r, n_ in zip(np.asarray(ep_rew).reshape(-1), np.asarray(ep_len).reshape(-1)):
                    self.episodes.append((float(r), float(n_)))
        out = dict(buf)
        out["rewards"] = self.rew_host.to(self.device, non_blocking=True)
        out["dones"] = self.done_host.to(self.device, non_blocking=True)
        return out


class DeviceRollout:
    """The rollout loop (reference ``ppo.py:281-356``) against a device-resident env
    (``envs/device.py``): ``rollout_steps`` x (policy forward + sampling, env step with autoreset,
    truncation bootstrap ``r += V(final_obs)``, buffer writes) with no host round trip, captured as
    ONE hipGraph (``fabric.cuda_graphs``) and replayed once per update.  Buffers are [T, N, ...]."""

    def __init__(self, agent, env, cfg, enabled: bool):
        from sheeprl_prey_amd.parallel.graphs import GraphedStep

        self.agent, self.env, self.cfg = agent, env, cfg
        T, N, dev = cfg.algo.rollout_steps, env.num_envs, env.device
        A = int(sum(agent.actions_dim))
        z = lambda *s: torch.zeros(*s, device=dev)  # noqa: E731
        self.buf = {"state": z(T, N, 4), "actions": z(T, N, A), "logprobs": z(T, N, 1), "values": z(T, N, 1),
                    "rewards": z(T, N, 1), "dones": z(T, N, 1)}
        self.stats = {"done_ret": z(T, N), "done_len": z(T, N)}
        self.graphed = GraphedStep(self._rollout, warmup=2, enabled=enabled, name="ppo_device_rollout")

    @torch.no_grad()
    def _rollout(self, _data: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        env, agent, buf = self.env, self.agent, self.buf
        for t in range(self.cfg.algo.rollout_steps):
            obs = env.obs
            buf["state"][t].copy_(obs)
            actions, logprobs, _, values = agent({"state": obs})
            idx = actions[0].argmax(-1)
            out = env.step(idx)
            v_final = agent.get_value({"state": out["final_obs"]})
            buf["actions"][t].copy_(torch.cat(actions, -1))
            buf["logprobs"][t].copy_(logprobs)
            buf["values"][t].copy_(values)
            buf["rewards"][t].copy_(out["reward"].unsqueeze(-1) + out["truncated"].unsqueeze(-1) * v_final)
            buf["dones"][t].copy_(torch.maximum(out["terminated"], out["truncated"]).unsqueeze(-1))
            self.stats["done_ret"][t].copy_(out["done_ret"])
            self.stats["done_len"][t].copy_(out["done_len"])
        return {}

    def __call__(self) -> Dict[str, torch.Tensor]:
        self.graphed({})
        return self.buf

    def finished_episodes(self):
        """(returns, lengths) of the episodes that ended during the last rollout (one D2H)."""
        r = self.stats["done_ret"].reshape(-1).cpu()
        n = self.stats["done_len"].reshape(-1).cpu()
        m = n > 0
        return r[m].tolist(), n[m].tolist()


_CHAIN_ACTS = {nn.Tanh: 4, nn.ReLU: 3, nn.SiLU: 1, nn.ELU: 2}


def _mlp_chain(seq: nn.Module):
    """``[Linear, act?]*`` -> (weights, biases, act codes) for the fused rollout kernel, or None when
    the stack holds anything else (LayerNorm, active dropout, widths > 256)."""
    W, B, A = [], [], []
    for m in ([seq] if isinstance(seq, nn.Linear) else list(seq)):
        if isinstance(m, nn.Linear):
            if max(m.weight.shape) > 256 or m.weight.dtype != torch.float32:
                return None
            W.append(m.weight)
            B.append(m.bias)
            A.append(0)
        elif type(m) in _CHAIN_ACTS:
            if not A or A[-1] != 0:
                return None
            A[-1] = _CHAIN_ACTS[type(m)]
        elif isinstance(m, nn.Identity) or (isinstance(m, nn.Dropout) and (m.p == 0 or not m.training)):
            continue
        else:
            return None
    return (W, B, A) if 1 <= len(W) <= 8 else None


class FusedCartPoleRollout:
    """The whole rollout (reference ``ppo.py:281-356``) as ONE kernel launch
    (``ops/csrc/ppo_rollout.hip``): a workgroup per env runs the T steps of policy MLPs,
    categorical sampling, CartPole step with autoreset and truncation bootstrap back to back.
    Same buffers / ``finished_episodes`` contract as :class:`DeviceRollout`; applies to discrete
    MLP-only agents on ``CartPoleDevice`` (``FusedCartPoleRollout.supported``)."""

    def __init__(self, agent, env, cfg, seed: int = 0, lds_weights: bool = True):
        self.agent, self.env, self.lds_weights = agent, env, lds_weights
        T, N, dev = cfg.algo.rollout_steps, env.num_envs, env.device
        z = lambda *s: torch.zeros(*s, device=dev)  # noqa: E731
        self.buf = {"state": z(T, N, 4), "actions": z(T, N, 2), "logprobs": z(T, N, 1), "values": z(T, N, 1),
                    "rewards": z(T, N, 1), "dones": z(T, N, 1)}
        self.stats = {"done_ret": z(T, N), "done_len": z(T, N)}
        self.chains = self.chains_of(agent)
        assert self.chains is not None, "agent not supported by the fused rollout"
        self.seed = int(seed) * 1000003

    @staticmethod
    def chains_of(agent):
        fe = agent.feature_extractor
        if fe.has_cnn_encoder or not fe.has_mlp_encoder or agent.is_continuous or len(agent.actor_heads) != 1:
            return None
        chains = [_mlp_chain(fe.mlp_encoder.model.model), _mlp_chain(agent.actor_backbone.model),
                  _mlp_chain(agent.actor_heads[0]), _mlp_chain(agent.critic.model)]
        return None if any(c is None for c in chains) else chains

    @classmethod
    def supported(cls, agent, env) -> bool:
        from sheeprl_prey_amd.envs.device import CartPoleDevice

        return (isinstance(env, CartPoleDevice) and env.device.type == "cuda" and list(agent.actions_dim) == [2]
                and not getattr(agent, "_srl_autocast", False)  # bf16-mixed: the agent's autocast forward instead
                and cls.chains_of(agent) is not None)

    @torch.no_grad()
    def __call__(self) -> Dict[str, torch.Tensor]:
        from sheeprl_prey_amd import ops

        e, a, h, c = self.chains
        env, b = self.env, self.buf
        self.seed += 1
        ops._ext().ppo_cartpole_rollout(*e, *a, *h, *c, env.state, env.steps, env.ep_ret, env.obs,
                                        [b["state"], b["actions"], b["logprobs"], b["values"], b["rewards"], b["dones"],
                                         self.stats["done_ret"], self.stats["done_len"]],
                                        env.max_steps, self.seed & 0x7FFFFFFFFFFFFFFF, self.lds_weights)
        return b

    finished_episodes = DeviceRollout.finished_episodes


@register_algorithm()
def main(runner, cfg: Dict[str, Any]):
    cfg, state = load_resume(runner, cfg)
    initial_ent_coef = copy.deepcopy(cfg.algo.ent_coef)
    initial_clip_coef = copy.deepcopy(cfg.algo.clip_coef)
    device = runner.device
    rank, world_size = runner.global_rank, runner.world_size
    runner.seed_everything(cfg.seed + rank)

    logger, log_dir = setup_logger(runner, cfg)
    envs = build_envs(runner, cfg, log_dir)
    observation_space = envs.single_observation_space
    check_obs_keys(cfg, observation_space)
    runner.print("Encoder CNN keys:", cfg.cnn_keys.encoder)
    runner.print("Encoder MLP keys:", cfg.mlp_keys.encoder)
    obs_keys = list(cfg.cnn_keys.encoder) + list(cfg.mlp_keys.encoder)
    is_continuous, _, actions_dim = action_info(envs.single_action_space)

    agent = PPOAgent(actions_dim, observation_space, cfg.algo.encoder, cfg.algo.actor, cfg.algo.critic,
                     cfg.cnn_keys.encoder, cfg.mlp_keys.encoder, cfg.env.screen_size, cfg.distribution, is_continuous)
    if state:
        agent.load_state_dict(state["agent"])
    agent = runner.setup_module(agent)
    optimizer = build_optimizer(cfg.algo.optimizer, agent.parameters())
    if state:
        optimizer.load_state_dict(state["optimizer"])

    aggregator = MetricAggregator({
        "Rewards/rew_avg": MeanMetric(sync_on_compute=cfg.metric.sync_on_compute),
        "Game/ep_len_avg": MeanMetric(sync_on_compute=cfg.metric.sync_on_compute),
        "Loss/value_loss": MeanMetric(sync_on_compute=cfg.metric.sync_on_compute),
        "Loss/policy_loss": MeanMetric(sync_on_compute=cfg.metric.sync_on_compute),
        "Loss/entropy_loss": MeanMetric(sync_on_compute=cfg.metric.sync_on_compute),
    })

    if cfg.buffer.size < cfg.algo.rollout_steps:
        raise ValueError(f"The size of the buffer ({cfg.buffer.size}) cannot be lower than the rollout steps ({cfg.algo.rollout_steps})")
    rb = ReplayBuffer(cfg.buffer.size, cfg.env.num_envs, device=device, memmap=cfg.buffer.memmap and device.type == "cpu",
                      memmap_dir=os.path.join(log_dir, "memmap_buffer", f"rank_{rank}"), obs_keys=obs_keys)
    step_data = TensorDict({}, batch_size=[cfg.env.num_envs], device=device)

    last_train = 0
    train_step = 0
    start_step = state["update"] // world_size if state else 1
    policy_step = state["update"] * cfg.env.num_envs * cfg.algo.rollout_steps if state else 0
    last_log = state["last_log"] if state else 0
    last_checkpoint = state["last_checkpoint"] if state else 0
    policy_steps_per_update = int(cfg.env.num_envs * cfg.algo.rollout_steps * world_size)
    num_updates = cfg.total_steps // policy_steps_per_update if not cfg.dry_run else 1
    warn_log_ckpt_every(cfg, policy_steps_per_update)

    scheduler = None
    if cfg.algo.anneal_lr:
        scheduler = PolynomialLR(optimizer, total_iters=num_updates, power=1.0)
        if state and state.get("scheduler"):
            scheduler.load_state_dict(state["scheduler"])

    trainer = None
    player = PPOPlayer(agent, cfg, is_continuous, enabled=device.type == "cuda" and bool(runner.cuda_graphs))
    o = envs.reset(seed=cfg.seed)[0]
    next_obs = {}
    for k in obs_keys:
        t = torch.as_tensor(o[k]).to(device)
        if k in cfg.cnn_keys.encoder:
            t = t.view(cfg.env.num_envs, -1, *t.shape[-2:])
        else:
            t = t.float()
        step_data[k] = t
        next_obs[k] = t

    # env.device=True: the envs live on the GPU (envs/device.py) and the whole rollout is one
    # launch (FusedCartPoleRollout) or one hipGraph replay (DeviceRollout)
    drollout = None
    if cfg.env.get("device", False):
        from sheeprl_prey_amd.envs.device import make_device_env

        if device.type != "cuda" or obs_keys != ["state"] or cfg.cnn_keys.encoder:
            raise ValueError("env.device=True needs a GPU run with mlp_keys.encoder=[state] and no cnn keys")
        denv = make_device_env(cfg.env.id, cfg.env.num_envs, device, seed=cfg.seed + rank * cfg.env.num_envs,
                               max_episode_steps=cfg.env.max_episode_steps)
        denv.reset()
        if FusedCartPoleRollout.supported(agent, denv):
            drollout = FusedCartPoleRollout(agent, denv, cfg, seed=cfg.seed + rank)
        else:
            drollout = DeviceRollout(agent, denv, cfg, enabled=bool(runner.cuda_graphs))

    for update in range(start_step, num_updates + 1):
        if drollout is not None:
            policy_step += cfg.env.num_envs * world_size * cfg.algo.rollout_steps
            with timer("Time/env_interaction_time"):
                buf = drollout()
                rb.add(TensorDict(dict(buf), batch_size=[cfg.algo.rollout_steps, cfg.env.num_envs]))
                next_obs = {"state": denv.obs}
            rets, lens = drollout.finished_episodes()
            for r, n_ in zip(rets, lens):
                aggregator.update("Rewards/rew_avg", r)
                aggregator.update("Game/ep_len_avg", n_)
            if rets:
                runner.print(f"Rank-{rank}: policy_step={policy_step}, episodes={len(rets)}, last_reward={rets[-1]}")
        for _ in range(cfg.algo.rollout_steps if drollout is None else 0):
            policy_step += cfg.env.num_envs * world_size
            with timer("Time/env_interaction_time"):
                pout = player({k: next_obs[k] for k in obs_keys})
                actions, logprobs, values = pout["actions"], pout["logprobs"], pout["values"]
                real_actions = pout["real"].cpu().numpy()
                o, rewards, dones, truncated, info = envs.step(real_actions.reshape(envs.action_space.shape))
                truncated_envs = np.nonzero(truncated)[0]
                if len(truncated_envs) > 0:
                    # bootstrap truncated episodes with V(final_observation)
                    real_next = {}
                    for k in obs_keys:
                        vals = np.stack([np.asarray(info["final_observation"][e][k]) for e in truncated_envs])
                        tv = torch.as_tensor(vals, dtype=torch.float32, device=device)
                        if k in cfg.cnn_keys.encoder:
                            tv = tv.view(len(truncated_envs), -1, *tv.shape[-2:]) / 255.0 - 0.5
                        real_next[k] = tv
                    with torch.no_grad():
                        v = agent.get_value(real_next).cpu().numpy()
                    rewards[truncated_envs] += v.reshape(rewards[truncated_envs].shape)
                dones = np.logical_or(dones, truncated)
                dones = torch.as_tensor(dones, dtype=torch.float32, device=device).view(cfg.env.num_envs, -1)
                rewards = torch.as_tensor(rewards, dtype=torch.float32, device=device).view(cfg.env.num_envs, -1)

            step_data["dones"] = dones
            step_data["values"] = values
            step_data["actions"] = actions
            step_data["logprobs"] = logprobs
            step_data["rewards"] = rewards
            step_data["returns"] = torch.zeros_like(rewards)
            step_data["advantages"] = torch.zeros_like(rewards)
            rb.add(step_data.unsqueeze(0))

            next_obs = {}
            for k in obs_keys:
                if k in cfg.cnn_keys.encoder:
                    t = torch.as_tensor(o[k], device=device)
                    t = t.view(cfg.env.num_envs, -1, *t.shape[-2:])
                else:
                    t = torch.as_tensor(o[k], device=device, dtype=torch.float32)
                step_data[k] = t
                next_obs[k] = t

            for i, ep_rew, ep_len in episode_stats(info):
                aggregator.update("Rewards/rew_avg", ep_rew)
                aggregator.update("Game/ep_len_avg", ep_len)
                runner.print(f"Rank-0: policy_step={policy_step}, reward_env_{i}={ep_rew[-1]}")

        with torch.no_grad():
            nobs = {k: next_obs[k] / 255 - 0.5 if k in cfg.cnn_keys.encoder else next_obs[k] for k in obs_keys}
            next_values = agent.get_value(nobs)
            returns, advantages = gae(rb["rewards"], rb["values"], rb["dones"], next_values, cfg.algo.rollout_steps,
                                      cfg.algo.gamma, cfg.algo.gae_lambda)
            rb["returns"] = returns.float()
            rb["advantages"] = advantages.float()

        local_data = rb.buffer.view(-1)
        if cfg.buffer.share_data and world_size > 1:
            gathered = runner.all_gather(local_data.to_dict())
            n = next(iter(gathered.values())).shape[0] * local_data.shape[0]
            local_data = TensorDict({k: v.reshape(n, *v.shape[2:]) for k, v in gathered.items()}, batch_size=[n])
        with timer("Time/train_time"):
            if trainer is None or trainer.n != local_data.shape[0]:
                trainer = PPOTrainer(runner, agent, optimizer, cfg, local_data.shape[0])
            trainer(local_data, aggregator)
        train_step += world_size

        if cfg.algo.anneal_lr:
            runner.log("Info/learning_rate", scheduler.get_last_lr()[0], policy_step)
            scheduler.step()
        else:
            runner.log("Info/learning_rate", cfg.algo.optimizer.lr, policy_step)
        runner.log("Info/clip_coef", cfg.algo.clip_coef, policy_step)
        if cfg.algo.anneal_clip_coef:
            cfg.algo.clip_coef = polynomial_decay(update, initial=initial_clip_coef, final=0.0, max_decay_steps=num_updates)
        runner.log("Info/ent_coef", cfg.algo.ent_coef, policy_step)
        if cfg.algo.anneal_ent_coef:
            cfg.algo.ent_coef = polynomial_decay(update, initial=initial_ent_coef, final=0.0, max_decay_steps=num_updates)

        if policy_step - last_log >= cfg.metric.log_every or update == num_updates or cfg.dry_run:
            runner.log_dict(aggregator.compute(), policy_step)
            aggregator.reset()
            log_throughput(runner, timer.compute(), policy_step, last_log, train_step, last_train, cfg.env.action_repeat)
            timer.reset()
            last_log = policy_step
            last_train = train_step

        if (cfg.checkpoint.every > 0 and policy_step - last_checkpoint >= cfg.checkpoint.every) or cfg.dry_run or update == num_updates:
            last_checkpoint = policy_step
            ckpt_state = {
                "agent": agent.state_dict(),
                "optimizer": optimizer.state_dict(),
                "scheduler": scheduler.state_dict() if scheduler is not None else None,
                "update": update * world_size,
                "batch_size": cfg.per_rank_batch_size * world_size,
                "last_log": last_log,
                "last_checkpoint": last_checkpoint,
            }
            ckpt_path = os.path.join(log_dir, f"checkpoint/ckpt_{policy_step}_{rank}.ckpt")
            runner.call("on_checkpoint_coupled", ckpt_path=ckpt_path, state=ckpt_state)

    envs.close()
    if runner.is_global_zero:
        test(agent, runner, cfg, log_dir)
