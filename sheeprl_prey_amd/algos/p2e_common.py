"""Plan2Explore on top of DreamerV1 / DreamerV2 (reference: ``sheeprl/algos/p2e_dv1/p2e_dv1.py:36-876``,
``sheeprl/algos/p2e_dv2/p2e_dv2.py:36-1081``; "Planning to Explore via Self-Supervised World Models").

The disagreement ensemble (``ensembles.n`` MLPs predicting the next posterior (DV2) / next obs
embedding (DV1)) is ONE ``EnsembleMLP``: every layer of all members is a single (batched) GEMM, and
the intrinsic reward ``var_members(prediction).mean(-1)`` is computed from one stacked output.

A gradient step while exploring is a ``PhasedStep`` of seven phases:
  wm | ensemble (wm step, ensemble NLL) | exploration actor (ensemble step, imagination with the
  exploration actor, intrinsic lambda returns) | exploration critic | task actor | task critic | final
separated by the corresponding gradient all-reduces; after ``exploration_steps`` only the task
phases run (``wm | task actor | task critic | final``).
"""
from __future__ import annotations

from typing import Any, Dict, Optional, Sequence

import torch
import torch.nn as nn
from torch import Tensor

from sheeprl_prey_amd import ops
from sheeprl_prey_amd.models.ensemble import EnsembleLinear, EnsembleMLP
from sheeprl_prey_amd.parallel.flat_optim import flatten_like
from sheeprl_prey_amd.parallel.graphs import PhasedStep

P2E_METRICS = (
    "Loss/world_model_loss", "Loss/value_loss_task", "Loss/policy_loss_task", "Loss/value_loss_exploration",
    "Loss/policy_loss_exploration", "Loss/observation_loss", "Loss/reward_loss", "Loss/state_loss",
    "Loss/continue_loss", "Loss/ensemble_loss", "State/kl", "State/p_entropy", "State/q_entropy",
    "Params/exploration_amout", "Rewards/intrinsic", "Values_exploration/predicted_values",
    "Values_exploration/lambda_values", "Grads/world_model", "Grads/actor_task", "Grads/critic_task",
    "Grads/actor_exploration", "Grads/critic_exploration", "Grads/ensemble", "Rewards/rew_avg", "Game/ep_len_avg",
)


def build_ensembles(cfg, input_dim: int, output_dim: int, device) -> EnsembleMLP:
    """``n`` members, each initialised with its own seed (``cfg.seed + i``, as the reference does) by
    Kaiming-uniform weights and zero biases (``utils.init_weights``)."""
    ec = cfg.algo.ensembles
    ens = EnsembleMLP(ec.n, input_dim, [ec.dense_units] * ec.mlp_layers, output_dim, activation=ec.dense_act,
                      layer_norm=bool(ec.get("layer_norm", False)))
    with torch.no_grad():
        for i in range(ec.n):
            g = torch.Generator().manual_seed(int(cfg.seed) + i)
            for m in ens.modules():
                if isinstance(m, EnsembleLinear):
                    w = m.weight[i]
                    bound = (6.0 / w.shape[1]) ** 0.5  # kaiming_uniform_(a=0): sqrt(6 / fan_in)
                    w.copy_(torch.empty_like(w).uniform_(-bound, bound, generator=g))
                    if m.bias is not None:
                        m.bias[i].zero_()
    return ens.to(device)


class P2EMixin:
    """Adds the exploration phases to a DreamerV1/V2 trainer (``self`` is the task trainer).

    ``flavor`` "dv2": the ensemble predicts the next (flattened) posterior; exploration actor
    objective = dynamics (continuous) / REINFORCE (discrete).  "dv1": it predicts the next obs
    embedding; actor loss -mean(discount*lambda) through the world model."""

    def setup_p2e(self, flavor: str, actor_expl, critic_expl, target_critic_expl, ensembles: EnsembleMLP,
                  ensemble_optimizer, actor_expl_optimizer, critic_expl_optimizer) -> None:
        self.flavor = flavor
        self.actor_expl, self.critic_expl, self.target_critic_expl = actor_expl, critic_expl, target_critic_expl
        self.ensembles = ensembles
        self.ensemble_optimizer = ensemble_optimizer
        self.actor_expl_optimizer, self.critic_expl_optimizer = actor_expl_optimizer, critic_expl_optimizer
        self.actor_expl_params = [p for p in actor_expl.parameters() if p.requires_grad]
        self.critic_expl_params = [p for p in critic_expl.parameters() if p.requires_grad]
        self.ensemble_params = [p for p in ensembles.parameters() if p.requires_grad]
        self.target_expl_flat = (flatten_like(target_critic_expl, critic_expl_optimizer)
                                 if target_critic_expl is not None else None)
        self.detach_heads = True
        g = bool(self.cfg.fabric.get("cuda_graphs", False))
        c = self._coll
        self.explore_step = PhasedStep(
            self.runner,
            [self._phase_wm, self._phase_ensemble, self._phase_expl_actor, self._phase_expl_critic,
             self._phase_task_actor, self._phase_critic_task, self._phase_final_task],
            [c(self.world_optimizer, True), c(ensemble_optimizer), c(actor_expl_optimizer), c(critic_expl_optimizer),
             c(self.actor_optimizer), c(self.critic_optimizer)], graphs=g, name="p2e_explore")
        self.task_step = PhasedStep(
            self.runner, [self._phase_wm, self._phase_task_actor_wm, self._phase_critic_task, self._phase_final_task],
            [c(self.world_optimizer, True), c(self.actor_optimizer), c(self.critic_optimizer)], graphs=g, name="p2e_task")
        self.is_exploring = True

    def train_step(self, data: Dict[str, Tensor]) -> Dict[str, Tensor]:
        return self.explore_step(data) if self.is_exploring else self.task_step(data)

    @torch.no_grad()
    def update_targets(self) -> None:
        self.update_target(1.0)
        if self.target_expl_flat is not None:
            self.target_expl_flat.copy_(self.critic_expl_optimizer.flat_param)

    # ------------------------------------------------------------------ ensemble
    def _ensemble_inputs(self, data) -> Tensor:
        st = self._st
        post = st["posteriors"]
        post = post.reshape(*post.shape[:2], -1)
        return torch.cat((post, st["recurrent_states"], data["actions"]), -1)

    def _ensemble_targets(self) -> Tensor:
        st = self._st
        if self.flavor == "dv2":
            post = st["posteriors"]
            return post.reshape(*post.shape[:2], -1)[1:]
        return st["embedded"][1:]

    def _phase_ensemble(self, data) -> None:
        st = self._st
        self._wm_step()
        inp = self._ensemble_inputs(data)
        pred = self.ensembles(inp.reshape(-1, inp.shape[-1]))
        n = self.ensembles.n
        T, B = data["rewards"].shape[:2]
        pred = pred.view(n, T, B, -1)[:, :-1]
        target = self._ensemble_targets().unsqueeze(0)
        from sheeprl_prey_amd.algos.dreamer_v2.loss import normal_nll

        # sum over members of the mean unit-Normal NLL of the next-step target
        loss = normal_nll(pred, target.expand_as(pred), 1).mean(dim=(1, 2)).sum()
        self.ensemble_optimizer.zero_grad()
        loss.backward(inputs=self.ensemble_params)
        st["out"]["Loss/ensemble_loss"] = loss.detach()

    def _intrinsic_reward(self, traj: Tensor, acts: Tensor) -> Tensor:
        with torch.no_grad():
            x = torch.cat((traj.detach(), acts.detach()), -1)
            lead = x.shape[:-1]
            ens = self.ensembles
            # member head GEMMs + variance over members + mean over features: one kernel on the GPU (K20)
            r = ops.ensemble_disagreement(ens.hidden(x.reshape(-1, x.shape[-1])), ens.head.weight, ens.head.bias)
            r = r.view(*lead, 1) * self.cfg.algo.intrinsic_reward_multiplier
        self._st["out"]["Rewards/intrinsic"] = r.mean()
        return r

    def _phase_expl_actor(self, data) -> None:
        st = self._st
        st["out"]["Grads/ensemble"] = self._clip(self.ensembles, self.ensemble_optimizer,
                                                 self.cfg.algo.ensembles.clip_gradients)
        self.ensemble_optimizer.step()
        if self.flavor == "dv2":
            mix = 0.0 if self.is_continuous else 1.0
            self._behaviour(data, self.actor_expl, self.target_critic_expl, self.actor_expl_optimizer,
                            self.actor_expl_params, mix, "_exploration", reward_fn=self._intrinsic_reward)
            vals = st["target_values_exploration"]
        else:
            self._behaviour(self.actor_expl, self.critic_expl, self.actor_expl_optimizer, self.actor_expl_params,
                            "_exploration", reward_fn=self._intrinsic_reward)
            vals = st["values_exploration"]
        st["out"]["Values_exploration/predicted_values"] = vals.mean()
        st["out"]["Values_exploration/lambda_values"] = st["lambda_values_exploration"].mean()

    def _phase_expl_critic(self, data) -> None:
        st = self._st
        st["out"]["Grads/actor_exploration"] = self._clip(self.actor_expl, self.actor_expl_optimizer,
                                                          self.cfg.algo.actor.clip_gradients)
        self.actor_expl_optimizer.step()
        self.critic_expl_optimizer.zero_grad()
        st["out"]["Loss/value_loss_exploration"] = self._critic_loss(self.critic_expl, self.critic_expl_params,
                                                                     "_exploration")

    # ------------------------------------------------------------------ task
    def _task_behaviour(self, data) -> None:
        if self.flavor == "dv2":
            mix = 0.0 if self.is_continuous else 1.0
            self._behaviour(data, self.actor, self.target_critic, self.actor_optimizer, self.actor_params, mix, "_task")
        else:
            self._behaviour(self.actor, self.critic, self.actor_optimizer, self.actor_params, "_task")

    def _phase_task_actor(self, data) -> None:
        st = self._st
        st["out"]["Grads/critic_exploration"] = self._clip(self.critic_expl, self.critic_expl_optimizer,
                                                           self.cfg.algo.critic.clip_gradients)
        self.critic_expl_optimizer.step()
        self._task_behaviour(data)

    def _phase_task_actor_wm(self, data) -> None:
        self._wm_step()
        self._task_behaviour(data)

    def _phase_critic_task(self, data) -> None:
        st = self._st
        st["out"]["Grads/actor_task"] = self._clip(self.actor, self.actor_optimizer, self.cfg.algo.actor.clip_gradients)
        self.actor_optimizer.step()
        self.critic_optimizer.zero_grad()
        st["out"]["Loss/value_loss_task"] = self._critic_loss(self.critic, self.critic_params, "_task")

    def _phase_final_task(self, data) -> Dict[str, Tensor]:
        st = self._st
        st["out"]["Grads/critic_task"] = self._clip(self.critic, self.critic_optimizer,
                                                    self.cfg.algo.critic.clip_gradients)
        self.critic_optimizer.step()
        out = dict(st["out"])
        # reference metric names
        for a, b in (("State/post_entropy", "State/p_entropy"), ("State/prior_entropy", "State/q_entropy")):
            if a in out:
                out[b] = out.pop(a)
        return out
