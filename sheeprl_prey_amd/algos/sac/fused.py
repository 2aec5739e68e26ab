"""The fused SAC gradient step (``ops/csrc/sac_fused.hip``): one SAC ``train`` call (reference
``sheeprl/algos/sac/sac.py:34-78``) as seven kernel launches, every parameter gradient written straight into
the flat optimiser slabs and both Adam updates (+ the step advance, + the target EMA) as one launch per phase:

    critic phase : Bellman target with in-kernel next actions | critic fwd + dq | critic dW (+ loss sum)
                   | [gradient all-reduce] | critic Adam + target EMA
    actor phase  : actor fwd + sample + every critic's Q and dQ/da + policy backward | actor dW + alpha grad
                   + losses + metric sums | [gradient all-reduce] | actor Adam + alpha Adam

The reparameterisation noise is Philox-4x32-10 keyed by a seed drawn from the (seeded) torch generator and
two device counters (update stream, player stream) that the kernels advance themselves, so every launch is
graph-capturable with no per-step host arguments.  The losses land in device scalars and a float64 metric
accumulator that ``MeanMetric.attach`` reads at log time (no per-step copy kernels).

``SACFusedUpdate.supported`` gates it: the SAC actor (2 ReLU layers, mean / log-std heads, clamped log-std),
an ``EnsembleMLP`` critic without dropout / LayerNorm (SAC, not DroQ), flat Adam optimisers, a GPU with the
native extension.  Anything else keeps the autograd path of ``SACTrainer``.
"""
from __future__ import annotations

import os
from typing import Dict, List

import torch
from torch import Tensor, nn

from sheeprl_prey_amd import ops
from sheeprl_prey_amd.algos.sac.agent import LOG_STD_MAX, LOG_STD_MIN, SACActor, SACCriticEnsemble

_LDS_MAX = 160 * 1024


def _pad16(v: int) -> int:
    return (v + 15) // 16 * 16


def _lds_ok(OD: int, A: int, H: int, Hc: int) -> bool:
    """Mirror of ``upd_lds`` / ``tgt_lds`` (the largest of the fused kernels' LDS footprints)."""
    actor = 2 * 16 * (H + 4) + 16 * (_pad16(2 * A) + 4) + 4 * 16 * A + 16
    upd = 16 * (_pad16(OD + A) + 4) + actor + 2 * 16 * (Hc + 4) + 8 * 16 + 3 * 16
    return 4 * upd <= _LDS_MAX


class SACFusedUpdate:
    @staticmethod
    def supported(agent, optimizers) -> bool:
        # SRL_SAC_FUSED=0: the autograd update; =critic: only the round-4 twin-Q critic kernels (A/B switches)
        if os.environ.get("SRL_SAC_FUSED", "1") in ("0", "critic") or not ops.native_available():
            return False
        if not agent.log_alpha.is_cuda:
            return False
        a = agent.actor
        if not isinstance(a, SACActor) or a.log_std_mode != 0:
            return False
        m = getattr(a.model, "model", None)
        if not (isinstance(m, nn.Sequential) and len(m) == 4 and isinstance(m[0], nn.Linear) and isinstance(m[2], nn.Linear)
                and type(m[1]) is nn.ReLU and type(m[3]) is nn.ReLU and m[0].bias is not None and m[2].bias is not None):
            return False
        H, OD, A = m[0].out_features, m[0].in_features, a.fc_mean.out_features
        if not (H % 128 == 0 and H <= 512 and m[2].in_features == H and m[2].out_features == H and OD <= 1024
                and a.fc_mean.in_features == H and a.fc_logstd.in_features == H and a.fc_logstd.out_features == A
                and 1 <= A <= 32 and a.fc_mean.bias is not None and a.fc_logstd.bias is not None):
            return False
        c = agent.critic
        if not isinstance(c, SACCriticEnsemble):
            return False
        ens = c.model
        if ens.norms is not None or ens.dropout > 0 or ens.act_name != "relu" or len(ens.layers) != 2 or ens.head is None:
            return False
        Hc = ens.layers[0].out_features
        if not (ens.head.out_features == 1 and 1 <= ens.n <= 8 and Hc % 128 == 0 and Hc <= 512
                and ens.layers[1].out_features == Hc and ens.layers[0].in_features == OD + A
                and ens.layers[0].bias is not None and ens.layers[1].bias is not None):
            return False
        if not _lds_ok(OD, A, H, Hc):
            return False
        from sheeprl_prey_amd.parallel.flat_optim import FlatAdam

        return all(isinstance(o, FlatAdam) and o.flat_param.is_cuda for o in optimizers)

    def __init__(self, agent, actor_optimizer, qf_optimizer, alpha_optimizer, gamma: float, reduce_min: bool = True):
        self.agent, self.gamma, self.reduce_min = agent, float(gamma), bool(reduce_min)
        self.actor_opt, self.qf_opt, self.alpha_opt = actor_optimizer, qf_optimizer, alpha_optimizer
        a = agent.actor
        m = a.model.model
        self.actor_w = [m[0].weight, m[0].bias, m[2].weight, m[2].bias, a.fc_mean.weight, a.fc_mean.bias,
                        a.fc_logstd.weight, a.fc_logstd.bias, a.action_scale, a.action_bias]
        ens, tgt = agent.critic.model, agent.critic_target.model
        self.critic_w = [ens.layers[0].weight, ens.layers[0].bias, ens.layers[1].weight, ens.layers[1].bias,
                         ens.head.weight, ens.head.bias]
        self.target_w = [tgt.layers[0].weight, tgt.layers[0].bias, tgt.layers[1].weight, tgt.layers[1].bias,
                         tgt.head.weight, tgt.head.bias]
        self.OD, self.H, self.A = m[0].in_features, m[0].out_features, a.fc_mean.out_features
        self.n, self.IN = ens.n, self.OD + self.A
        self.lo, self.hi = float(LOG_STD_MIN), float(LOG_STD_MAX)
        dev = agent.log_alpha.device
        self.device = dev
        self.ctr = torch.zeros(2, dtype=torch.int64, device=dev)  # [0] update draws, [1] player draws
        self.ticket = torch.zeros(1, dtype=torch.int32, device=dev)
        self.tickets = torch.zeros(8, dtype=torch.int32, device=dev)  # adam_multi: [0:4] critic phase, [4:8] actor
        self.seed = int(torch.randint(1, 2**62, (1,)).item())
        self.acc = torch.zeros(3, 2, dtype=torch.float64, device=dev)  # (sum, count): value, policy, alpha loss
        self.qf_loss = torch.zeros(1, device=dev)
        self.losses = torch.zeros(2, device=dev)
        self.one = torch.ones(1, device=dev)
        self.critic_grads = qf_optimizer.grad_views(self.critic_w)
        self.actor_grads = actor_optimizer.grad_views(self.actor_w[:8]) + alpha_optimizer.grad_views([agent.log_alpha])
        self._ws: Dict[int, Dict[str, object]] = {}
        self._act_out: Dict[int, Tensor] = {}
        self._attached = None

    # ------------------------------------------------------------------ workspaces (one set per batch size)
    def _wsp(self, M: int):
        w = self._ws.get(M)
        if w is None:
            C = ops._ext()
            dev, H, n, A = self.device, self.H, self.n, self.A
            ZP, nb = C.sac_fused_zp(A), C.sac_fused_blocks(M)
            e = lambda *s: torch.empty(*s, device=dev)  # noqa: E731
            w = {"y": e(M),
                 "ws": [e(M, _pad16(self.OD)), e(M, H), e(M, H), e(M, ZP), e(M, H), e(M, H), e(n, M), e(n, M, A), e(nb, 2)],
                 "cnt": torch.zeros(nb, dtype=torch.int32, device=dev)}
            self._ws[M] = w
        return w

    @staticmethod
    def _hyper(opt) -> List[float]:
        g = opt.param_groups[0]
        b1, b2 = g["betas"]
        return [float(g["lr"]), float(b1), float(b2), float(g["eps"]), float(g["weight_decay"]),
                1.0 if getattr(opt, "decoupled", False) else 0.0]

    @staticmethod
    def _slab(opt) -> List[Tensor]:
        return [opt.flat_param, opt.flat_grad, opt.exp_avg, opt.exp_avg_sq, opt.scalars]

    # ------------------------------------------------------------------ critic phase
    def critic(self, d: Dict[str, Tensor]) -> Tensor:
        """Target, critic forward / backward: the critic gradient in the slab, the loss in ``self.qf_loss``."""
        C = ops._ext()
        obs = d["observations"].contiguous()
        M = obs.shape[0]
        w = self._wsp(M)
        self.qf_opt.grad_views([])  # keep every .grad linked to the slab the kernels write
        C.sac_fused_target(d["next_observations"].contiguous(), d["rewards"].reshape(-1).float().contiguous(),
                           d["dones"].reshape(-1).float().contiguous(), self.agent.log_alpha.detach(), self.actor_w,
                           self.lo, self.hi, self.target_w, self.ctr, self.seed, self.gamma, w["y"], None, None, None)
        lossp, _q, *saved = C.sac_critic_fwd(obs, d["actions"].contiguous(), w["y"], *self.critic_w)
        C.sac_fused_critic_wgrad(saved, self.one, self.IN, self.critic_grads, lossp, self.qf_loss)
        return self.qf_loss

    def critic_apply(self, ema_w: Tensor) -> None:
        target = self.agent._target_flat
        slab = self._slab(self.qf_opt) + ([target, ema_w.reshape(1)] if target is not None else [])
        ops._ext().sac_adam_multi([slab], [self._hyper(self.qf_opt)], ops.fault_block(self.device), self.tickets[:4])
        if target is None:  # no flat target layout: the per-tensor EMA
            self.agent.qfs_target_ema(ema_w)

    # ------------------------------------------------------------------ actor phase
    def actor(self, obs: Tensor) -> Tensor:
        """Actor + alpha objective forward / backward: gradients in the slabs, [policy loss, alpha loss]."""
        obs = obs.contiguous()
        w = self._wsp(obs.shape[0])
        self.actor_opt.grad_views([])
        self.alpha_opt.grad_views([])
        a = self.agent
        ops._ext().sac_fused_actor(obs, a.log_alpha.detach(), a.target_entropy.reshape(1).float(), self.actor_w, self.lo,
                                   self.hi, self.critic_w, self.ctr, self.seed, self.reduce_min, w["ws"], w["cnt"],
                                   self.actor_grads, self.qf_loss, self.losses, self.acc, None, None, None, None)
        return self.losses

    def actor_apply(self) -> None:
        ops._ext().sac_adam_multi([self._slab(self.actor_opt), self._slab(self.alpha_opt)],
                                  [self._hyper(self.actor_opt), self._hyper(self.alpha_opt)],
                                  ops.fault_block(self.device), self.tickets[4:])

    # ------------------------------------------------------------------ player
    def act(self, obs: Tensor) -> Tensor:
        """Sampled actions for the observation rows (one launch; the player stream's counter advances)."""
        obs = obs.contiguous()
        M = obs.shape[0]
        out = self._act_out.get(M)
        if out is None:
            out = self._act_out[M] = torch.empty(M, self.A, device=self.device)
        ops._ext().sac_fused_act(obs, self.actor_w, self.lo, self.hi, self.ctr[1:], self.ticket, self.seed, out, None,
                                 None)
        return out

    # ------------------------------------------------------------------ metrics
    KEYS = ("Loss/value_loss", "Loss/policy_loss", "Loss/alpha_loss")

    def attach(self, aggregator) -> None:
        """Route the three loss metrics of ``aggregator`` to the kernels' device accumulator."""
        if aggregator is None or aggregator is self._attached:
            return
        for i, k in enumerate(self.KEYS):
            if k in aggregator:
                aggregator.metrics[k].attach(self.acc[i])
        self._attached = aggregator
