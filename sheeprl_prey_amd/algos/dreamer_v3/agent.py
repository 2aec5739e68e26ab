"""DreamerV3 agent (reference: ``sheeprl/algos/dreamer_v3/agent.py:28-1068``).

Module structure and ``state_dict`` keys follow the reference (so checkpoints line up), but the
hot paths are re-shaped for MI355X:

* every ``Linear -> LayerNorm -> SiLU`` runs LN+SiLU as one fused HIP kernel, and the channel
  LayerNorm of the conv stacks runs directly on NCHW (no permute copies);
* the GRU epilogue (LN over 3H + gates) is one fused kernel;
* unimix + straight-through one-hot sampling is one fused kernel per categorical block;
* ``RSSM.scan_dynamic`` runs the T-step posterior scan with the step-invariant GEMM work hoisted
  out of the loop: the embedding half of the representation layer ([T*B, 4096] x [4096, 512]) and
  the action half of the recurrent input layer are computed for all T in one large GEMM each, so
  the sequential loop only carries the h/z-dependent small-M GEMMs.
"""
from __future__ import annotations

import os

import copy
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F
from torch import Tensor, nn
from torch.distributions import Distribution, Independent, Normal, TanhTransform, TransformedDistribution

from sheeprl_prey_amd import ops
from sheeprl_prey_amd.ops import conv as conv_ops
from sheeprl_prey_amd.config.instantiate import get_class
from sheeprl_prey_amd.models.models import CNN, MLP, DeCNN, LayerNormGRUCell, Linear, MultiDecoder, MultiEncoder
from sheeprl_prey_amd.models.world_model import WorldModel
from sheeprl_prey_amd.utils.distribution import (
    OneHotCategoricalStraightThroughValidateArgs,
    OneHotCategoricalValidateArgs,
    TruncatedNormal,
)
from sheeprl_prey_amd.utils.model import LayerNormChannelLast, ModuleType, cnn_forward


def _act(name):
    return get_class(name) if isinstance(name, str) else name


# ------------------------------------------------------------------ Hafner initialisation
def init_weights(m: nn.Module) -> None:
    """Truncated-normal fan-avg init (reference ``dreamer_v3/utils.py:162-187``)."""
    if isinstance(m, nn.Linear):
        denoms = (m.in_features + m.out_features) / 2.0
        std = np.sqrt(1.0 / denoms) / 0.87962566103423978
        nn.init.trunc_normal_(m.weight.data, mean=0.0, std=std, a=-2.0 * std, b=2.0 * std)
        if m.bias is not None:
            m.bias.data.fill_(0.0)
    elif isinstance(m, (nn.Conv2d, nn.ConvTranspose2d)):
        space = m.kernel_size[0] * m.kernel_size[1]
        denoms = (space * m.in_channels + space * m.out_channels) / 2.0
        std = np.sqrt(1.0 / denoms) / 0.87962566103423978
        nn.init.trunc_normal_(m.weight.data, mean=0.0, std=std, a=-2.0, b=2.0)
        if m.bias is not None:
            m.bias.data.fill_(0.0)
    elif isinstance(m, nn.LayerNorm):
        if m.weight is not None:
            m.weight.data.fill_(1.0)
        if m.bias is not None:
            m.bias.data.fill_(0.0)


def uniform_init_weights(given_scale: float):
    """Uniform init of output heads (reference ``dreamer_v3/utils.py:190-207``)."""

    def f(m: nn.Module) -> None:
        if isinstance(m, nn.Linear):
            denoms = (m.in_features + m.out_features) / 2.0
            limit = np.sqrt(3 * given_scale / denoms)
            nn.init.uniform_(m.weight.data, a=-limit, b=limit)
            if m.bias is not None:
                m.bias.data.fill_(0.0)
        elif isinstance(m, nn.LayerNorm):
            if m.weight is not None:
                m.weight.data.fill_(1.0)
            if m.bias is not None:
                m.bias.data.fill_(0.0)

    return f


# ------------------------------------------------------------------ encoders / decoders
class CNNEncoder(nn.Module):
    """``stages`` x (Conv k4 s2 p1 -> channel LN(eps 1e-3) -> SiLU), channels [1,2,4,8]*mult."""

    def __init__(self, keys: Sequence[str], input_channels: Sequence[int], image_size: Tuple[int, int],
                 channels_multiplier: int, layer_norm: bool = True, activation: ModuleType = nn.SiLU, stages: int = 4) -> None:
        super().__init__()
        self.keys = keys
        self.input_dim = (sum(input_channels), *image_size)
        self.model = nn.Sequential(
            CNN(
                input_channels=self.input_dim[0],
                hidden_channels=[(2**i) * channels_multiplier for i in range(stages)],
                cnn_layer=nn.Conv2d,
                layer_args={"kernel_size": 4, "stride": 2, "padding": 1, "bias": not layer_norm},
                activation=activation,
                norm_layer=[LayerNormChannelLast for _ in range(stages)] if layer_norm else None,
                norm_args=[{"normalized_shape": (2**i) * channels_multiplier, "eps": 1e-3} for i in range(stages)]
                if layer_norm else None,
            ),
            nn.Flatten(-3, -1),
        )
        with torch.no_grad():
            self.output_dim = self.model(torch.zeros(1, *self.input_dim)).shape[-1]

    def forward(self, obs: Dict[str, Tensor]) -> Tensor:
        """``obs``: the scaled float frames (reference form), or the raw uint8 frames, which are
        scaled by 1/255 here (on the fused path inside the NHWC conversion: no float copy of the batch)."""
        # one key: no concatenation copy (torch.cat of a single tensor still copies it)
        x = obs[self.keys[0]] if len(self.keys) == 1 else torch.cat([obs[k] for k in self.keys], -3)
        raw = x.dtype == torch.uint8
        if x.is_cuda and (raw or x.dtype == torch.float32) and ops.fused_enabled() and conv_ops.ENABLED:
            if not hasattr(self, "_fused_spec"):
                self._fused_spec = conv_ops.encoder_spec(self.model, tuple(self.input_dim[1:]), self.input_dim[0])
            flat = x.reshape(-1, *x.shape[-3:])
            if self._fused_spec is not None and flat.shape[0] >= conv_ops.MIN_FRAMES:
                # whole stack as one implicit-GEMM autograd op (ops/conv.py): NHWC, LN+SiLU fused
                out = conv_ops.encoder_forward(self._fused_spec, flat, 1.0 / 255.0 if raw else 1.0)
                return out.reshape(*x.shape[:-3], -1)
            if self._fused_spec is not None and conv_ops.SMALL_ENABLED and not torch.is_grad_enabled():
                # the player's few frames: split-K small-batch stack (csrc/conv_small.hip)
                out = conv_ops.encoder_small(self._fused_spec, flat, 1.0 / 255.0 if raw else 1.0)
                return out.reshape(*x.shape[:-3], -1)
        if raw:
            x = x / 255.0
        return cnn_forward(self.model, x, x.shape[-3:], (-1,))


class MLPEncoder(nn.Module):
    def __init__(self, keys: Sequence[str], input_dims: Sequence[int], mlp_layers: int = 4, dense_units: int = 512,
                 layer_norm: bool = True, activation: ModuleType = nn.SiLU, symlog_inputs: bool = True) -> None:
        super().__init__()
        self.keys = keys
        self.input_dim = sum(input_dims)
        self.model = MLP(
            self.input_dim, None, [dense_units] * mlp_layers, activation=activation, layer_args={"bias": not layer_norm},
            norm_layer=[nn.LayerNorm for _ in range(mlp_layers)] if layer_norm else None,
            norm_args=[{"normalized_shape": dense_units, "eps": 1e-3} for _ in range(mlp_layers)] if layer_norm else None,
        )
        self.output_dim = dense_units
        self.symlog_inputs = symlog_inputs

    def forward(self, obs: Dict[str, Tensor]) -> Tensor:
        if self.symlog_inputs:
            x = ops.symlog_cat([obs[k] for k in self.keys])  # one launch on GPU (sign / abs / log1p / mul + cat in torch)
        else:
            x = torch.cat([obs[k] for k in self.keys], -1)
        return self.model(x)


class CNNDecoder(nn.Module):
    """Linear(latent -> 8*mult*4*4) -> (stages-1) x (ConvT k4 s2 p1 -> LN -> SiLU) -> ConvT -> +0.5."""

    def __init__(self, keys: Sequence[str], output_channels: Sequence[int], channels_multiplier: int,
                 latent_state_size: int, cnn_encoder_output_dim: int, image_size: Tuple[int, int],
                 activation: ModuleType = nn.SiLU, layer_norm: bool = True, stages: int = 4) -> None:
        super().__init__()
        self.keys = keys
        self.output_channels = output_channels
        self.cnn_encoder_output_dim = cnn_encoder_output_dim
        self.image_size = image_size
        self.output_dim = (sum(output_channels), *image_size)
        self.model = nn.Sequential(
            Linear(latent_state_size, cnn_encoder_output_dim),
            nn.Unflatten(1, (-1, 4, 4)),
            DeCNN(
                input_channels=(2 ** (stages - 1)) * channels_multiplier,
                hidden_channels=[(2**i) * channels_multiplier for i in reversed(range(stages - 1))] + [self.output_dim[0]],
                cnn_layer=nn.ConvTranspose2d,
                layer_args=[{"kernel_size": 4, "stride": 2, "padding": 1, "bias": not layer_norm} for _ in range(stages - 1)]
                + [{"kernel_size": 4, "stride": 2, "padding": 1}],
                activation=[activation for _ in range(stages - 1)] + [None],
                norm_layer=([LayerNormChannelLast for _ in range(stages - 1)] + [None]) if layer_norm else None,
                norm_args=([{"normalized_shape": (2 ** (stages - i - 2)) * channels_multiplier, "eps": 1e-3}
                            for i in range(stages - 1)] + [None]) if layer_norm else None,
            ),
        )

    def forward(self, latent_states: Tensor, onehot=None) -> Dict[str, Tensor]:
        out = None
        if latent_states.is_cuda and latent_states.dtype == torch.float32 and ops.fused_enabled() and conv_ops.ENABLED:
            if not hasattr(self, "_fused_spec"):
                self._fused_spec = conv_ops.decoder_spec(self.model, self.output_dim[0])
            x = latent_states.reshape(-1, latent_states.shape[-1])
            if self._fused_spec is not None and x.shape[0] >= conv_ops.MIN_FRAMES:
                lin, stages = self._fused_spec
                from sheeprl_prey_amd.ops import onehot as oh

                if onehot is not None and oh.layer_supported(lin, onehot[3]):
                    # the posterior columns of the Linear gathered from its transposed weight (ops/onehot.py)
                    idx, G, off, n1 = onehot
                    h = oh.first_layer(x, idx.reshape(-1, idx.shape[-1]), G, off, lin, None, n1)
                else:
                    h = lin(x)
                out = conv_ops.decoder_forward(stages, h, 0.5)
                out = out.reshape(*latent_states.shape[:-1], *self.output_dim)
        if out is None:
            out = cnn_forward(self.model, latent_states, (latent_states.shape[-1],), self.output_dim) + 0.5
        return {k: o for k, o in zip(self.keys, torch.split(out, self.output_channels, -3))}


class MLPDecoder(nn.Module):
    def __init__(self, keys: Sequence[str], output_dims: Sequence[int], latent_state_size: int, mlp_layers: int = 4,
                 dense_units: int = 512, activation: ModuleType = nn.SiLU, layer_norm: bool = True) -> None:
        super().__init__()
        self.output_dims = output_dims
        self.keys = keys
        self.model = MLP(
            latent_state_size, None, [dense_units] * mlp_layers, activation=activation, layer_args={"bias": not layer_norm},
            norm_layer=[nn.LayerNorm for _ in range(mlp_layers)] if layer_norm else None,
            norm_args=[{"normalized_shape": dense_units, "eps": 1e-3} for _ in range(mlp_layers)] if layer_norm else None,
        )
        self.heads = nn.ModuleList([Linear(dense_units, d) for d in self.output_dims])

    def forward(self, latent_states: Tensor, onehot=None) -> Dict[str, Tensor]:
        x = None
        if onehot is not None:
            from sheeprl_prey_amd.ops.onehot import mlp_forward

            x = mlp_forward(self.model, latent_states, *onehot)
        if x is None:
            x = self.model(latent_states)
        return {k: h(x) for k, h in zip(self.keys, self.heads)}


# ------------------------------------------------------------------ recurrent model / RSSM
class RecurrentModel(nn.Module):
    """Linear(no bias) -> LN(1e-3) -> SiLU -> LayerNormGRUCell (reference ``agent.py:260-309``)."""

    def __init__(self, input_size: int, recurrent_state_size: int, dense_units: int, activation_fn: ModuleType = nn.SiLU,
                 layer_norm: bool = True) -> None:
        super().__init__()
        self.mlp = MLP(
            input_dims=input_size, output_dim=None, hidden_sizes=[dense_units], activation=activation_fn,
            layer_args={"bias": not layer_norm},
            norm_layer=[nn.LayerNorm] if layer_norm else None,
            norm_args=[{"normalized_shape": dense_units, "eps": 1e-3}] if layer_norm else None,
        )
        self.rnn = LayerNormGRUCell(dense_units, recurrent_state_size, bias=False, batch_first=False, layer_norm=True)

    def forward(self, input: Tensor, recurrent_state: Tensor) -> Tensor:
        return self.rnn(self.mlp(input), recurrent_state)


def _lin(mlp: MLP, i: int) -> nn.Linear:
    return mlp.model[i]


class RSSM(nn.Module):
    """Discrete RSSM with unimix categoricals (reference ``agent.py:312-455``)."""

    def __init__(self, recurrent_model: nn.Module, representation_model: nn.Module, transition_model: nn.Module,
                 distribution_cfg: Dict[str, Any], discrete: int = 32, unimix: float = 0.01) -> None:
        super().__init__()
        self.recurrent_model = recurrent_model
        self.representation_model = representation_model
        self.transition_model = transition_model
        self.discrete = discrete
        self.unimix = unimix
        self.distribution_cfg = distribution_cfg

    # ---- reference-semantics single steps (player / tests) ----------------------------
    def dynamic(self, posterior: Tensor, recurrent_state: Tensor, action: Tensor, embedded_obs: Tensor, is_first: Tensor):
        action = (1 - is_first) * action
        recurrent_state = (1 - is_first) * recurrent_state + is_first * torch.tanh(torch.zeros_like(recurrent_state))
        posterior = posterior.view(*posterior.shape[:-2], -1)
        posterior = (1 - is_first) * posterior + is_first * self._transition(recurrent_state, sample_state=False)[1].view_as(posterior)
        recurrent_state = self.recurrent_model(torch.cat((posterior, action), -1), recurrent_state)
        prior_logits, prior = self._transition(recurrent_state)
        posterior_logits, posterior = self._representation(recurrent_state, embedded_obs)
        return recurrent_state, posterior, prior, posterior_logits, prior_logits

    def _uniform_mix(self, logits: Tensor) -> Tensor:
        return ops.reference.unimix_logits(logits, self.discrete, self.unimix)

    def _sample(self, logits: Tensor, sample: bool = True, forced: Optional[Tensor] = None) -> Tuple[Tensor, Tensor]:
        mixed, st = ops.unimix_sample(logits, self.discrete, self.unimix, sample=sample, forced=forced)
        return mixed, st.view(*st.shape[:-1], -1, self.discrete)

    def _representation(self, recurrent_state: Tensor, embedded_obs: Tensor) -> Tuple[Tensor, Tensor]:
        return self._sample(self.representation_model(torch.cat((recurrent_state, embedded_obs), -1)))

    def _transition(self, recurrent_out: Tensor, sample_state: bool = True,
                    forced: Optional[Tensor] = None) -> Tuple[Tensor, Tensor]:
        return self._sample(self.transition_model(recurrent_out), sample=sample_state, forced=forced)

    def imagination(self, prior: Tensor, recurrent_state: Tensor, actions: Tensor,
                    forced: Optional[Tensor] = None) -> Tuple[Tensor, Tensor]:
        """``forced``: the prior sample to take (one-hot, teacher forcing of the eager oracle)."""
        recurrent_state = self.recurrent_model(torch.cat((prior, actions), -1), recurrent_state)
        _, imagined_prior = self._transition(recurrent_state, forced=forced)
        return imagined_prior, recurrent_state

    # ---- MI355X imagination: buffer-resident no-grad rollout ---------------------------
    _actor_tail_ok = True  # the fused rollout actor tail (tests toggle it)
    # merged h_{t+1} GEMM of the imagination step (every GEMM over h_{t+1} as one, 505 -> 463 dispatches per Atari
    # step).  Untuned it was slower (313.0 / 313.5 vs 323.3 env-steps/s; profiles/r4_imag_merge.md); with its shapes
    # in the committed TunableOp results it is equal (323.0 vs 323.2 mean of three interleaved 150-step runs,
    # profiles/r4_merge_ab.md), so the rollouts use it by default for recurrent states up to 1024 wide; the continuous
    # rollout (imagine_cont.py) measured 123.6 / 123.7 vs 123.3 / 123.6 env-steps/s with / without.  For the XL state
    # (deter 4096) the unmerged K = Hd + D GRU projection is a ~150 TF/s library GEMM and splitting it costs more
    # than the launches saved (47.8 / 47.6 vs 48.2 / 48.3 env-steps/s, merged shapes tuned).  Tests force it with
    # True / False.
    _merge_h_ok = "auto"
    _merge_h_cont_ok = "auto"
    MERGE_MAX_H = 1024

    @staticmethod
    def merge_enabled(flag, Hd: int) -> bool:
        """The merge policy: "1" / True on, "0" / False off, "auto" (default) for recurrent states <= MERGE_MAX_H."""
        if flag is True or flag is False:
            return flag
        return flag == "1" or (flag == "auto" and Hd <= RSSM.MERGE_MAX_H)
    # one-launch prior head (prior_head.hip; used on the merged path): 30.6 us vs ~28 us for LayerNorm + GEMM + sampler
    _prior_head_ok = True

    def imagine_fast_ok(self, actor) -> bool:
        gru = self.recurrent_model.rnn
        rec = list(self.recurrent_model.mlp.model)
        return (isinstance(gru.layer_norm, nn.LayerNorm) and isinstance(rec[0], nn.Linear)
                and not getattr(self, "_srl_autocast", False) and not getattr(actor, "_srl_autocast", False)
                and type(actor) is Actor and not actor.is_continuous and ops.native_available() and ops.fused_enabled()
                and gru.layer_norm.weight is not None and gru.layer_norm.bias is not None)

    @torch.no_grad()
    def imagine_discrete(self, post: Tensor, h: Tensor, actor: "Actor", horizon: int, record: bool = False,
                         indices: bool = False, gather: bool = True):
        """Imagination rollout for discrete actors without autograd (reference loop: ``dreamer_v3.py:
        235-257`` over ``RSSM.imagination`` + ``Actor.forward``; the discrete objective back-propagates
        only through log-probs of detached actions, so no graph is needed).

        Every step writes straight into one buffer ``[H+1, M, Ap + S + Hd + D]`` holding (action | pad | prior |
        h | x), x = the recurrent MLP's output of the step: the sampling, LayerNorm and LN-GRU kernels
        store into row-strided slices of it, so the GRU input projection is ONE GEMM over (h | x)
        (K = Hd + D) and the trajectories ``[H+1, M, S + Hd]`` / actions ``[H+1, M, A]`` are views.

        One-hot gathers (``ops/onehot.py``): actions and priors are exact one-hots, so the samplers also
        emit their hot columns (``IDX [H+1, M, nh + G]``: action columns, then A + prior column) and
        the recurrent MLP's [action | prior] layer is a row gather of its transposed weight + LayerNorm
        + act in one kernel (no GEMM), the actor trunk's first layer a K = Hd GEMM + gather.

        ``record``: the actor trunk's activations of every step are kept (``ops.mlp_trunk``) and
        returned, the ``TrunkRecord`` the actor loss back-propagates through instead of running the
        actor forward over the trajectories a second time.  ``indices``: also return ``IDX``."""
        from sheeprl_prey_amd.ops import onehot as oh
        from sheeprl_prey_amd.ops.mlp_trunk import TrunkRecord, trunk_layers

        C = ops._ext()
        M, S = post.shape
        Hd = h.shape[1]
        A = int(sum(actor.actions_dim))
        disc = self.discrete
        nh, G = len(actor.actions_dim), S // disc
        dev = post.device
        # every uniform of the rollout in one launch: per step nh x M for the actions, G x M for the prior
        U = torch.rand(horizon + 1, M * (nh + G), device=dev)
        layers = trunk_layers(actor.model)
        trunk_rec = TrunkRecord(layers, horizon + 1, M, dev) if (record and layers is not None) else None
        rec_sp = oh.mlp_split(self.recurrent_model.mlp)
        rec_lin = list(self.recurrent_model.mlp.model)[0]
        rec_ln = rec_sp[1] if rec_sp is not None else None
        D = rec_lin.out_features
        use_gather = (gather and rec_sp is not None and rec_ln is not None and not rec_sp[2] and oh.layer_supported(rec_lin, A + S)
                      and rec_lin.bias is None and all(a <= 64 for a in actor.actions_dim))
        gru = self.recurrent_model.rnn
        Wg = gru.linear.weight  # columns: (h | feat)
        ln = gru.layer_norm
        # prior columns start at Ap >= A: with the gathered recurrent layer the buffer's (action | prior) block is
        # never read as a dense operand, so the actions are padded to put h (the dense part of every head's first
        # layer) on a 16-byte boundary with a row stride % 4 == 0 - the heads' weight-gradient kernels then stage
        # it with 16-byte loads (ops.wgrad)
        Ap = A + ((-(A + S)) % 4) if use_gather else A
        Wd = Ap + S + Hd + D
        Wd += (-Wd) % 4
        buf = post.new_empty(horizon + 1, M, Wd)
        buf[0, :, Ap:Ap + S].copy_(post)
        buf[0, :, Ap + S:Ap + S + Hd].copy_(h)
        IDX = torch.empty(horizon + 1, M, nh + G, dtype=torch.int32, device=dev)
        oh.onehot_index(post, disc, IDX[0, :, nh:], A)
        W = rec_lin.weight  # columns: (prior | action)
        # the actor trunk's first layer: prior columns gathered from its transposed weight, h by a GEMM
        a0 = layers[0][0] if layers is not None else None
        want_a = gather and layers is not None and oh.layer_supported(a0, S)
        rec_table = a_table = Wp = None
        if use_gather:
            # [A + S, D]: row = hot column of (action | prior); both tables transposed in one launch
            na = W.shape[1] - S
            rec_table = W.new_empty(W.shape[1], W.shape[0])
            srcs, outs = [W[:, S:], W[:, :S]], [rec_table[:na], rec_table[na:]]
            if want_a:
                srcs.append(a0.weight[:, :S])
                outs.append(None)
            with torch.no_grad():
                tabs = ops.transpose_many(srcs, outs)
            a_table = tabs[2] if want_a else None
        else:
            Wp = torch.cat((W[:, S:], W[:, :S]), 1)  # columns: (action | prior)
            if want_a:
                a_table = a0.weight[:, :S].t().contiguous()
        act_scratch = None
        if trunk_rec is not None and a_table is not None:
            trunk_rec.onehot = (IDX[:, :, nh:], G, A, S)  # the trunk backward scatters the prior columns' dW
        one_head = nh == 1 and self._actor_tail_ok
        # every GEMM reading h_{t+1} as ONE: the transition's first layer, the actor trunk's dense first-layer part
        # (used at step t+1) and the h half of step t+1's GRU input projection - [M, Hd] x [Hd, Ntr + Na + 3H]; the
        # GRU then multiplies only x_{t+1} (K = D) and the LN-GRU kernel adds the two parts
        tr_sp = oh.mlp_split(self.transition_model)
        merge = (self.merge_enabled(self._merge_h_ok, Hd) and use_gather and a_table is not None and layers is not None
                 and gru.linear.bias is None
                 and tr_sp is not None and tr_sp[1] is not None and len(tr_sp[2]) > 0)
        if merge:
            tr_lin, tr_ln, tr_rest = tr_sp
            Ntr, Na = tr_lin.out_features, a0.out_features
            Wm = torch.cat((tr_lin.weight, a0.weight[:, S:], Wg[:, :Hd]), 0)
            Wgx_t = Wg[:, Hd:].t()
            # the transition layer's bias rides in the GEMM epilogue (zero on the actor / GRU columns: the actor's bias
            # is added by the gather kernel, the GRU projection has none)
            bm = None
            if tr_lin.bias is not None:  # one concatenation with a cached zero tail (no fill + copy per step)
                nz = Wm.shape[0] - Ntr
                zt = getattr(self, "_bm_zeros", None)
                if zt is None or zt.numel() != nz or zt.device != dev:
                    zt = self._bm_zeros = torch.zeros(nz, device=dev, dtype=Wm.dtype)
                bm = torch.cat((tr_lin.bias.detach(), zt))
            hm = torch.addmm(bm, h, Wm.t()) if bm is not None else torch.mm(h, Wm.t())
            ytr, mtr, rtr = post.new_empty(M, Ntr), post.new_empty(M), post.new_empty(M)
            tr_act = ops._act_code(tr_ln.act)
            # LayerNorm + act + output Linear + unimix sample of the prior in one launch (prior_head.hip)
            phead = (self._prior_head_ok and disc == 32 and len(tr_rest) == 1 and isinstance(tr_rest[0], nn.Linear)
                     and S % 256 == 0 and Ntr % 16 == 0 and Ntr <= 1024)
        for t in range(horizon + 1):
            traj_t = buf[t, :, Ap:Ap + S + Hd]
            # single-head actors: last LayerNorm + head + unimix sample in one kernel (TrunkRecord.step tail)
            tail = ((actor.mlp_heads[0], U[t, :M], float(actor._unimix), buf[t, :, :A], IDX[t, :, :1], 0)
                    if one_head else None)
            ga = ((IDX[t, :, nh:], G, A, S, a_table) + ((hm[:, Ntr:Ntr + Na],) if merge else ())
                  if a_table is not None else None)
            if trunk_rec is not None:
                out = trunk_rec.step(t, traj_t, gather=ga, tail=tail)
            elif layers is not None and a_table is not None:
                if act_scratch is None:
                    act_scratch = TrunkRecord(layers, 1, M, dev)
                out = act_scratch.step(0, traj_t, gather=ga, tail=tail)
            else:
                out = actor.model(traj_t)
            c0 = 0
            for i, (head, a) in enumerate(zip(actor.mlp_heads, actor.actions_dim)):
                if out is None:
                    break  # sampled by the fused tail
                C.unimix_sample_into(head(out), U[t, i * M:(i + 1) * M], int(a), float(actor._unimix), buf[t, :, c0:c0 + a],
                                     IDX[t, :, i:i + 1], c0)
                c0 += a
            if t == horizon:
                break
            xs = buf[t, :, Ap + S + Hd:Ap + S + Hd + D]
            if use_gather:
                oh.gather_first_layer(buf[t, :, :A + S], IDX[t], nh + G, 0, rec_lin, rec_ln, A + S, table=rec_table,
                                      y_out=xs)
            else:
                x = torch.mm(buf[t, :, :A + S], Wp.t())
                if rec_lin.bias is not None:
                    x = x + rec_lin.bias
                for m in list(self.recurrent_model.mlp.model)[1:]:
                    x = m(x)
                xs.copy_(x)
            if merge:
                # x half of the GRU input projection; the h half is the last block of hm (h_t)
                gx = torch.mm(xs, Wgx_t)
                C.ln_gru_into(gx, buf[t, :, Ap + S:Ap + S + Hd], ln.weight, ln.bias, float(ln.eps),
                              buf[t + 1, :, Ap + S:Ap + S + Hd], x2=hm[:, Ntr + Na:])
                if bm is not None:
                    torch.addmm(bm, buf[t + 1, :, Ap + S:Ap + S + Hd], Wm.t(), out=hm)
                else:
                    torch.mm(buf[t + 1, :, Ap + S:Ap + S + Hd], Wm.t(), out=hm)
                if phead and C.prior_head(hm[:, :Ntr], tr_ln.weight, tr_ln.bias, float(tr_ln.eps), tr_act, tr_rest[0].weight,
                                          tr_rest[0].bias, U[t, nh * M:], float(self.unimix), buf[t + 1, :, Ap:Ap + S],
                                          IDX[t + 1, :, nh:], A):
                    continue
                C.ln_act_fwd_into(hm, hm.stride(0), ytr, Ntr, tr_ln.weight, tr_ln.bias, mtr, rtr, M, Ntr, 1,
                                  float(tr_ln.eps), tr_act)
                logits = ytr
                for m in tr_rest:
                    logits = m(logits)
            else:
                gx = torch.mm(buf[t, :, Ap + S:Ap + S + Hd + D], Wg.t())  # (h | x) in one GEMM
                if gru.linear.bias is not None:
                    gx = gx + gru.linear.bias
                C.ln_gru_into(gx, buf[t, :, Ap + S:Ap + S + Hd], ln.weight, ln.bias, float(ln.eps),
                              buf[t + 1, :, Ap + S:Ap + S + Hd])
                logits = self.transition_model(buf[t + 1, :, Ap + S:Ap + S + Hd])
            C.unimix_sample_into(logits.contiguous(), U[t, nh * M:], disc, float(self.unimix), buf[t + 1, :, Ap:Ap + S],
                                 IDX[t + 1, :, nh:], A)
        out = (buf[:, :, Ap:Ap + S + Hd], buf[:, :, :A])
        if record:
            out = out + (trunk_rec,)
        if indices:
            out = out + (IDX,)
        return out

    # ---- MI355X scan: T-step posterior rollout with hoisted GEMMs --------------------
    def _mlp_head(self, mlp: MLP, x_pre: Tensor) -> Tensor:
        """Finish an ``MLP(hidden=[h], out=o)`` whose first Linear output is ``x_pre``."""
        seq = mlp.model
        x = x_pre
        for m in list(seq)[1:]:
            x = m(x)
        return x

    def scan_dynamic(self, embedded_obs: Tensor, actions: Tensor, is_first: Tensor, uniform: Optional[Tensor] = None,
                     forced: Optional[Tensor] = None):
        """Posterior scan over ``T`` (reference loop: ``dreamer_v3.py:122-129``).

        embedded_obs [T, B, E], actions [T, B, A] (already shifted), is_first [T, B, 1].  ``forced`` [T, B, S]
        (one-hot): the posterior samples to take (teacher forcing; eager path only).
        Returns recurrent_states [T,B,H], posteriors [T,B,S,D], posteriors_logits [T,B,S*D],
        priors_logits [T,B,S*D]."""
        T, B = embedded_obs.shape[:2]
        if getattr(self, "_srl_autocast", False):
            # bf16-mixed: every sub-model through its own (autocast) forward, as the reference does
            return self._scan_by_steps(embedded_obs, actions, is_first, uniform)
        if ops._native(embedded_obs) and getattr(self, "fused_scan", True) and forced is None:
            from sheeprl_prey_amd.ops.rssm import fused_scan, fused_scan_supported

            if fused_scan_supported(self):
                H = self.recurrent_model.rnn.hidden_size
                h0 = torch.zeros(1, H, device=embedded_obs.device, dtype=embedded_obs.dtype)
                with torch.no_grad():
                    z0 = self._transition(h0, sample_state=False)[1].reshape(-1)
                hs, post, post_logits, prior_logits = fused_scan(self, embedded_obs, actions, is_first, z0, uniform)
                return hs, post.view(T, B, -1, self.discrete), post_logits, prior_logits
        rec_mlp = self.recurrent_model.mlp
        gru = self.recurrent_model.rnn
        rep, trans = self.representation_model, self.transition_model
        H = gru.hidden_size
        stoch = trans.model[-1].out_features
        rec_lin = _lin(rec_mlp, 0)
        Wz = rec_lin.weight[:, :stoch]
        Wa = rec_lin.weight[:, stoch:]
        rep_lin = _lin(rep, 0)
        Wh_rep = rep_lin.weight[:, :H]
        We_rep = rep_lin.weight[:, H:]
        # hoisted: action half of the recurrent input layer and embedding half of the representation layer
        act_masked = (1 - is_first) * actions
        a_proj = F.linear(act_masked, Wa)  # [T, B, dense]
        if rec_lin.bias is not None:
            a_proj = a_proj + rec_lin.bias
        e_proj = F.linear(embedded_obs, We_rep, rep_lin.bias)  # [T, B, hidden]
        # initial state: h0 = tanh(0) = 0, z0 = mode of the transition from h0
        h0 = torch.zeros(1, H, device=embedded_obs.device, dtype=embedded_obs.dtype)
        z0 = self._transition(h0, sample_state=False)[1].reshape(1, -1)
        h = torch.zeros(B, H, device=embedded_obs.device, dtype=embedded_obs.dtype)
        z = torch.zeros(B, stoch, device=embedded_obs.device, dtype=embedded_obs.dtype)
        if uniform is None:
            uniform = torch.rand(T, B, stoch // self.discrete, device=embedded_obs.device)
        hs, posts, post_logits, prior_logits = [], [], [], []
        for t in range(T):
            first = is_first[t]
            h = (1 - first) * h
            z = (1 - first) * z + first * z0
            x = torch.addmm(a_proj[t], z, Wz.t())
            feat = self._mlp_head(rec_mlp, x)
            h = gru.gates(gru.project(feat, h), h)
            pl = self._uniform_mix_fused(trans(h))
            rep_pre = torch.addmm(e_proj[t], h, Wh_rep.t())
            ql, zs = ops.unimix_sample(self._mlp_head(rep, rep_pre), self.discrete, self.unimix, sample=True,
                                       uniform=uniform[t], forced=forced[t] if forced is not None else None)
            z = zs
            hs.append(h)
            posts.append(zs)
            post_logits.append(ql)
            prior_logits.append(pl)
        recurrent_states = torch.stack(hs)
        posteriors = torch.stack(posts).view(T, B, -1, self.discrete)
        return recurrent_states, posteriors, torch.stack(post_logits), torch.stack(prior_logits)

    def _scan_by_steps(self, embedded_obs: Tensor, actions: Tensor, is_first: Tensor, uniform: Optional[Tensor] = None):
        """``dynamic`` step by step (reference loop ``dreamer_v3.py:122-129``): each sub-model is called
        through its forward, so set-up hooks (autocast) apply."""
        T, B = embedded_obs.shape[:2]
        H = self.recurrent_model.rnn.hidden_size
        S = self.transition_model.model[-1].out_features
        h = torch.zeros(B, H, device=embedded_obs.device)
        z = torch.zeros(B, S // self.discrete, self.discrete, device=embedded_obs.device)
        hs, posts, post_logits, prior_logits = [], [], [], []
        for t in range(T):
            h, z, _, ql, pl = self.dynamic(z, h, actions[t], embedded_obs[t], is_first[t])
            hs.append(h)
            posts.append(z)
            post_logits.append(ql)
            prior_logits.append(pl)
        return torch.stack(hs), torch.stack(posts), torch.stack(post_logits), torch.stack(prior_logits)

    def _uniform_mix_fused(self, logits: Tensor) -> Tensor:
        """Unimix logits only (no sampling) - the prior in the posterior scan is never sampled."""
        if ops._native(logits) and self.discrete <= 64:
            mixed, _ = ops.unimix_sample(logits, self.discrete, self.unimix, sample=False)
            return mixed
        return ops.reference.unimix_logits(logits, self.discrete, self.unimix)


# ------------------------------------------------------------------ actor
class Actor(nn.Module):
    """Actor MLP + heads (reference ``agent.py:602-747``): discrete -> unimix one-hot categorical
    with straight-through samples; continuous -> trunc_normal / normal / tanh_normal."""

    def __init__(self, latent_state_size: int, actions_dim: Sequence[int], is_continuous: bool,
                 distribution_cfg: Dict[str, Any], init_std: float = 0.0, min_std: float = 0.1, dense_units: int = 1024,
                 activation: ModuleType = nn.SiLU, mlp_layers: int = 5, layer_norm: bool = True, unimix: float = 0.01,
                 ln_eps: float = 1e-3, bias: Optional[bool] = None) -> None:
        super().__init__()
        self.distribution_cfg = distribution_cfg
        dist = str(distribution_cfg.get("type", "auto")).lower()
        if dist not in ("auto", "normal", "tanh_normal", "discrete", "trunc_normal"):
            raise ValueError(
                "The distribution must be on of: `auto`, `discrete`, `normal`, `tanh_normal` and `trunc_normal`. "
                f"Found: {dist}"
            )
        if dist == "discrete" and is_continuous:
            raise ValueError("You have choose a discrete distribution but `is_continuous` is true")
        if dist == "auto":
            dist = "trunc_normal" if is_continuous else "discrete"
        self.distribution = dist
        self.model = MLP(
            input_dims=latent_state_size, output_dim=None, hidden_sizes=[dense_units] * mlp_layers, activation=activation,
            flatten_dim=None, layer_args={"bias": (not layer_norm) if bias is None else bias},
            norm_layer=[nn.LayerNorm for _ in range(mlp_layers)] if layer_norm else None,
            norm_args=[{"normalized_shape": dense_units, "eps": ln_eps} for _ in range(mlp_layers)] if layer_norm else None,
        )
        if is_continuous:
            self.mlp_heads = nn.ModuleList([Linear(dense_units, int(np.sum(actions_dim)) * 2)])
        else:
            self.mlp_heads = nn.ModuleList([Linear(dense_units, a) for a in actions_dim])
        self.actions_dim = actions_dim
        self.is_continuous = is_continuous
        self.init_std = torch.tensor(init_std)
        self.min_std = min_std
        self._unimix = unimix

    def _continuous_dist(self, pre: Tensor) -> Distribution:
        va = self.distribution_cfg.get("validate_args", False)
        mean, std = torch.chunk(pre, 2, -1)
        if self.distribution == "tanh_normal":
            mean = 5 * torch.tanh(mean / 5)
            std = F.softplus(std + self.init_std) + self.min_std
            return Independent(TransformedDistribution(Normal(mean, std), TanhTransform(), validate_args=va), 1, validate_args=va)
        if self.distribution == "normal":
            return Independent(Normal(mean, std, validate_args=va), 1, validate_args=va)
        std = 2 * torch.sigmoid((std + self.init_std) / 2) + self.min_std
        # bounds as device tensors (fill kernels): python scalars would be H2D-copied, which a hipGraph
        # capture does not allow
        lo, hi = mean.new_full((), -1.0), mean.new_full((), 1.0)
        return Independent(TruncatedNormal(torch.tanh(mean), std, lo, hi, validate_args=va), 1, validate_args=va)

    def forward(self, state: Tensor, is_training: bool = True, mask: Optional[Dict[str, np.ndarray]] = None,
                forced: Optional[Sequence[Tensor]] = None):
        """``forced``: per discrete head, the one-hot action to take (teacher forcing of the eager oracle)."""
        out = self.model(state)
        pre_dist = [head(out) for head in self.mlp_heads]
        va = self.distribution_cfg.get("validate_args", False)
        if self.is_continuous:
            d = self._continuous_dist(pre_dist[0])
            if is_training:
                actions = d.rsample()
            else:
                sample = d.sample((100,))
                log_prob = d.log_prob(sample)
                actions = sample[log_prob.argmax(0)].view(1, 1, -1)
            return (actions,), (d,)
        actions, dists = [], []
        for i, logits in enumerate(pre_dist):
            C = logits.shape[-1]
            mixed, st = ops.unimix_sample(logits, C, self._unimix, sample=is_training,
                                          forced=forced[i] if forced is not None else None)
            dists.append(OneHotCategoricalStraightThroughValidateArgs(logits=mixed, validate_args=va))
            actions.append(st)
        return tuple(actions), tuple(dists)

    def sample_actions(self, state: Tensor, is_training: bool = True) -> Tuple[Tensor, ...]:
        """The actions of ``forward`` without building the distributions (discrete: their logits normalisation
        is ~10 kernels per env step the player never reads; truncated-normal: the last LayerNorm, the head Linear and
        the draw are ONE kernel instead of ~16 small ones)."""
        if self.is_continuous:
            fast = self._tn_sample(state) if is_training else None
            return (fast,) if fast is not None else self.forward(state, is_training)[0]
        fast = self._tail_sample(state) if is_training else None
        if fast is not None:
            return (fast,)
        out = self.model(state)
        return tuple(ops.unimix_sample(head(out), head.out_features, self._unimix, sample=is_training)[1]
                     for head in self.mlp_heads)

    def _uniform_mix(self, logits: Tensor) -> Tensor:
        return ops.reference.unimix_logits(logits, logits.shape[-1], self._unimix)

    @torch.no_grad()
    def _tail_sample(self, state: Tensor) -> Optional[Tensor]:
        """One-hot action draw of the player (one discrete head, no grad): the trunk up to its last pre-activation,
        then its LayerNorm + act, the head Linear and the unimix draw in one launch (``actor_tail.hip``, the
        imagination rollout's kernel); None when it does not apply."""
        from sheeprl_prey_amd.ops.mlp_trunk import trunk_layers

        if (len(self.mlp_heads) != 1 or not state.is_cuda or not ops.fused_enabled() or getattr(self, "_srl_autocast", False)
                or not RSSM._actor_tail_ok):
            return None
        layers = trunk_layers(self.model)
        if layers is None:
            return None
        x = state.reshape(-1, state.shape[-1])
        for lin, ln in layers[:-1]:
            x = ln(lin(x))
        lin, ln = layers[-1]
        z = lin(x)
        head = self.mlp_heads[0]
        M, N, A = z.shape[0], z.shape[1], head.out_features
        u = torch.rand(M, device=z.device)
        y, mean, rstd, out = z.new_empty(M, N), z.new_empty(M), z.new_empty(M), z.new_empty(M, A)
        if not ops._ext().actor_tail(z, y, ln.weight, ln.bias, mean, rstd, float(ln.eps), ops._act_code(ln.act), head.weight,
                                     head.bias, u, float(self._unimix), out, None, 0, None):
            return None
        return out.view(*state.shape[:-1], A)

    @torch.no_grad()
    def _tn_sample(self, state: Tensor) -> Optional[Tensor]:
        """Truncated-normal action draw of the player (no grad): the trunk up to its last pre-activation, then its
        LayerNorm + act, the head Linear and the inverse-CDF draw in one launch (``truncnorm.hip``
        head_linear_sample_fwd, the imagination rollout's kernel); None when it does not apply."""
        from sheeprl_prey_amd.ops.mlp_trunk import trunk_layers

        if (self.distribution != "trunc_normal" or len(self.mlp_heads) != 1 or not state.is_cuda
                or not ops.fused_enabled() or getattr(self, "_srl_autocast", False)):
            return None
        layers = trunk_layers(self.model)
        if layers is None:
            return None
        x = state.reshape(-1, state.shape[-1])
        for lin, ln in layers[:-1]:
            x = ln(lin(x))
        lin, ln = layers[-1]
        z = lin(x)
        head = self.mlp_heads[0]
        M, K, A = z.shape[0], z.shape[1], head.out_features // 2
        eps = float(torch.finfo(torch.float32).eps)
        u = torch.empty(M, A, device=z.device).uniform_(eps, 1.0 - eps)
        pre, loc, scale = z.new_empty(M, 2 * A), z.new_empty(M, A), z.new_empty(M, A)
        out, y, mean, rstd = z.new_empty(M, A), z.new_empty(M, K), z.new_empty(M), z.new_empty(M)
        if not ops._ext().tn_head_linear_sample_fwd(z, head.weight, head.bias, u, float(self.init_std), float(self.min_std),
                                                     -1.0, 1.0, pre, loc, scale, out, ln_w=ln.weight, ln_b=ln.bias,
                                                     ln_eps=float(ln.eps), act=ops._act_code(ln.act), y_out=y, mean=mean,
                                                     rstd=rstd):
            return None
        return out.view(*state.shape[:-1], A)


class MinedojoActor(Actor):
    """Actor with MineDojo action masks (reference ``agent.py:750-828``)."""

    def forward(self, state: Tensor, is_training: bool = True, mask: Optional[Dict[str, np.ndarray]] = None):
        out = self.model(state)
        logits_list = [head(out) for head in self.mlp_heads]
        va = self.distribution_cfg.get("validate_args", False)
        actions, dists = [], []
        functional_action = None
        for i, logits in enumerate(logits_list):
            if mask is not None:
                if i == 0:
                    logits[torch.logical_not(mask["mask_action_type"].expand_as(logits))] = -torch.inf
                elif i == 1:
                    m = mask["mask_craft_smelt"].expand_as(logits)
                    craft = (functional_action == 15).unsqueeze(-1)
                    logits = torch.where(craft & torch.logical_not(m), torch.full_like(logits, -torch.inf), logits)
                elif i == 2:
                    me = mask["mask_destroy"].expand_as(logits)
                    mp = mask["mask_equip/place"].expand_as(logits)
                    fa = functional_action.unsqueeze(-1)
                    bad = ((fa == 16) | (fa == 17)) & torch.logical_not(mp) | (fa == 18) & torch.logical_not(me)
                    logits = torch.where(bad, torch.full_like(logits, -torch.inf), logits)
            d = OneHotCategoricalStraightThroughValidateArgs(logits=logits, validate_args=va)
            dists.append(d)
            actions.append(d.rsample() if is_training else d.mode)
            if functional_action is None:
                functional_action = actions[0].argmax(dim=-1)
        return tuple(actions), tuple(dists)


# ------------------------------------------------------------------ player
class PlayerDV3(nn.Module):
    """Env-interaction model: keeps (h, z, a) per env on the device (reference ``agent.py:458-599``)."""

    def __init__(self, encoder: nn.Module, rssm: RSSM, actor: nn.Module, actions_dim: Sequence[int], expl_amount: float,
                 num_envs: int, stochastic_size: int, recurrent_state_size: int, device="cpu", discrete_size: int = 32) -> None:
        super().__init__()
        self.encoder = encoder
        self.rssm = rssm
        self.actor = actor
        self.device = device
        self.expl_amount = expl_amount
        self.actions_dim = actions_dim
        self.stochastic_size = stochastic_size
        self.discrete_size = discrete_size
        self.recurrent_state_size = recurrent_state_size
        self.num_envs = num_envs
        # ``use_graphs``: each exploration step is one hipGraph replay (the ~60 small launches of
        # encoder + RSSM step + actor collapse into one); (h, z, a) then live in fixed buffers that the
        # graph updates in place, so resets must write into them (``init_states`` does).
        self.use_graphs = False
        self._graphed = None

    @torch.no_grad()
    def init_states(self, reset_envs: Optional[Sequence[int]] = None) -> None:
        if reset_envs is None or len(reset_envs) == 0:
            actions = torch.zeros(1, self.num_envs, int(np.sum(self.actions_dim)), device=self.device)
            h = torch.tanh(torch.zeros(1, self.num_envs, self.recurrent_state_size, device=self.device))
            z = self.rssm._transition(h, sample_state=False)[1].reshape(1, self.num_envs, -1)
            if self._graphed is not None and self.actions.shape[1] != self.num_envs:
                # a new env count (e.g. the single-env test episode after training on N envs): the captured
                # graphs were recorded for the old buffer shapes - drop them, the next call re-captures
                self._graphed = None
            if self._graphed is not None:  # keep the captured buffers' addresses
                self.actions.copy_(actions)
                self.recurrent_state.copy_(h)
                self.stochastic_state.copy_(z)
            else:
                self.actions, self.recurrent_state, self.stochastic_state = actions, h, z
        else:
            idx = torch.as_tensor(list(reset_envs), device=self.device)
            self.actions[:, idx] = 0
            self.recurrent_state[:, idx] = torch.tanh(torch.zeros_like(self.recurrent_state[:, idx]))
            self.stochastic_state[:, idx] = self.rssm._transition(self.recurrent_state[:, idx], sample_state=False)[1].reshape(
                1, len(reset_envs), -1)

    def get_exploration_action(self, obs: Dict[str, Tensor], is_continuous: bool, mask=None) -> Tuple[Tensor, ...]:
        if self.use_graphs and mask is None and torch.cuda.is_available() and self.actions.is_cuda:
            # two captures: with the exploration ops (amount > 0: a device scalar the graph reads, so a decaying
            # amount needs no re-capture) and without them (amount == 0, the DreamerV3 default: the random
            # one-hot / where kernels would be identities)
            explore = float(self.expl_amount) > 0.0
            if self._graphed is None:
                self._graphed = {}
            if explore not in self._graphed:
                from sheeprl_prey_amd.parallel.graphs import GraphedStep

                self._is_continuous = is_continuous
                if not hasattr(self, "_expl_t"):
                    self._expl_t = torch.zeros((), device=self.actions.device)
                fn = self._graph_step if explore else self._graph_step_greedy
                self._graphed[explore] = GraphedStep(fn, warmup=2, enabled=True,
                                                     name="dv3_player" if explore else "dv3_player_greedy")
            if explore:
                self._expl_t.fill_(float(self.expl_amount))
            out = self._graphed[explore](obs)
            return tuple(out[f"a{i}"] for i in range(len(out)))
        return self._exploration_action(obs, is_continuous, mask)

    @torch.no_grad()
    def _graph_step_greedy(self, obs: Dict[str, Tensor]) -> Dict[str, Tensor]:
        return self._graph_step(obs, explore=False)

    @torch.no_grad()
    def _graph_step(self, obs: Dict[str, Tensor], explore: bool = True) -> Dict[str, Tensor]:
        bufs = (self.actions, self.recurrent_state, self.stochastic_state)
        if explore:
            acts = self._exploration_action(obs, self._is_continuous, None, expl=self._expl_t)
        else:
            acts = self.get_greedy_action(obs)
            if self._is_continuous:
                acts = (torch.cat(acts, -1),)
        for b, new in zip(bufs, (self.actions, self.recurrent_state, self.stochastic_state)):
            b.copy_(new)
        self.actions, self.recurrent_state, self.stochastic_state = bufs
        return {f"a{i}": a for i, a in enumerate(acts)}

    def _exploration_action(self, obs: Dict[str, Tensor], is_continuous: bool, mask=None,
                            expl: Optional[Tensor] = None) -> Tuple[Tensor, ...]:
        """``expl``: device-scalar exploration amount (graph path: always applied, a zero amount is
        the identity); otherwise the Python ``expl_amount`` gates the exploration ops."""
        actions = self.get_greedy_action(obs, mask=mask)
        amount = expl if expl is not None else self.expl_amount
        explore = expl is not None or self.expl_amount > 0.0
        if is_continuous:
            self.actions = torch.cat(actions, -1)
            if explore:  # Normal(a, expl) draw via randn (capturable)
                self.actions = torch.clip(self.actions + amount * torch.randn_like(self.actions), -1, 1)
            out = [self.actions]
        else:
            out = []
            for act in actions:
                if explore:
                    rnd = F.one_hot(torch.randint(0, act.shape[-1], act.shape[:-1], device=act.device), act.shape[-1]).to(act)
                    act = torch.where(torch.rand(act.shape[:1], device=act.device).view(-1, *([1] * (act.dim() - 1))) < amount, rnd, act)
                out.append(act)
            self.actions = torch.cat(out, -1)
        return tuple(out)

    def get_greedy_action(self, obs: Dict[str, Tensor], is_training: bool = True, mask=None) -> Sequence[Tensor]:
        embedded_obs = self.encoder(obs)
        self.recurrent_state = self.rssm.recurrent_model(torch.cat((self.stochastic_state, self.actions), -1), self.recurrent_state)
        _, self.stochastic_state = self.rssm._representation(self.recurrent_state, embedded_obs)
        self.stochastic_state = self.stochastic_state.view(*self.stochastic_state.shape[:-2], self.stochastic_size * self.discrete_size)
        latent = torch.cat((self.stochastic_state, self.recurrent_state), -1)
        if type(self.actor) is Actor and mask is None:
            actions = self.actor.sample_actions(latent, is_training)
        else:
            actions, _ = self.actor(latent, is_training, mask)
        self.actions = torch.cat(actions, -1)
        return actions


# ------------------------------------------------------------------ factory
def build_models(runner, actions_dim: Sequence[int], is_continuous: bool, cfg: Dict[str, Any], obs_space,
                 world_model_state=None, actor_state=None, critic_state=None, target_critic_state=None):
    """Build world model, actor, critic, target critic (reference ``agent.py:831-1068``)."""
    wm_cfg = cfg.algo.world_model
    actor_cfg = cfg.algo.actor
    critic_cfg = cfg.algo.critic
    recurrent_state_size = wm_cfg.recurrent_model.recurrent_state_size
    stochastic_size = wm_cfg.stochastic_size * wm_cfg.discrete_size
    latent_state_size = stochastic_size + recurrent_state_size
    cnn_stages = int(np.log2(cfg.env.screen_size) - np.log2(4))
    cnn_keys_enc = list(cfg.cnn_keys.encoder or [])
    mlp_keys_enc = list(cfg.mlp_keys.encoder or [])
    cnn_encoder = (
        CNNEncoder(keys=cnn_keys_enc, input_channels=[int(np.prod(obs_space[k].shape[:-2])) for k in cnn_keys_enc],
                   image_size=obs_space[cnn_keys_enc[0]].shape[-2:],
                   channels_multiplier=wm_cfg.encoder.cnn_channels_multiplier, layer_norm=wm_cfg.encoder.layer_norm,
                   activation=_act(wm_cfg.encoder.cnn_act), stages=cnn_stages)
        if cnn_keys_enc else None
    )
    mlp_encoder = (
        MLPEncoder(keys=mlp_keys_enc, input_dims=[obs_space[k].shape[0] for k in mlp_keys_enc],
                   mlp_layers=wm_cfg.encoder.mlp_layers, dense_units=wm_cfg.encoder.dense_units,
                   activation=_act(wm_cfg.encoder.dense_act), layer_norm=wm_cfg.encoder.layer_norm)
        if mlp_keys_enc else None
    )
    encoder = MultiEncoder(cnn_encoder, mlp_encoder)
    rm_cfg = dict(wm_cfg.recurrent_model)
    recurrent_model = RecurrentModel(input_size=int(sum(actions_dim) + stochastic_size),
                                     recurrent_state_size=rm_cfg["recurrent_state_size"], dense_units=rm_cfg["dense_units"],
                                     layer_norm=rm_cfg.get("layer_norm", True))
    rep_cfg, tr_cfg = wm_cfg.representation_model, wm_cfg.transition_model
    representation_model = MLP(
        input_dims=recurrent_state_size + encoder.cnn_output_dim + encoder.mlp_output_dim, output_dim=stochastic_size,
        hidden_sizes=[rep_cfg.hidden_size], activation=_act(rep_cfg.dense_act), flatten_dim=None,
        norm_layer=[nn.LayerNorm] if rep_cfg.layer_norm else None,
        norm_args=[{"normalized_shape": rep_cfg.hidden_size}] if rep_cfg.layer_norm else None,
    )
    transition_model = MLP(
        input_dims=recurrent_state_size, output_dim=stochastic_size, hidden_sizes=[tr_cfg.hidden_size],
        activation=_act(tr_cfg.dense_act), flatten_dim=None,
        norm_layer=[nn.LayerNorm] if tr_cfg.layer_norm else None,
        norm_args=[{"normalized_shape": tr_cfg.hidden_size}] if tr_cfg.layer_norm else None,
    )
    rssm = RSSM(recurrent_model.apply(init_weights), representation_model.apply(init_weights),
                transition_model.apply(init_weights), cfg.distribution, discrete=wm_cfg.discrete_size, unimix=cfg.algo.unimix)
    cnn_keys_dec = list(cfg.cnn_keys.decoder or [])
    mlp_keys_dec = list(cfg.mlp_keys.decoder or [])
    cnn_decoder = (
        CNNDecoder(keys=cnn_keys_dec, output_channels=[int(np.prod(obs_space[k].shape[:-2])) for k in cnn_keys_dec],
                   channels_multiplier=wm_cfg.observation_model.cnn_channels_multiplier, latent_state_size=latent_state_size,
                   cnn_encoder_output_dim=cnn_encoder.output_dim, image_size=obs_space[cnn_keys_dec[0]].shape[-2:],
                   activation=_act(wm_cfg.observation_model.cnn_act), layer_norm=wm_cfg.observation_model.layer_norm,
                   stages=cnn_stages)
        if cnn_keys_dec else None
    )
    mlp_decoder = (
        MLPDecoder(keys=mlp_keys_dec, output_dims=[obs_space[k].shape[0] for k in mlp_keys_dec],
                   latent_state_size=latent_state_size, mlp_layers=wm_cfg.observation_model.mlp_layers,
                   dense_units=wm_cfg.observation_model.dense_units, activation=_act(wm_cfg.observation_model.dense_act),
                   layer_norm=wm_cfg.observation_model.layer_norm)
        if mlp_keys_dec else None
    )
    observation_model = MultiDecoder(cnn_decoder, mlp_decoder)

    def head(out_dim, c):
        n = c.mlp_layers
        return MLP(input_dims=latent_state_size, output_dim=out_dim, hidden_sizes=[c.dense_units] * n,
                   activation=_act(c.dense_act), flatten_dim=None,
                   norm_layer=[nn.LayerNorm for _ in range(n)] if c.layer_norm else None,
                   norm_args=[{"normalized_shape": c.dense_units} for _ in range(n)] if c.layer_norm else None)

    reward_model = head(wm_cfg.reward_model.bins, wm_cfg.reward_model)
    continue_model = head(1, wm_cfg.discount_model)
    world_model = WorldModel(encoder.apply(init_weights), rssm, observation_model.apply(init_weights),
                             reward_model.apply(init_weights), continue_model.apply(init_weights))
    actor_cls = get_class(cfg.algo.actor.cls)
    actor = actor_cls(latent_state_size=latent_state_size, actions_dim=actions_dim, is_continuous=is_continuous,
                      init_std=actor_cfg.init_std, min_std=actor_cfg.min_std, dense_units=actor_cfg.dense_units,
                      activation=_act(actor_cfg.dense_act), mlp_layers=actor_cfg.mlp_layers,
                      distribution_cfg=cfg.distribution, layer_norm=actor_cfg.layer_norm, unimix=cfg.algo.unimix)
    critic = head(critic_cfg.bins, critic_cfg)
    actor.apply(init_weights)
    critic.apply(init_weights)
    if cfg.algo.hafner_initialization:
        actor.mlp_heads.apply(uniform_init_weights(1.0))
        critic.model[-1].apply(uniform_init_weights(0.0))
        rssm.transition_model.model[-1].apply(uniform_init_weights(1.0))
        rssm.representation_model.model[-1].apply(uniform_init_weights(1.0))
        world_model.reward_model.model[-1].apply(uniform_init_weights(0.0))
        world_model.continue_model.model[-1].apply(uniform_init_weights(1.0))
        if mlp_decoder is not None:
            mlp_decoder.heads.apply(uniform_init_weights(1.0))
        if cnn_decoder is not None:
            cnn_decoder.model[-1].model[-1].apply(uniform_init_weights(1.0))
    if world_model_state:
        world_model.load_state_dict(world_model_state)
    if actor_state:
        actor.load_state_dict(actor_state)
    if critic_state:
        critic.load_state_dict(critic_state)
    world_model = runner.setup_module(world_model)
    actor = runner.setup_module(actor)
    critic = runner.setup_module(critic)
    target_critic = copy.deepcopy(critic)
    if target_critic_state:
        target_critic.load_state_dict(target_critic_state)
    for p in target_critic.parameters():
        p.requires_grad_(False)
    return world_model, actor, critic, target_critic
