"""Persistent imagination rollout for discrete DreamerV3 actors (``csrc/imagine.hip``).

Reference loop: ``dreamer_v3.py:235-257`` (``RSSM.imagination``, ``agent.py:439-455``, and
``Actor.forward``, ``agent.py:682-739``).  The whole horizon - actor MLP, action heads with unimix
sampling, recurrent input layer, LayerNorm-GRU, transition MLP with unimix prior sampling - is ONE
launch; see the kernel header for the decomposition.  ``fused_imagine`` returns ``None`` when the
modules or shapes are outside what the kernel handles, and the caller keeps the per-op rollout.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
from torch import Tensor, nn

from sheeprl_prey_amd.ops.reference import ACTS

_ACTS = {nn.SiLU: "silu", nn.ELU: "elu", nn.ReLU: "relu", nn.Tanh: "tanh"}


def _parse_mlp(seq: nn.Module) -> Optional[Tuple[List[tuple], Optional[nn.Linear]]]:
    """``[(Linear, LayerNorm, act_code), ...]`` hidden layers and the optional output Linear of an MLP
    ``Sequential`` (after ``fuse_norm_act``), or None if it has any other structure."""
    layers: List[list] = []
    for m in seq.children():
        if isinstance(m, nn.Identity):
            continue
        if isinstance(m, nn.Linear):
            layers.append([m, None, "none"])
        elif isinstance(m, nn.LayerNorm) and layers and layers[-1][1] is None and len(m.normalized_shape) == 1:
            if m.weight is None or m.bias is None:
                return None
            layers[-1][1] = m
            layers[-1][2] = getattr(m, "act", "none")
        elif type(m) in _ACTS and layers and layers[-1][1] is not None and layers[-1][2] == "none":
            layers[-1][2] = _ACTS[type(m)]
        else:
            return None
    if not layers:
        return None
    out = None
    if layers[-1][1] is None:
        out = layers.pop()[0]
    if any(ln is None for _, ln, _ in layers) or any(a not in ACTS for _, _, a in layers):
        return None
    return [(lin, ln, ACTS[a]) for lin, ln, a in layers], out


def _empty(ref: Tensor) -> Tensor:
    return ref.new_empty(0)


def _pad_rows(x: Tensor, m: int) -> Tensor:
    """Zero rows appended up to a multiple of ``m`` (the kernel reads whole 16-row weight tiles)."""
    n = -(-x.shape[0] // m) * m
    if n == x.shape[0]:
        return x.contiguous()
    out = x.new_zeros((n,) + tuple(x.shape[1:]))
    out[: x.shape[0]] = x
    return out


def _b(lin: nn.Linear, ref: Tensor) -> Tensor:
    return lin.bias.detach() if lin.bias is not None else _empty(ref)


class _Plan:
    """Module structure + launch geometry, cached per (rssm, actor, M)."""

    def __init__(self, rssm, actor, M: int):
        from sheeprl_prey_amd.ops import _ext

        self.ok = False
        a = _parse_mlp(actor.model.model if hasattr(actor.model, "model") else actor.model)
        r = _parse_mlp(rssm.recurrent_model.mlp.model)
        tr = _parse_mlp(rssm.transition_model.model)
        gru = rssm.recurrent_model.rnn
        if a is None or r is None or tr is None or a[1] is not None or r[1] is not None or tr[1] is None:
            return
        if len(r[0]) != 1 or len(tr[0]) != 1 or not isinstance(gru.layer_norm, nn.LayerNorm):
            return
        if gru.layer_norm.weight is None or gru.layer_norm.bias is None:
            return
        self.actor_layers = a[0]
        self.rec = r[0][0]
        self.trans, self.trans_out = tr[0][0], tr[1]
        self.gru = gru
        self.heads = list(actor.mlp_heads)
        self.head_sizes = [int(h.out_features) for h in self.heads]
        self.S = int(self.trans_out.out_features)
        self.Hd = int(gru.hidden_size)
        self.D = int(self.rec[0].out_features)
        self.Da = int(self.actor_layers[0][0].out_features)
        self.Ht = int(self.trans[0].out_features)
        self.A = sum(self.head_sizes)
        self.disc = int(rssm.discrete)
        self.La = len(self.actor_layers)
        if any(int(l.out_features) != self.Da for l, _, _ in self.actor_layers) or max(self.head_sizes) > 32:
            return
        if int(self.actor_layers[0][0].in_features) != self.S + self.Hd or int(self.rec[0].in_features) != self.S + self.A:
            return
        if int(gru.linear.in_features) != self.Hd + self.D or int(self.trans[0].in_features) != self.Hd:
            return
        if int(self.trans_out.in_features) != self.Ht or any(int(h.in_features) != self.Da for h in self.heads):
            return
        acts = {c for _, _, c in self.actor_layers} | {self.rec[2], self.trans[2]}
        if acts != {ACTS["silu"]} or len({l[1].eps for l in self.actor_layers}) != 1:
            return  # the kernel's LayerNorm staging is specialised for SiLU (every DreamerV3 preset)
        self.NB, self.nslots, self.sync_words, _ = _ext().imagine_info(
            M, self.S, self.Hd, self.D, self.Da, self.Ht, self.A, len(self.heads), self.disc, self.La)
        self.ok = self.NB > 0
        self.ints_tail = [self.La, self.Ht, self.disc, self.actor_layers[0][2], self.rec[2], self.trans[2]] + self.head_sizes


_PLANS: dict = {}


def _plan(rssm, actor, M: int) -> _Plan:
    key = (id(rssm), id(actor), M)
    p = _PLANS.get(key)
    if p is None:
        p = _PLANS[key] = _Plan(rssm, actor, M)
    return p


def fused_imagine(rssm, actor, post: Tensor, h: Tensor, horizon: int, U: Tensor) -> Optional[Tensor]:
    """Imagined trajectories as one buffer ``[horizon + 1, M, A + S + Hd]`` = (action | prior | h)
    (the layout of ``RSSM.imagine_discrete``), or None when unsupported.

    ``U [horizon + 1, M * (heads + G)]`` holds every uniform of the rollout (per step: one per row and
    head, then one per row and prior categorical), the same draw order as the per-op rollout."""
    from sheeprl_prey_amd.ops import _ext

    M = post.shape[0]
    p = _plan(rssm, actor, M)
    if not p.ok or post.dtype != torch.float32 or h.dtype != torch.float32:
        return None
    S, Hd, A, G = p.S, p.Hd, p.A, p.S // p.disc
    dev = post.device
    buf = post.new_empty(horizon + 1, M, A + S + Hd)
    buf[0, :, A:A + S].copy_(post)
    buf[0, :, A + S:].copy_(h)
    idx = post.view(M, G, p.disc).argmax(-1).to(torch.int32)
    Y = post.new_empty(2, M, max(p.Da, p.D, p.Ht))
    part = post.new_empty(2, M, p.NB, 2)
    sync = torch.empty(p.sync_words, device=dev, dtype=torch.int32)
    d = lambda t: t.detach()  # noqa: E731
    Wa0 = d(p.actor_layers[0][0].weight)
    ln_r, ln_g, ln_t = p.rec[1], p.gru.layer_norm, p.trans[1]
    ts = [
        Wa0[:, :S].t().contiguous(),
        _pad_rows(torch.cat([d(hd.weight) for hd in p.heads], 0), 16),
        _pad_rows(torch.cat([_b(hd, post) for hd in p.heads], 0), 16) if all(hd.bias is not None for hd in p.heads)
        else _empty(post),
        d(p.rec[0].weight).t().contiguous(), _b(p.rec[0], post), d(ln_r.weight), d(ln_r.bias),
        d(p.gru.linear.weight), _b(p.gru.linear, post), d(ln_g.weight), d(ln_g.bias),
        d(p.trans[0].weight), _b(p.trans[0], post), d(ln_t.weight), d(ln_t.bias),
        d(p.trans_out.weight), _b(p.trans_out, post),
        U, buf, Y, part, idx, sync,
    ]
    for lin, ln, _ in p.actor_layers:
        ts += [d(lin.weight), _b(lin, post), d(ln.weight), d(ln.bias)]
    ints = [M, horizon, S, Hd, p.D, p.Da] + p.ints_tail
    fl = [float(actor._unimix), float(rssm.unimix), float(p.actor_layers[0][1].eps), float(ln_r.eps), float(ln_g.eps),
          float(ln_t.eps)]
    _ext().imagine_rollout(ts, ints, fl)
    p.last_sync = sync  # error word at [nslots * 32] (tests)
    return buf
