"""Whole-stack implicit-GEMM convolutions for the Dreamer CNN encoder / decoder (HIP, ``csrc/conv.hip``).

Reference modules: ``dreamer_v3/agent.py:48-80`` (``CNNEncoder``: ``stages`` x Conv2d k4 s2 p1 (no bias)
-> channel LayerNorm -> SiLU, flatten) and ``:160-206`` (``CNNDecoder``: Linear -> unflatten ->
ConvTranspose2d k4 s2 p1 (+LN+SiLU) x (stages-1) -> ConvTranspose2d (bias) -> +0.5).

One ``autograd.Function`` per stack keeps every intermediate activation in NHWC and fuses each
channel LayerNorm + activation into the epilogue of the convolution that produces it (forward), and
each LayerNorm/activation backward into the epilogue of the data-gradient convolution that produces
its input gradient (backward).  The stack's weights stay in the reference's ``state_dict`` layout;
they are re-packed (one tiny kernel per layer) at use.  Eligibility (``encoder_spec`` /
``decoder_spec``): k4 s2 p1 convolutions, channel counts in ``_OK_CH`` (every preset's multiplier:
32 / 64 / 96 x 2^k, i.e. Atari-100k, L, XL and the 128 px 5-stage stacks), 1-4 image channels (RGB or
grayscale), power-of-two image size of at least 32; anything else runs the eager modules (MIOpen).
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence, Tuple

import torch
from torch import Tensor, nn

from sheeprl_prey_amd.ops import sidestream as ss

_OK_CH = (32, 64, 96, 128, 192, 256, 384, 512, 768, 1024)  # conv.hip tile table
ENABLED = True  # A/B switch: False routes the stacks through the per-layer modules (MIOpen + LN kernels)
# Below this many frames (e.g. the env-interaction player, one frame per env) the deepest stage has
# too few output rows to fill the chip (E4: 16 rows per frame) and a single workgroup walks all of K:
# no-grad calls there take the split-K small-batch stack (csrc/conv_small.hip, ``encoder_small``).
MIN_FRAMES = 64
SMALL_ENABLED = True  # False sends the small no-grad batches to the per-layer modules (MIOpen; tests toggle it)


def _C():
    from sheeprl_prey_amd import ops

    return ops._ext()


def _act_code(act: str) -> int:
    from sheeprl_prey_amd.ops.reference import ACTS

    return ACTS[(act or "none").lower()]


def _pow2(v: int) -> bool:
    return v > 0 and (v & (v - 1)) == 0


def _is_k4s2p1(m: nn.Module) -> bool:
    return (tuple(m.kernel_size) == (4, 4) and tuple(m.stride) == (2, 2) and tuple(m.padding) == (1, 1)
            and tuple(m.dilation) == (1, 1) and m.groups == 1 and getattr(m, "padding_mode", "zeros") == "zeros"
            and tuple(getattr(m, "output_padding", (0, 0))) == (0, 0))


def _stages(seq: nn.Sequential, conv_type) -> Optional[List[Tuple[nn.Module, Optional[nn.Module]]]]:
    """[(conv, fused LN-or-None)] of a ``[conv, LayerNormChannelLast(act), Identity]*`` sequence."""
    from sheeprl_prey_amd.utils.model import LayerNormChannelLast

    mods = [m for m in seq if not isinstance(m, nn.Identity)]
    out = []
    i = 0
    while i < len(mods):
        conv = mods[i]
        if not isinstance(conv, conv_type) or not _is_k4s2p1(conv):
            return None
        ln = None
        if i + 1 < len(mods) and isinstance(mods[i + 1], LayerNormChannelLast):
            ln = mods[i + 1]
            i += 1
        elif i + 1 < len(mods):
            return None  # an unfused activation / dropout / other norm: not this path
        out.append((conv, ln))
        i += 1
    return out


def encoder_spec(model: nn.Module, image_hw: Tuple[int, int], in_ch: int):
    """Stages of a ``CNNEncoder.model`` if the fused path covers it, else None."""
    try:
        seq = model[0].model
    except (AttributeError, IndexError, TypeError):
        return None
    st = _stages(seq, nn.Conv2d)
    if not st or in_ch > 4 or not (_pow2(image_hw[0]) and _pow2(image_hw[1])) or min(image_hw) < 32:
        return None
    h, w = image_hw
    for conv, ln in st:
        if conv.bias is not None or ln is None or conv.out_channels not in _OK_CH or ln.weight is None or ln.bias is None:
            return None
        if len(ln.normalized_shape) != 1 or ln.normalized_shape[0] != conv.out_channels:
            return None
        h, w = h // 2, w // 2
        if h < 1 or w < 1:
            return None
    return st


def decoder_spec(model: nn.Module, out_ch: int):
    """(linear, stages) of a ``CNNDecoder.model`` if the fused path covers it, else None."""
    try:
        lin, unflat, decnn = model[0], model[1], model[2]
    except (IndexError, TypeError):
        return None
    if not isinstance(lin, nn.Linear) or not isinstance(unflat, nn.Unflatten):
        return None
    st = _stages(decnn.model, nn.ConvTranspose2d)
    if not st or len(st) < 3:  # the last layer's input grid (4 * 2^(stages-1)) must be a multiple of 16
        return None
    for conv, ln in st[:-1]:
        if ln is None or conv.bias is not None or conv.in_channels not in _OK_CH or conv.out_channels not in _OK_CH:
            return None
        if ln.weight is None or ln.bias is None or ln.normalized_shape[0] != conv.out_channels:
            return None
    last, ln_last = st[-1]
    if ln_last is not None or last.bias is None or last.in_channels % 32 or not 1 <= last.out_channels <= 4:
        return None
    if out_ch != last.out_channels:
        return None
    return lin, st


# ---------------------------------------------------------------------------------- encoder
class EncoderConvFn(torch.autograd.Function):
    """x: [N, C<=4, H, W] float (already scaled), or the raw uint8 frames with ``meta["scale"]``
    (the scaling is folded into the NHWC conversion) -> flat features [N, C_L * H_L * W_L] (C,H,W order)."""

    @staticmethod
    def forward(ctx, x: Tensor, meta, *params: Tensor) -> Tensor:
        C = _C()
        L = len(meta["cout"])
        act, eps = meta["act"], meta["eps"]
        ws, gs, bs = params[:L], params[L:2 * L], params[2 * L:3 * L]
        q = C.conv_to_nhwc4(x.contiguous(), float(meta.get("scale", 1.0)))
        # every weight pack of the step in ONE launch: the forward's DOWN forms and (with grad) the backward's UP forms
        grad = any(ctx.needs_input_grad)
        jobs = [(ws[i], 0, q.shape[3] if i == 0 else ws[i].shape[1]) for i in range(L)]
        if grad:
            jobs += [(ws[i], 1, ws[i].shape[1]) for i in range(1, L)]
        packs = C.conv_pack_many([j[0] for j in jobs], [j[1] for j in jobs], [int(j[2]) for j in jobs])
        saved = []
        for i in range(L):
            z, y, mean, rstd = C.conv_gemm(0, q, packs[i], ws[i].shape[0], 0, gs[i], bs[i], eps[i], act[i], i == L - 1,
                                           None, None, None, None, None, None, 0.0, 0)
            saved += [q, z, mean, rstd]
            q = y
        ctx.save_for_backward(*saved, *params, *packs[L:])
        ctx.meta, ctx.L, ctx.in_ch = meta, L, x.shape[1]
        return q

    @staticmethod
    def backward(ctx, dy: Tensor):
        C = _C()
        L, meta = ctx.L, ctx.meta
        sv = ctx.saved_tensors
        acts = sv[:4 * L]
        params = sv[4 * L:4 * L + 3 * L]
        up_packs = sv[4 * L + 3 * L:]  # UP forms of layers 1..L-1 (made by the forward's one pack launch)
        ws, gs, bs = params[:L], params[L:2 * L], params[2 * L:3 * L]
        act = meta["act"]
        dgb = torch.zeros(2 * sum(int(g.numel()) for g in gs), device=dy.device, dtype=dy.dtype)
        dgs, dbs, o = [], [], 0
        for g in gs:
            dgs.append(dgb[o:o + g.numel()])
            o += g.numel()
            dbs.append(dgb[o:o + g.numel()])
            o += g.numel()
        q, z, mean, rstd = acts[4 * (L - 1):4 * L]
        dz = C.conv_ln_bwd_flat(dy.contiguous(), z, mean, rstd, gs[-1], bs[-1], act[-1], dgs[-1], dbs[-1])
        dws: List[Optional[Tensor]] = [None] * L
        parts: List[Tensor] = []  # the LayerNorm-backward convs' dgamma / dbeta partials, reduced together at the end
        for i in range(L - 1, -1, -1):
            q = acts[4 * i]
            cin = ws[i].shape[1]
            dws[i] = C.conv_wgrad(dz, q, cin)
            if i > 0:
                wp = up_packs[i - 1]
                _, zp, mp, rp = acts[4 * (i - 1):4 * i]
                dz, part = C.conv_gemm_lnbwd_part(1, dz, wp, cin, gs[i - 1], bs[i - 1], act[i - 1], zp, mp, rp)
                parts.append(part)
        if parts:  # layers L-2 .. 0, one pair of launches for all of them (assigned: the buffer's other slices)
            C.conv_part_reduce_many(parts, dgs[L - 2::-1], dbs[L - 2::-1], True)
        return (None, None, *dws, *[d.view_as(g) for d, g in zip(dgs, gs)], *[d.view_as(b) for d, b in zip(dbs, bs)])


def encoder_forward(stages, x: Tensor, scale: float = 1.0) -> Tensor:
    from sheeprl_prey_amd.ops import _act_code as act_code

    convs = [c for c, _ in stages]
    lns = [ln for _, ln in stages]
    meta = {"cout": [c.out_channels for c in convs], "act": [act_code(ln.act) for ln in lns], "eps": [float(ln.eps) for ln in lns],
            "scale": float(scale)}
    params = [c.weight for c in convs] + [ln.weight for ln in lns] + [ln.bias for ln in lns]
    return EncoderConvFn.apply(x, meta, *params)


def encoder_small(stages, x: Tensor, scale: float = 1.0) -> Tensor:
    """No-grad encoder stack for a few frames (the player): [N, C, H, W] float / uint8 -> flat features, two
    launches per stage (split-K MFMA conv + slice-sum / LayerNorm / activation), NCHW between stages."""
    from sheeprl_prey_amd.ops import _act_code as act_code

    convs = [c for c, _ in stages]
    lns = [ln for _, ln in stages]
    return _C().conv_small_encoder(x.contiguous(), [c.weight for c in convs], [ln.weight for ln in lns],
                                   [ln.bias for ln in lns], [float(ln.eps) for ln in lns],
                                   [act_code(ln.act) for ln in lns], float(scale))


def _wgrad(C, P: Tensor, Q: Tensor, cb: int, w: Tensor) -> Optional[Tensor]:
    """Decoder weight gradient of parameter ``w``: in line, or (inside a deferral scope) queued to run beside the
    scan backward and None returned (``ops/sidestream.py`` assigns it to ``w.grad``)."""
    return ss.param_grads(P.device, lambda: (C.conv_wgrad(P, Q, cb),), [w], P, Q)[0]


# ---------------------------------------------------------------------------------- decoder
class DecoderConvFn(torch.autograd.Function):
    """h: [N, C0*4*4] (Linear output, C,H,W order) -> image [N, 3, 2^L*4, 2^L*4] NCHW, + c0."""

    @staticmethod
    def forward(ctx, h: Tensor, meta, *params: Tensor) -> Tensor:
        C = _C()
        L = len(meta["cout"])  # LN stages; the last (plain) conv follows
        act, eps = meta["act"], meta["eps"]
        ws = params[:L + 1]
        gs, bs = params[L + 1:2 * L + 1], params[2 * L + 1:3 * L + 1]
        bias_last = params[3 * L + 1]
        N = h.shape[0]
        c0 = ws[0].shape[0]
        p = h.reshape(N, c0, 4, 4).permute(0, 2, 3, 1).contiguous()
        # every weight pack of the step in ONE launch: the forward's UP forms and (with grad) the backward's DOWN forms
        # (the last layer's against the 4-channel NHWC image gradient)
        grad = any(ctx.needs_input_grad)
        jobs = [(ws[i], 1, ws[i].shape[1]) for i in range(L)]
        if grad:
            jobs += [(ws[i], 0, ws[i].shape[1]) for i in range(L)] + [(ws[L], 0, 4)]
        packs = C.conv_pack_many([j[0] for j in jobs], [j[1] for j in jobs], [int(j[2]) for j in jobs])
        saved = []
        for i in range(L):
            cout = ws[i].shape[1]
            z, y, mean, rstd = C.conv_gemm(1, p, packs[i], cout, 0, gs[i], bs[i], eps[i], act[i], False,
                                           None, None, None, None, None, None, 0.0, 0)
            saved += [p, z, mean, rstd]
            p = y
        out = C.conv_up_small(p, ws[L], bias_last, float(meta["c0"]))
        saved.append(p)
        ctx.save_for_backward(*saved, *params, *packs[L:])
        ctx.meta, ctx.L = meta, L
        ctx.wparams = params[:L + 1]  # the conv weights (leaves) a deferred weight gradient is assigned to
        return out

    @staticmethod
    def backward(ctx, dout: Tensor):
        C = _C()
        L, meta = ctx.L, ctx.meta
        sv = ctx.saved_tensors
        acts, p_last = sv[:4 * L], sv[4 * L]
        params = sv[4 * L + 1:4 * L + 1 + 3 * L + 2]
        down_packs = sv[4 * L + 1 + 3 * L + 2:]  # DOWN forms of layers 0..L-1, then the last layer's (the forward's pack launch)
        ws = params[:L + 1]
        gs, bs = params[L + 1:2 * L + 1], params[2 * L + 1:3 * L + 1]
        act = meta["act"]
        dout = dout.contiguous()
        # every slice is assigned by the deferred partial reduction below (no zero fill)
        dgb = torch.empty(2 * sum(int(g.numel()) for g in gs), device=dout.device, dtype=dout.dtype)
        dgs, dbs, o = [], [], 0
        for g in gs:
            dgs.append(dgb[o:o + g.numel()])
            o += g.numel()
            dbs.append(dgb[o:o + g.numel()])
            o += g.numel()
        # NHWC4 form of the image gradient and the last layer's bias gradient in one pass over it
        q, dbias = C.conv_to_nhwc4_sum(dout)
        dws: List[Optional[Tensor]] = [None] * (L + 1)
        cout_last = ws[L].shape[1]
        # the weight gradients leave the critical path (data gradients -> scan backward -> encoder): inside the
        # world-model backward they are queued and run beside the scan backward (ops/sidestream.py)
        dws[L] = _wgrad(C, p_last, q, cout_last, ctx.wparams[L])
        assert q.shape[3] == 4, q.shape
        wp = down_packs[L]
        _, zp, mp, rp = acts[4 * (L - 1):4 * L]
        dz, part = C.conv_gemm_lnbwd_part(0, q, wp, ws[L].shape[0], gs[L - 1], bs[L - 1], act[L - 1], zp, mp, rp)
        parts = [part]  # the LayerNorm-backward convs' dgamma / dbeta partials, reduced together at the end
        dh = None
        for i in range(L - 1, -1, -1):
            p = acts[4 * i]
            cout = ws[i].shape[1]
            dws[i] = _wgrad(C, p, dz, cout, ctx.wparams[i])
            wp = down_packs[i]
            cin = ws[i].shape[0]
            if i > 0:
                _, zp, mp, rp = acts[4 * (i - 1):4 * i]
                dz, part = C.conv_gemm_lnbwd_part(0, dz, wp, cin, gs[i - 1], bs[i - 1], act[i - 1], zp, mp, rp)
                parts.append(part)
            else:
                dh = C.conv_gemm(0, dz, wp, cin, 2, None, None, 0.0, 0, True, None, None, None, None, None, None,
                                 0.0, cin)[0]
        C.conv_part_reduce_many(parts, dgs[::-1], dbs[::-1], True)  # layers L-1 .. 0
        dh = dh.reshape(dh.shape[0], -1)
        return (dh, None, *dws, *[d.view_as(g) for d, g in zip(dgs, gs)], *[d.view_as(b) for d, b in zip(dbs, bs)],
                dbias)


def decoder_forward(stages, h: Tensor, c0: float = 0.0) -> Tensor:
    from sheeprl_prey_amd.ops import _act_code as act_code

    ln_st = stages[:-1]
    last = stages[-1][0]
    meta = {"cout": [c.out_channels for c, _ in ln_st], "act": [act_code(ln.act) for _, ln in ln_st],
            "eps": [float(ln.eps) for _, ln in ln_st], "c0": float(c0)}
    params = ([c.weight for c, _ in ln_st] + [last.weight] + [ln.weight for _, ln in ln_st] + [ln.bias for _, ln in ln_st]
              + [last.bias])
    return DecoderConvFn.apply(h, meta, *params)
