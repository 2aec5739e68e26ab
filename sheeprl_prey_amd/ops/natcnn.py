"""NatureCNN trunk on the hand-written implicit-GEMM kernels (``csrc/natcnn.hip``).

Reference: ``sheeprl/models/models.py:287-327`` (Conv 8x8 s4 -> ReLU -> Conv 4x4 s2 -> ReLU -> Conv
3x3 s1 -> ReLU, valid padding).  The stack runs NHWC end to end; one autograd node owns all three
convolutions: forward saves the inputs and the ReLU outputs (the ReLU mask of the backward is
``y > 0``), backward runs weight+bias gradient and data gradient GEMMs per layer.  Weights stay in
the reference's ``[Co, Ci, KH, KW]`` parameters (checkpoint parity); the packed ``[Co, KH*KW*Ci]``
view is a differentiable permute.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
from torch import Tensor, nn


class _ConvReluStack(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: Tensor, geo: Tuple[Tuple[int, int, int], ...], *params: Tensor) -> Tensor:
        from sheeprl_prey_amd.ops import _ext

        C = _ext()
        ys: List[Tensor] = []
        h = x
        for (KH, KW, S), wp, b in zip(geo, params[0::2], params[1::2]):
            h = C.nc_conv_fwd(h, wp, b, KH, KW, S)
            ys.append(h)
        ctx.save_for_backward(x, *ys, *params)
        ctx.geo = geo
        return h

    @staticmethod
    def backward(ctx, dy: Tensor):
        from sheeprl_prey_amd.ops import _ext

        C = _ext()
        saved = ctx.saved_tensors
        L = len(ctx.geo)
        x, ys, params = saved[0], saved[1:1 + L], saved[1 + L:]
        grads: List[Optional[Tensor]] = [None] * (2 * L)
        d = dy.contiguous()
        for l in reversed(range(L)):
            KH, KW, S = ctx.geo[l]
            inp = x if l == 0 else ys[l - 1]
            need_dx = l > 0 or ctx.needs_input_grad[0]
            dx, dw, db = C.nc_conv_bwd(inp, ys[l], d, params[2 * l], KH, KW, S, need_dx)
            grads[2 * l] = dw
            grads[2 * l + 1] = db
            d = dx
        return (d if ctx.needs_input_grad[0] else None, None, *grads)


def conv_relu_plan(model: nn.Sequential) -> Optional[List[nn.Conv2d]]:
    """The Conv2d layers of a ``[Conv2d, ReLU]*`` stack the kernels cover (valid padding, dilation 1,
    groups 1, bias, channels multiple of 4), or None."""
    convs: List[nn.Conv2d] = []
    mods = [m for m in model if not isinstance(m, nn.Identity)]
    if len(mods) % 2:
        return None
    for conv, act in zip(mods[0::2], mods[1::2]):
        if not isinstance(conv, nn.Conv2d) or not isinstance(act, nn.ReLU):
            return None
        if (conv.padding not in ((0, 0), 0, "valid") or conv.dilation != (1, 1) or conv.groups != 1 or conv.bias is None
                or conv.stride[0] != conv.stride[1] or conv.in_channels % 4 or conv.out_channels % 4):
            return None
        convs.append(conv)
    return convs or None


def conv_relu_stack(convs: Sequence[nn.Conv2d], x: Tensor) -> Tensor:
    """``relu(conv(...relu(conv(x))))`` for NCHW ``x`` [N, C, H, W]; returns NCHW (a view of NHWC)."""
    geo = tuple((int(c.kernel_size[0]), int(c.kernel_size[1]), int(c.stride[0])) for c in convs)
    params: List[Tensor] = []
    for c in convs:
        params += [c.weight.permute(0, 2, 3, 1).reshape(c.out_channels, -1), c.bias]
    y = _ConvReluStack.apply(x.permute(0, 2, 3, 1).contiguous(), geo, *params)
    return y.permute(0, 3, 1, 2)
