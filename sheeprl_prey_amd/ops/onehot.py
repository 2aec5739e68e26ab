"""First layers over one-hot inputs as row gathers (``csrc/onehot.hip``).

DreamerV3's latents are ``[z | h]`` with ``z`` the straight-through sample of 32 categoricals (exactly
one-hot in the forward).  For the first Linear of every MLP reading a latent the ``z`` columns are a sum
of 32 rows of the transposed weight: the layer becomes a ``K = |h|`` library GEMM plus ONE kernel that
adds the gathered rows and applies the layer's LayerNorm + activation (one wave per row).  At the
Atari-100k shapes that removes 2/3 of the FLOPs of every such layer (K 1536 -> 512) and the separate
LayerNorm launch.  The backward is the dense one (``dW = dz^T x``, ``dx = dz W``): the straight-through
gradient of ``z`` is dense.

Index layout: ``idx[r, j]`` = absolute input column of the j-th hot entry of row r, minus ``off`` = the
row of the transposed weight table (``W[:, cols].T``).
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import Tensor, nn

from sheeprl_prey_amd import ops

_ERR: dict = {}


def _err_word(device) -> Tensor:
    key = str(device)
    w = _ERR.get(key)
    if w is None:
        w = _ERR[key] = torch.zeros(1, dtype=torch.int32, device=device)
    return w


def check_onehot_error() -> None:
    """Host check (off the hot path) of the gather kernel's error word (an index outside its table)."""
    for w in _ERR.values():
        if int(w.item()) != 0:
            w.zero_()
            raise RuntimeError("onehot_gather_ln: a hot index was outside its weight table (skipped rows read as 0)")


def onehot_index(x: Tensor, classes: int, out: Tensor, off: int = 0) -> Tensor:
    """``out[r, g] = off + g*classes + argmax(x[r, g*classes:(g+1)*classes])`` (x row-strided 2-D)."""
    ops._ext().onehot_index(x, int(classes), out, int(off))
    return out


def layer_supported(lin: nn.Linear, n_onehot: int) -> bool:
    N = lin.out_features
    return N % 4 == 0 and N <= 4096 and 0 < n_onehot <= lin.in_features


def _ln_parts(ln: Optional[nn.Module]):
    if ln is None:
        return None, None, 0.0, ops._act_code("none"), False
    return ln.weight, ln.bias, float(ln.eps), ops._act_code(getattr(ln, "act", "none")), True


def gather_first_layer(x: Tensor, idx: Tensor, G: int, off: int, lin: nn.Linear, ln: Optional[nn.Module], n_onehot: int,
                       table: Optional[Tensor] = None, y_out: Optional[Tensor] = None, z_out: Optional[Tensor] = None,
                       mean: Optional[Tensor] = None, rstd: Optional[Tensor] = None, Y: Optional[Tensor] = None) -> Tensor:
    """No-grad forward of ``act(LN(lin(x)))`` where ``x[:, :n_onehot]`` is one-hot with hot columns
    ``idx[:, :G] - off`` (x may be a row-strided 2-D view; the dense tail ``x[:, n_onehot:]`` goes through
    a K = in - n_onehot GEMM - or ``Y``, that product computed by the caller, e.g. as one column block of a
    wider GEMM over the same rows).  ``table`` = ``lin.weight[:, :n_onehot].T`` (contiguous) when cached by
    the caller.  Outputs may be preallocated row-strided views."""
    C = ops._ext()
    W = lin.weight
    M, N = x.shape[0], W.shape[0]
    if table is None:
        table = ops.transpose_many([W[:, :n_onehot]])[0]
    if Y is None and x.shape[1] > n_onehot:
        Y = torch.mm(x[:, n_onehot:], W[:, n_onehot:].t())
    if y_out is None:
        y_out = torch.empty(M, N, device=x.device, dtype=x.dtype)
    g, b, eps, act, use_ln = _ln_parts(ln)
    ok = C.onehot_gather_ln(Y, idx, int(G), int(off), table, lin.bias, g, b, eps, act, use_ln, z_out, y_out, mean, rstd,
                            _err_word(x.device))
    if not ok:
        raise RuntimeError(f"onehot_gather_ln: unsupported layer width {N}")
    return y_out


class _GatherFirstLayer(torch.autograd.Function):
    """``act(LN(lin(x)))`` with the one-hot columns gathered (forward) and the dense backward."""

    @staticmethod
    def forward(ctx, x, idx, W, bias, gamma, beta, G, off, n_onehot, eps, act, use_ln, table=None):
        C = ops._ext()
        x2 = x.reshape(-1, x.shape[-1])
        idx2 = idx.reshape(-1, idx.shape[-1])
        M, N = x2.shape[0], W.shape[0]
        if table is None:
            table = ops.transpose_many([W[:, :n_onehot]])[0]
        Y = torch.mm(x2[:, n_onehot:], W[:, n_onehot:].t()) if x2.shape[1] > n_onehot else None
        z = torch.empty(M, N, device=x.device, dtype=x.dtype)
        y = torch.empty(M, N, device=x.device, dtype=x.dtype)
        mean = torch.empty(M, device=x.device, dtype=x.dtype) if use_ln else None
        rstd = torch.empty(M, device=x.device, dtype=x.dtype) if use_ln else None
        ok = C.onehot_gather_ln(Y, idx2, int(G), int(off), table, bias, gamma, beta, float(eps), int(act), bool(use_ln), z, y,
                                mean, rstd, _err_word(x.device))
        if not ok:
            raise RuntimeError(f"onehot_gather_ln: unsupported layer width {N}")
        ctx.save_for_backward(x2, idx2, W, gamma, beta, z, mean, rstd)
        ctx.params = (W, bias)  # the leaves a deferred weight gradient is assigned to (ops/sidestream.py)
        ctx.meta = (act, use_ln, bias is not None, x.shape, int(G), int(off), int(n_onehot))
        return y.view(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        x2, idx2, W, gamma, beta, z, mean, rstd = ctx.saved_tensors
        act, use_ln, has_bias, xshape, G, off, n_onehot = ctx.meta
        C = ops._ext()
        N = W.shape[0]
        dy2 = dy.reshape(-1, N).contiguous()
        dg = db = None
        if use_ln:
            dz, dg, db = C.ln_act_bwd(z, dy2, gamma, beta, mean, rstd, int(act))
        elif act != ops._act_code("none"):
            zz = z.detach().requires_grad_(True)
            with torch.enable_grad():
                yy = ops.reference.act_fn(zz, {v: k for k, v in ops.ACTS.items()}[act])
            dz = torch.autograd.grad(yy, zz, dy2)[0]
        else:
            dz = dy2
        dx = None
        if ctx.needs_input_grad[0]:
            dx = dz.mm(W).view(xshape)
        from sheeprl_prey_amd.ops import sidestream as ss

        meta = (ctx.meta, tuple(ctx.needs_input_grad))
        if ss.active(dz.device) and ctx.needs_input_grad[2]:
            # inside a deferral scope (the world-model backward): parameter gradients beside the scan backward
            dW, dbias = ss.param_grads(dz.device, lambda: _GatherFirstLayer._param_grads(meta, dz, x2, idx2),
                                       ctx.params, dz, x2, idx2)
        else:
            dW, dbias = _GatherFirstLayer._param_grads(meta, dz, x2, idx2)
        return (dx, None, dW, dbias, dg if ctx.needs_input_grad[4] else None, db if ctx.needs_input_grad[5] else None,
                None, None, None, None, None, None, None)

    @staticmethod
    def _param_grads(meta, dz, x2, idx2, out=None):
        (act, use_ln, has_bias, xshape, G, off, n_onehot), needs = meta
        dW = dbias = None
        if needs[2] and ops.wgrad_ok(dz):
            # one-hot columns scattered, the dense tail by the split-K kernel, the bias sum on the side (wgrad.hip)
            want_b = has_bias and needs[3]
            if x2.shape[1] > n_onehot and ops.wgrad_onehot_ok(dz, G, n_onehot):
                dW, dbias = ops.wgrad(dz, x2[:, n_onehot:], onehot=(idx2, G, off, n_onehot), bias=want_b, out=out)
            else:
                dW, dbias = ops.wgrad(dz, x2, bias=want_b, out=out)
        elif needs[2]:
            dW = dz.t().mm(x2)  # x2 may be row-strided (a view into the trajectory buffer): mm takes the stride
        if has_bias and needs[3] and dbias is None:
            dbias = ops._ext().colsum(dz)
        return dW, dbias


def first_layer(x: Tensor, idx: Tensor, G: int, off: int, lin: nn.Linear, ln: Optional[nn.Module], n_onehot: int,
                table: Optional[Tensor] = None) -> Tensor:
    """Autograd form of ``gather_first_layer`` (any leading dims; x may be row-strided; ``table`` as there)."""
    g, b, eps, act, use_ln = _ln_parts(ln)
    return _GatherFirstLayer.apply(x, idx, lin.weight, lin.bias, g, b, int(G), int(off), int(n_onehot), eps, act, use_ln,
                                   table)


def mlp_split(mlp: nn.Module):
    """(first Linear, its fused LayerNorm or None, the remaining modules) of a ``models.MLP`` whose first
    block is ``[Linear, LayerNorm(act), Identity]`` or a plain ``[Linear, ...]``; None otherwise."""
    from sheeprl_prey_amd.utils.model import LayerNorm

    if getattr(mlp, "flatten_dim", None) is not None:
        return None
    seq = list(getattr(mlp, "model", mlp))
    if not seq or not isinstance(seq[0], nn.Linear):
        return None
    if len(seq) >= 3 and type(seq[1]) is LayerNorm and isinstance(seq[2], nn.Identity):
        if len(seq[1].normalized_shape) != 1 or seq[1].weight is None or seq[1].bias is None:
            return None
        return seq[0], seq[1], seq[3:]
    if len(seq) == 1 or not isinstance(seq[1], (nn.LayerNorm, nn.Dropout)):
        return seq[0], None, seq[1:]
    return None


def head_table(mlp: nn.Module, n_onehot: int) -> Optional[Tensor]:
    """The one-hot columns of ``mlp``'s first Linear (``W[:, :n_onehot]``, a source for ``ops.transpose_many``: several
    heads' tables in one launch) or None when ``mlp_forward`` would not gather."""
    sp = mlp_split(mlp)
    if sp is None or not layer_supported(sp[0], n_onehot):
        return None
    return sp[0].weight[:, :n_onehot]


def mlp_forward(mlp: nn.Module, x: Tensor, idx: Tensor, G: int, off: int, n_onehot: int,
                table: Optional[Tensor] = None) -> Optional[Tensor]:
    """``mlp(x)`` with the first layer's one-hot columns gathered; None when the MLP layout or the layer
    width is not covered (the caller runs ``mlp(x)``).  ``table``: the transposed one-hot columns, when the
    caller made them (``head_table``)."""
    sp = mlp_split(mlp)
    if sp is None or not ops._native(x) or x.dtype != torch.float32:
        return None
    lin, ln, rest = sp
    if not layer_supported(lin, n_onehot):
        return None
    need_grad = torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in mlp.parameters()))
    if need_grad:
        h = first_layer(x, idx, G, off, lin, ln, n_onehot, table=table)
    else:
        lead = x.shape[:-1]
        h = gather_first_layer(x.reshape(-1, x.shape[-1]), idx.reshape(-1, idx.shape[-1]), G, off, lin, ln,
                               n_onehot, table=table).view(*lead, lin.out_features)
    for m in rest:
        h = m(h)
    return h
