"""Fused ops: HIP kernels on GPU tensors, eager PyTorch on CPU tensors.

GPU tensors ALWAYS go through the compiled extension ``sheeprl_prey_amd/ops/_C*.so``
(built in-tree by ``python setup.py build_ext --inplace`` / ``__graft_entry__.build``); if it is
missing on a GPU box the op raises instead of silently falling back.  ``set_fused(False)``
explicitly routes GPU tensors through the eager reference (for A/B measurements only).
"""
from __future__ import annotations

import importlib
import os
from typing import Optional, Sequence, Tuple

import torch
from torch import Tensor

from sheeprl_prey_amd.ops import reference as ref
from sheeprl_prey_amd.ops.reference import ACTS

_C = None
_LOAD_ERROR: Optional[BaseException] = None
_FUSED = True


def _ext():
    global _C, _LOAD_ERROR
    if _C is None and _LOAD_ERROR is None:
        try:
            _C = importlib.import_module("sheeprl_prey_amd.ops._C")
        except BaseException as e:  # noqa: BLE001
            _LOAD_ERROR = e
    if _C is None:
        raise RuntimeError(
            "sheeprl_prey_amd HIP extension is not built/loadable "
            f"({_LOAD_ERROR!r}). Run `python setup.py build_ext --inplace` (PYTORCH_ROCM_ARCH=gfx950)."
        )
    return _C


def native_available() -> bool:
    try:
        _ext()
        return True
    except RuntimeError:
        return False


def set_fused(flag: bool) -> None:
    global _FUSED
    _FUSED = bool(flag)


def fused_enabled() -> bool:
    """Fused (fp32-only) HIP paths are on - and no CUDA autocast region (``precision=bf16-mixed``)
    is active: under autocast the ops run as eager torch code so they compute in bf16 like the rest."""
    return _FUSED and not torch.is_autocast_enabled("cuda")


def _native(t: Tensor) -> bool:
    if t.is_cuda and fused_enabled():
        _ext()  # loud failure if missing
        return True
    return False


def _act_code(act: str) -> int:
    a = (act or "none").lower()
    if a not in ACTS:
        raise ValueError(f"unsupported fused activation {act}")
    return ACTS[a]


# =============================================================== Linear (library GEMMs, column-sum bias grad)
_LIN2D = True  # row-strided 2-D linear forward (tests toggle it)


def _lin2d(x: Tensor, weight: Tensor, bias: Optional[Tensor]) -> Tensor:
    """``F.linear`` with >2-D inputs flattened to one GEMM when the leading dims fold into a row stride
    (e.g. row-strided views into the imagination buffer): the bias then rides in the GEMM epilogue
    (addmm) instead of a separate broadcast add over the whole output."""
    if x.dim() > 2 and _LIN2D:
        try:
            x2 = x.view(-1, x.shape[-1])
        except RuntimeError:
            return torch.nn.functional.linear(x, weight, bias)
        y = torch.addmm(bias, x2, weight.t()) if bias is not None else x2.mm(weight.t())
        return y.view(*x.shape[:-1], weight.shape[0])
    return torch.nn.functional.linear(x, weight, bias)


# =============================================================== tall-layer weight gradients (wgrad.hip)
WGRAD_MIN_ROWS = 4096  # below this many rows the library GEMM takes the weight gradient (0 disables the kernel)
WGRAD_MAX_TILES = 32  # dense parts with more 128 x 128 output tiles go to the library GEMM


def _rows2d(t: Tensor) -> Tensor:
    """``t`` as a row-strided 2-D [rows, last] view (no copy when the leading dims fold into one stride)."""
    if t.dim() == 2 and t.stride(-1) == 1:
        return t
    try:
        v = t.view(-1, t.shape[-1])
    except RuntimeError:
        v = t.reshape(-1, t.shape[-1])
    return v if v.stride(-1) == 1 else v.contiguous()


def wgrad_ok(dz: Tensor) -> bool:
    """The split-K kernel is used for the weight gradients of layers over >= WGRAD_MIN_ROWS rows (the
    imagination heads: 15-16k rows), where the library GEMM runs its M reduction in a handful of tiles."""
    rows = dz.numel() // max(1, dz.shape[-1])
    return WGRAD_MIN_ROWS > 0 and rows >= WGRAD_MIN_ROWS and _native(dz) and dz.dtype == torch.float32


def wgrad_onehot_ok(dz: Tensor, G: int, n_onehot: int) -> bool:
    """The one-hot scatter covers <= 32 classes per group and 16-byte aligned dZ rows of N % 4 == 0."""
    C = n_onehot // max(1, G)
    return (C * G == n_onehot and C <= 32 and dz.shape[-1] % 4 == 0 and dz.stride(-2) % 4 == 0 and dz.stride(-1) == 1
            and dz.data_ptr() % 16 == 0)


def transpose_many(xs, outs=None):
    """Contiguous transposes of up to 8 fp32 matrices (2-D, unit column stride; column slices of weights are
    fine) in ONE launch (csrc/transpose.hip); ``outs`` optionally names contiguous [cols, rows] destinations
    (None entries allocate).  No autograd: for weight tables the HIP kernels read.  CPU: ``.t().contiguous()``."""
    xs = list(xs)
    if xs[0].is_cuda:
        return _ext().transpose_many(xs, outs)
    res = []
    for j, x in enumerate(xs):
        o = outs[j] if outs is not None and j < len(outs) else None
        if o is None:
            res.append(x.detach().t().contiguous())
        else:
            o.copy_(x.detach().t())
            res.append(o)
    return res


def wgrad(dz: Tensor, x: Optional[Tensor] = None, onehot=None, bias: bool = False, out=None):
    """``(dW, db)`` of a linear layer ``z = [onehot | x] W^T + b`` from ``dz`` = dL/dz over M rows:
    ``dW [N, Kone + Kd] = [onehot | x]^T dz``, ``db = dz.sum(0)`` (None unless ``bias``; needs ``x``).
    ``onehot = (idx, G, off, n_onehot)``: the first ``n_onehot = G*C`` input columns are exact one-hots whose hot
    column is ``idx[m, g] - off`` (idx row-strided int32 [M, >= G]); they are scattered, not multiplied.
    ``out = (dW, db)``: preallocated results (``ops/sidestream.py`` deferral), filled in place where the
    kernel path allows; the caller copies whatever else is returned."""
    dz2 = _rows2d(dz)
    M, N = dz2.shape
    x2 = _rows2d(x) if x is not None else None
    idx2 = None
    G = C = off = 0
    if onehot is not None:
        idx, G, off, n1 = onehot
        idx2 = _rows2d(idx)
        C = n1 // G
    Kd = x2.shape[1] if x2 is not None else 0
    if x2 is not None and ((N + 127) // 128) * ((Kd + 127) // 128) > WGRAD_MAX_TILES:
        # a wide output fills the chip with library tiles (XL: 1024 x 1024 over 16384 rows, hipBLASLt 292 us vs
        # 342 us split-K; 1024 x 4096: 900 vs 1194 us) - the split-K kernel only wins on small N x K
        dense = dz2.t().mm(x2)
        db = _ext().colsum(dz2 if dz2.stride(-1) == 1 else dz2.contiguous()) if bias else None
        if idx2 is None:
            return dense, db
        dWo = torch.empty(N, G * C, device=dz.device, dtype=torch.float32)
        _ext().wgrad(dz2, None, idx2, int(G), int(C), int(off), dWo, None, False)
        return torch.cat((dWo, dense), 1), db
    dW = out[0] if out is not None and out[0] is not None else torch.empty(N, G * C + Kd, device=dz.device, dtype=torch.float32)
    db = None
    if bias:
        db = out[1] if out is not None and out[1] is not None else torch.empty(N, device=dz.device, dtype=torch.float32)
    _ext().wgrad(dz2, x2, idx2, int(G), int(C), int(off), dW, db, False)
    return dW, db


class _Linear(torch.autograd.Function):
    """``F.linear`` whose backward takes the bias gradient with a row-split column-sum kernel
    (``norm.hip: colsum1``): torch's dim-0 sum of a [15360, 255] two-hot head gradient ran 165 us on
    gfx950 and rocBLAS gemv ~68 us; dX / dW are the usual two GEMMs (hipBLASLt); row-strided inputs
    (views into the imagination trajectory buffer) are used in place."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        ctx.params = (weight, bias)  # the leaves a deferred weight gradient is assigned to (ops/sidestream.py)
        return _lin2d(x, weight, bias)

    @staticmethod
    def backward(ctx, gy):
        from sheeprl_prey_amd.ops import sidestream as ss

        x, w = ctx.saved_tensors
        g2 = gy.reshape(-1, gy.shape[-1])
        dx = None
        if ctx.needs_input_grad[0]:
            dx = (g2 @ w).view(*gy.shape[:-1], w.shape[1])
        if ss.active(gy.device) and ctx.needs_input_grad[1]:
            # inside a deferral scope (the world-model backward): the parameter gradients leave the data-gradient
            # chain and run beside the scan backward (ops/sidestream.py)
            meta = (tuple(ctx.needs_input_grad), ctx.has_bias)
            dw, db = ss.param_grads(gy.device, lambda: _Linear._param_grads(meta, g2, x), ctx.params, g2, x)
            return dx, dw, db
        dw, db = _Linear._param_grads((tuple(ctx.needs_input_grad), ctx.has_bias), g2, x)
        return dx, dw, db

    @staticmethod
    def _param_grads(meta, g2, x, out=None):
        needs, has_bias = meta
        dw = db = None
        if needs[1] and wgrad_ok(g2):
            return wgrad(g2, x, bias=has_bias and needs[2], out=out)
        if needs[1]:
            if out is not None and out[0] is not None:
                dw = torch.mm(g2.t(), x.reshape(-1, x.shape[-1]), out=out[0])
            else:
                dw = g2.t() @ x.reshape(-1, x.shape[-1])
        if has_bias and needs[2]:
            db = _ext().colsum(g2 if g2.stride(-1) == 1 else g2.contiguous())
        return dw, db


def linear(x: Tensor, weight: Tensor, bias: Optional[Tensor] = None) -> Tensor:
    if _native(x) and x.dtype == torch.float32 and x.dim() >= 2 and torch.is_grad_enabled():
        return _Linear.apply(x, weight, bias)
    if _native(x) and x.dtype == torch.float32:
        return _lin2d(x, weight, bias)
    return torch.nn.functional.linear(x, weight, bias)


# =============================================================== LayerNorm + activation
class _LNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps, act):
        shape = x.shape
        x2 = x.contiguous().view(-1, shape[-1])
        y, mean, rstd = _ext().ln_act_fwd(x2, weight, bias, eps, act)
        ctx.save_for_backward(x2, weight, bias, mean, rstd)
        ctx.act, ctx.shape = act, shape
        return y.view(shape)

    @staticmethod
    def backward(ctx, dy):
        x2, weight, bias, mean, rstd = ctx.saved_tensors
        dx, dg, db = _ext().ln_act_bwd(x2, dy.contiguous().view_as(x2), weight, bias, mean, rstd, ctx.act)
        return dx.view(ctx.shape), (dg if weight is not None else None), (db if bias is not None else None), None, None


def ln_act(x: Tensor, weight: Optional[Tensor], bias: Optional[Tensor], eps: float = 1e-5, act: str = "none") -> Tensor:
    """``act(LayerNorm(x))`` over the last dim."""
    if _native(x) and x.dtype == torch.float32 and x.shape[-1] <= 12288:
        return _LNAct.apply(x, weight, bias, float(eps), _act_code(act))
    return ref.ln_act(x, weight, bias, eps, act)


class _LNActNCHW(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps, act):
        x = x.contiguous()
        y, mean, rstd = _ext().ln_nchw_fwd(x, weight, bias, eps, act)
        ctx.save_for_backward(x, weight, bias, mean, rstd)
        ctx.act = act
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, bias, mean, rstd = ctx.saved_tensors
        dx, dg, db = _ext().ln_nchw_bwd(x, dy.contiguous(), weight, bias, mean, rstd, ctx.act)
        return dx, (dg if weight is not None else None), (db if bias is not None else None), None, None


def ln_act_nchw(x: Tensor, weight: Optional[Tensor], bias: Optional[Tensor], eps: float = 1e-5, act: str = "none") -> Tensor:
    """``act(LayerNorm over C)`` of an NCHW tensor, without the NHWC round trip."""
    if _native(x) and x.dtype == torch.float32 and x.dim() == 4:
        return _LNActNCHW.apply(x, weight, bias, float(eps), _act_code(act))
    return ref.ln_act_nchw(x, weight, bias, eps, act)


# =============================================================== LayerNorm-GRU epilogue
class _LNGRU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, h, weight, bias, eps):
        H = h.shape[-1]
        x2 = x.contiguous().view(-1, 3 * H)
        h2 = h.contiguous().view(-1, H)
        hn, mean, rstd = _ext().ln_gru_fwd(x2, h2, weight, bias, eps)
        ctx.save_for_backward(x2, h2, weight, bias, mean, rstd)
        ctx.xshape, ctx.hshape = x.shape, h.shape
        return hn.view(h.shape)

    @staticmethod
    def backward(ctx, dhn):
        x2, h2, weight, bias, mean, rstd = ctx.saved_tensors
        dx, dh, dg, db = _ext().ln_gru_bwd(x2, h2, weight, bias, mean, rstd, dhn.contiguous().view_as(h2))
        return dx.view(ctx.xshape), dh.view(ctx.hshape), dg, db, None


def ln_gru(x: Tensor, h: Tensor, weight: Tensor, bias: Tensor, eps: float = 1e-5) -> Tensor:
    """GRU gates of ``LayerNormGRUCell`` applied to the projected input ``x = [h, in] @ W``."""
    if _native(x) and x.dtype == torch.float32 and h.shape[-1] <= 4096:
        return _LNGRU.apply(x, h, weight, bias, float(eps))
    return ref.ln_gru(x, h, weight, bias, eps)


# =============================================================== unimix + straight-through sampling
class _UnimixSample(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, uniform, classes, alpha, sample):
        ctx.set_materialize_grads(False)  # unused outputs: None, not a zero-filled tensor (one fill launch each)
        l2 = logits.contiguous()
        mixed, st = _ext().unimix_sample_fwd(l2, uniform if sample else None, classes, alpha)
        ctx.save_for_backward(l2)
        ctx.classes, ctx.alpha, ctx.sample = classes, alpha, sample
        if not sample:
            ctx.mark_non_differentiable(st)
        return mixed, st

    @staticmethod
    def backward(ctx, g_mixed, g_st):
        (l2,) = ctx.saved_tensors
        gm = g_mixed.contiguous() if g_mixed is not None else None
        gs = g_st.contiguous() if (g_st is not None and ctx.sample) else None
        if gm is None and gs is None:
            return torch.zeros_like(l2), None, None, None, None
        dl = _ext().unimix_sample_bwd(l2, gm, gs, ctx.classes, ctx.alpha)
        return dl, None, None, None, None


def unimix_sample(
    logits: Tensor, classes: int, unimix: float = 0.01, sample: bool = True, uniform: Optional[Tensor] = None,
    forced: Optional[Tensor] = None,
) -> Tuple[Tensor, Tensor]:
    """(mixed logits, one-hot sample with straight-through grads | mode one-hot).

    ``logits[..., G*C]`` holds G categoricals of ``classes`` classes each.  ``forced``: a given one-hot sample
    (teacher forcing of the eager oracle, see ``DreamerV3Trainer.teacher``) - always the eager form."""
    if forced is not None:
        return ref.unimix_sample(logits, classes, unimix, sample=sample, forced=forced)
    if _native(logits) and logits.dtype == torch.float32 and classes <= 1024:
        if sample and uniform is None:
            uniform = torch.rand(logits.numel() // classes, device=logits.device)
        return _UnimixSample.apply(logits, uniform, int(classes), float(unimix), bool(sample))
    return ref.unimix_sample(logits, classes, unimix, uniform=uniform, sample=sample)


# =============================================================== two-hot
_BINS = {}


def twohot_bins(num_bins: int, low: float = -20.0, high: float = 20.0, device=None) -> Tensor:
    key = (num_bins, low, high, str(device))
    if key not in _BINS:
        _BINS[key] = torch.linspace(low, high, num_bins, device=device)
    return _BINS[key]


class _TwoHotNLL(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, bins):
        K = logits.shape[-1]
        l2 = logits.contiguous().view(-1, K)
        y = target.detach().contiguous().view(-1).float()
        loss = _ext().twohot_nll_fwd(l2, y, bins)
        ctx.save_for_backward(l2, y, bins)
        ctx.shape = logits.shape
        return loss.view(logits.shape[:-1])

    @staticmethod
    def backward(ctx, gl):
        l2, y, bins = ctx.saved_tensors
        dl = _ext().twohot_nll_bwd(l2, y, bins, gl.contiguous().view(-1))
        return dl.view(ctx.shape), None, None


def twohot_nll(logits: Tensor, target: Tensor, low: float = -20.0, high: float = 20.0) -> Tensor:
    """``-TwoHotEncodingDistribution(logits, dims=1).log_prob(target)`` with target [..., 1] or [...]."""
    if target.dim() == logits.dim():
        target = target.squeeze(-1)
    bins = twohot_bins(logits.shape[-1], low, high, device=logits.device)
    if _native(logits) and logits.dtype == torch.float32 and logits.shape[-1] <= 512:
        return _TwoHotNLL.apply(logits, target, bins)
    return ref.twohot_nll(logits, target, bins)


class _ValueLoss2(torch.autograd.Function):
    """Critic objective with its logits gradient computed in the forward pass (``csrc/dist.hip`` value_loss2_kernel)."""

    @staticmethod
    def forward(ctx, logits, y1, y2, w, bins):
        loss, dl = _ext().value_loss2(logits.contiguous(), y1.detach().contiguous().float(), y2.detach().contiguous().float(),
                                      w.detach().contiguous().float(), bins)
        ctx.save_for_backward(dl)
        return loss

    @staticmethod
    def backward(ctx, g):
        (dl,) = ctx.saved_tensors
        return dl * g, None, None, None, None


def twohot_value_loss(logits: Tensor, y1: Tensor, y2: Tensor, w: Tensor, low: float = -20.0, high: float = 20.0) -> Tensor:
    """``mean(w * (twohot_nll(logits, y1) + twohot_nll(logits, y2)))`` (DreamerV3 critic loss, reference
    ``dreamer_v3.py:327-336``): one forward pass writing the loss and the logits gradient, one scaling launch backward.
    ``y1``, ``y2``, ``w`` hold one value per logits row (no gradient flows into them)."""
    K = logits.shape[-1]
    R = logits.numel() // K
    bins = twohot_bins(K, low, high, device=logits.device)
    if (_native(logits) and logits.dtype == torch.float32 and K <= 512 and y1.numel() == R and y2.numel() == R
            and w.numel() == R):
        return _ValueLoss2.apply(logits, y1.reshape(-1), y2.reshape(-1), w.reshape(-1), bins)
    lead = logits.shape[:-1]
    nll = twohot_nll(logits, y1.reshape(lead)) + twohot_nll(logits, y2.reshape(lead))
    return torch.mean(nll * w.reshape(lead))


class _TwoHotMean(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, bins):
        K = logits.shape[-1]
        l2 = logits.contiguous().view(-1, K)
        out, s = _ext().twohot_mean_fwd(l2, bins)
        ctx.save_for_backward(l2, bins, s)
        ctx.shape = logits.shape
        return out.view(*logits.shape[:-1], 1)

    @staticmethod
    def backward(ctx, g):
        l2, bins, s = ctx.saved_tensors
        dl = _ext().twohot_mean_bwd(l2, bins, s, g.contiguous().view(-1))
        return dl.view(ctx.shape), None


def twohot_mean(logits: Tensor, low: float = -20.0, high: float = 20.0) -> Tensor:
    """``TwoHotEncodingDistribution(logits, dims=1).mean`` -> [..., 1]."""
    bins = twohot_bins(logits.shape[-1], low, high, device=logits.device)
    if _native(logits) and logits.dtype == torch.float32 and logits.shape[-1] <= 512:
        return _TwoHotMean.apply(logits, bins)
    return ref.twohot_mean(logits, bins).unsqueeze(-1)


# =============================================================== KL balancing
class _KLBalance(torch.autograd.Function):
    @staticmethod
    def forward(ctx, post, prior, groups, classes, dyn, rep, free):
        ctx.set_materialize_grads(False)  # unused outputs: None, not a zero-filled tensor (one fill launch each)
        a = post.contiguous()
        b = prior.contiguous()
        kl, loss, ea, eb = _ext().kl_fwd(a, b, groups, classes, dyn, rep, free)
        ctx.save_for_backward(a, b, kl)
        ctx.cfg = (groups, classes, dyn, rep, free)
        ctx.mark_non_differentiable(kl, ea, eb)
        shape = post.shape[:-1] if post.shape[-1] == groups * classes else post.shape[:-2]
        ctx.shape = post.shape
        return loss.view(shape), kl.view(shape), ea.view(shape), eb.view(shape)

    @staticmethod
    def backward(ctx, gl, _gkl, _gea, _geb):
        if gl is None:
            return None, None, None, None, None, None, None
        a, b, kl = ctx.saved_tensors
        groups, classes, dyn, rep, free = ctx.cfg
        da, db = _ext().kl_bwd(a, b, kl, gl.contiguous().view(-1), groups, classes, dyn, rep, free)
        return da.view(ctx.shape), db.view(ctx.shape), None, None, None, None, None


def kl_balance(
    post_logits: Tensor, prior_logits: Tensor, groups: int, classes: int, dyn: float = 0.5, rep: float = 0.1,
    free_nats: float = 1.0, entropies: Optional[list] = None,
) -> Tuple[Tensor, Tensor]:
    """DreamerV3 KL loss per row: ``dyn*max(KL(sg(post)||prior),free) + rep*max(KL(post||sg(prior)),free)``.
    Returns (loss, kl).  ``entropies`` (a list): receives the per-row summed categorical entropies of the
    posterior and the prior (detached) - on the GPU a by-product of the KL kernel's log-softmaxes."""
    if _native(post_logits) and post_logits.dtype == torch.float32 and classes <= 64:
        loss, kl, ea, eb = _KLBalance.apply(post_logits, prior_logits, int(groups), int(classes), float(dyn), float(rep),
                                            float(free_nats))
        if entropies is not None:
            entropies.extend((ea, eb))
        return loss, kl
    if entropies is not None:
        with torch.no_grad():
            for lg in (post_logits, prior_logits):
                lp = lg.detach().reshape(-1, groups, classes).log_softmax(-1)
                entropies.append(-(lp.exp() * lp).sum((-1, -2)).view(lg.shape[:-1] if lg.shape[-1] == groups * classes
                                                                          else lg.shape[:-2]))
    return ref.kl_balance(post_logits, prior_logits, groups, classes, dyn, rep, free_nats)


# =============================================================== scans
class _Lambda(torch.autograd.Function):
    @staticmethod
    def forward(ctx, r, v, c, lam):
        r2, v2, c2 = r.contiguous(), v.contiguous(), c.contiguous()
        out = _ext().lambda_fwd(r2, v2, c2, lam)
        ctx.save_for_backward(v2, c2, out)
        ctx.lam = lam
        return out

    @staticmethod
    def backward(ctx, g):
        v2, c2, out = ctx.saved_tensors
        dr, dv, dc = _ext().lambda_bwd(v2, c2, out, g.contiguous(), ctx.lam)
        return dr, dv, dc, None


def lambda_returns(rewards: Tensor, values: Tensor, continues: Tensor, lmbda: float = 0.95) -> Tensor:
    """DreamerV3 lambda-values over [H, ...] (reference ``dreamer_v3/utils.py:44-55``)."""
    if _native(rewards) and rewards.dtype == torch.float32:
        return _Lambda.apply(rewards, values, continues, float(lmbda))
    return ref.lambda_returns(rewards, values, continues, lmbda)


@torch.no_grad()
def gae_scan(rewards: Tensor, values: Tensor, dones: Tensor, next_value: Tensor, gamma: float, lam: float):
    """(returns, advantages) for a [T, N, 1] rollout."""
    if _native(rewards):
        ret, adv = _ext().gae(
            rewards.float().contiguous(), values.float().contiguous(), dones.float().contiguous(),
            next_value.float().contiguous().view(-1), float(gamma), float(lam),
        )
        return ret, adv
    return ref.gae(rewards, values, dones, next_value, gamma, lam)


# =============================================================== flat optimiser
_FAULT: dict = {}


def fault_block(device) -> Tensor:
    """The device's fault block, int32 [4]: [0] persistent-scan health (sticky wait-timeout bits),
    [1] replay-gather error, [2] optimiser updates skipped because [0] or [1] was set, [3] unused.
    Kernels write [0] / [1]; the flat optimisers' norm / advance kernels read them and skip the update of
    a faulted step on the device (no host sync); the host reads the block at log time."""
    key = str(torch.device(device))
    b = _FAULT.get(key)
    if b is None:
        b = _FAULT[key] = torch.zeros(4, dtype=torch.int32, device=device)
    return b


def skipped_updates(reset: bool = False) -> int:
    """Optimiser updates skipped on the device because of a recorded kernel fault (syncs)."""
    n = 0
    for b in _FAULT.values():
        n += int(b[2].item())
        if reset:
            b[2].zero_()
    return n


def check_faults() -> None:
    """Host health check shared by every algorithm loop (``algos/common.py:log_throughput``, log time; syncs):
    words 0 / 1 of a device fault block are sticky and make every flat-optimiser update skip, so a fault
    that no algorithm-specific check consumed (DreamerV3 reads and resets them itself first) must not leave
    the run silently frozen - reset the words and raise."""
    bad = []
    for key, b in _FAULT.items():
        w = b[:2].cpu()
        if int(w[0]) | int(w[1]):
            b[:2].zero_()
            bad.append((key, int(w[0]), int(w[1])))
    if bad:
        raise RuntimeError("device fault block set (scan health word, replay-gather error word) on "
                           f"{bad}: the optimiser updates of the affected steps were skipped")


def _guard_tripped(guard: Optional[Tensor]) -> bool:
    if guard is None:
        return False
    if int(guard[0].item()) | int(guard[1].item()):
        guard[2] += 1
        return True
    return False


def flat_grad_norm(grad: Tensor, scalars: Tensor, max_norm: float, guard: Optional[Tensor] = None) -> Tensor:
    if _native(grad):
        return _ext().flat_grad_norm(grad, scalars, float(max_norm), guard)
    norm = torch.linalg.vector_norm(grad)
    coef = torch.ones((), device=grad.device)
    if 0 < max_norm < float("inf"):
        coef = torch.clamp(max_norm / (norm + 1e-6), max=1.0)
    if _guard_tripped(guard):
        scalars[3] = 1.0
        return norm
    scalars[0] += 1
    scalars[1] = coef
    scalars[2] = norm
    scalars[3] = 0.0
    return norm


def flat_advance(scalars: Tensor, guard: Optional[Tensor] = None) -> None:
    if _native(scalars):
        _ext().flat_advance(scalars, guard)
        return
    if _guard_tripped(guard):
        scalars[3] = 1.0
        return
    scalars[0] += 1
    scalars[1] = 1.0
    scalars[3] = 0.0


def flat_adam(p, g, m, v, scalars, lr, b1, b2, eps, wd, decoupled) -> None:
    if _native(p):
        _ext().flat_adam(p, g, m, v, scalars, lr, b1, b2, eps, wd, bool(decoupled))
        return
    if float(scalars[3].item()) != 0.0:
        return
    t = float(scalars[0].item())
    coef = scalars[1]
    grad = g * coef
    if decoupled:
        p.mul_(1 - lr * wd)
    elif wd:
        grad = grad.add(p, alpha=wd)
    m.lerp_(grad, 1 - b1)
    v.mul_(b2).addcmul_(grad, grad, value=1 - b2)
    bc1 = 1 - b1**t
    bc2s = (1 - b2**t) ** 0.5
    denom = (v.sqrt() / bc2s).add_(eps)
    p.addcdiv_(m, denom, value=-lr / bc1)


__all__ = [
    "ln_act", "ln_act_nchw", "ln_gru", "unimix_sample", "twohot_nll", "twohot_mean", "twohot_bins", "kl_balance",
    "lambda_returns", "twohot_value_loss", "gae_scan", "flat_grad_norm", "flat_advance", "flat_adam", "fault_block", "skipped_updates", "check_faults", "native_available", "set_fused",
]


# =============================================================== tanh-squashed Gaussian (SAC actors)
class _SquashedGaussian(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mean, log_std, eps, scale, bias, mode, lo, hi):
        ctx.set_materialize_grads(False)  # unused outputs: None, not a zero-filled tensor (one fill launch each)
        m, r, e = mean.contiguous(), log_std.contiguous(), eps.contiguous()
        action, logp = _ext().squashed_gaussian_fwd(m, r, e, scale, bias, mode, lo, hi)
        ctx.save_for_backward(m, r, e, scale)
        ctx.cfg = (mode, lo, hi)
        return action, logp

    @staticmethod
    def backward(ctx, ga, glp):
        if ga is None and glp is None:
            return (None,) * 8
        m, r, e, scale = ctx.saved_tensors
        dmean, draw = _ext().squashed_gaussian_bwd(
            m, r, e, scale, ga.contiguous() if ga is not None else None,
            glp.contiguous() if glp is not None else None, *ctx.cfg)
        return dmean, draw, None, None, None, None, None, None


def squashed_gaussian(mean: Tensor, log_std: Tensor, scale: Tensor, bias: Tensor, mode: int = 0, lo: float = -5.0,
                      hi: float = 2.0, eps: Optional[Tensor] = None) -> Tuple[Tensor, Tensor]:
    """Reparameterised tanh-squashed Gaussian sample and its log-prob (SAC Eq. 26).

    ``mode=0``: ``log_std`` clamped to [lo, hi] (SAC/DroQ); ``mode=1``: tanh-rescaled into [lo, hi]
    (SAC-AE).  Returns (action [..., A], logp [..., 1])."""
    if eps is None:
        eps = torch.randn_like(mean)
    A = mean.shape[-1]
    if _native(mean) and mean.dtype == torch.float32 and A <= 64:
        return _SquashedGaussian.apply(mean, log_std, eps, scale.float().contiguous(), bias.float().contiguous(),
                                       int(mode), float(lo), float(hi))
    return ref.squashed_gaussian(mean, log_std, eps, scale, bias, mode, lo, hi)


# =============================================================== truncated normal (DreamerV2/V3 continuous actors)
class _TruncNormRsample(torch.autograd.Function):
    @staticmethod
    def forward(ctx, loc, scale, lo, hi, u):
        x = _ext().truncnorm_rsample_fwd(loc, scale, lo, hi, u)
        ctx.save_for_backward(loc, scale, lo, hi, u)
        return x

    @staticmethod
    def backward(ctx, gx):
        gl, gs = _ext().truncnorm_rsample_bwd(*ctx.saved_tensors, gx.contiguous())
        return gl, gs, None, None, None


class _TruncNormLogProb(torch.autograd.Function):
    @staticmethod
    def forward(ctx, value, loc, scale, lo, hi):
        lp = _ext().truncnorm_logprob_fwd(value, loc, scale, lo, hi)
        ctx.save_for_backward(value, loc, scale, lo, hi)
        return lp

    @staticmethod
    def backward(ctx, g):
        value, loc, scale, lo, hi = ctx.saved_tensors
        gv, gl, gs = _ext().truncnorm_logprob_bwd(value, loc, scale, lo, hi, g.contiguous())
        lead = value.numel() // loc.numel()  # broadcast over leading sample dimensions
        return gv, gl.view(lead, *loc.shape).sum(0), gs.view(lead, *loc.shape).sum(0), None, None


def _tn_bound(b: Tensor, like: Tensor) -> Tensor:
    return b.reshape(1).float() if b.numel() == 1 else b.expand_as(like).float().contiguous()


def _tn_native(loc: Tensor, lo: Tensor, hi: Tensor) -> bool:
    return (_native(loc) and loc.dtype == torch.float32 and not lo.requires_grad and not hi.requires_grad
            and lo.device == loc.device and hi.device == loc.device)


def truncnorm_rsample(loc: Tensor, scale: Tensor, lo: Tensor, hi: Tensor, u: Tensor) -> Tensor:
    """Reparameterised truncated-normal sample for uniforms ``u`` (one fused launch forward and backward
    on GPU; ``loc``, ``scale``, ``u`` share one shape, bounds are scalars or that shape)."""
    if _tn_native(loc, lo, hi) and loc.shape == scale.shape == u.shape:
        return _TruncNormRsample.apply(loc.contiguous(), scale.contiguous(), _tn_bound(lo, loc), _tn_bound(hi, loc),
                                       u.contiguous())
    return ref.truncnorm_rsample(loc, scale, lo, hi, u)


def truncnorm_log_prob(value: Tensor, loc: Tensor, scale: Tensor, lo: Tensor, hi: Tensor) -> Tensor:
    """Truncated-normal log-density; ``value`` is ``[sample..., *loc.shape]``."""
    if (_tn_native(loc, lo, hi) and loc.shape == scale.shape and value.dtype == torch.float32
            and value.shape[value.dim() - loc.dim():] == loc.shape):
        return _TruncNormLogProb.apply(value.contiguous(), loc.contiguous(), scale.contiguous(), _tn_bound(lo, loc),
                                       _tn_bound(hi, loc))
    return ref.truncnorm_log_prob(value, loc, scale, lo, hi)


# =============================================================== DreamerV3 discrete actor objective
class _ActorLossDiscrete(torch.autograd.Function):
    """``csrc/actor_loss.hip``: the loss and its gradient w.r.t. the mixed logits in one pass."""

    @staticmethod
    def forward(ctx, z, actions, lam, base, disc, offset, invscale, heads, ent_coef):
        loss, dz = _ext().actor_loss_discrete(z.contiguous(), actions.contiguous(), lam.contiguous(), base.contiguous(),
                                              disc.contiguous(), offset.reshape(1).contiguous(),
                                              invscale.reshape(1).contiguous(), list(heads), float(ent_coef))
        ctx.save_for_backward(dz)
        return loss

    @staticmethod
    def backward(ctx, g):
        (dz,) = ctx.saved_tensors
        return dz * g, None, None, None, None, None, None, None, None


def actor_loss_discrete(z: Tensor, actions: Tensor, lam: Tensor, base: Tensor, disc: Tensor, offset: Tensor,
                        invscale: Tensor, heads, ent_coef: float) -> Optional[Tensor]:
    """DreamerV3 discrete policy loss (reference ``dreamer_v3.py:258-301``) from the per-head mixed
    logits ``z`` [T, M, A]; None when the fused kernel does not apply (the caller keeps the eager form)."""
    if not (_native(z) and z.dim() == 3
            and all(t.dtype == torch.float32 for t in (z, actions, lam, base, disc, offset, invscale))):
        return None
    return _ActorLossDiscrete.apply(z, actions.detach(), lam.detach(), base.detach(), disc.detach(), offset.detach(),
                                    invscale.detach(), tuple(int(h) for h in heads), float(ent_coef))


# =============================================================== DreamerV3 continuous actor objective
class _ActorLossCont(torch.autograd.Function):
    """``csrc/actor_loss.hip`` actor_loss_cont_kernel: the loss and its gradients w.r.t. the head outputs, the
    lambda returns and the baseline in one pass (packed); the backward scales them by the upstream scalar."""

    @staticmethod
    def forward(ctx, pre, lam, base, disc, offset, invscale, ent_coef, init_std, min_std):
        loss, g = _ext().actor_loss_cont(pre.contiguous(), lam.contiguous(), base.contiguous(), disc.contiguous(),
                                         offset.reshape(1).contiguous(), invscale.reshape(1).contiguous(), float(ent_coef),
                                         float(init_std), float(min_std), -1.0, 1.0)
        ctx.save_for_backward(g)
        ctx.shapes = (pre.shape, lam.shape, base.shape)
        return loss

    @staticmethod
    def backward(ctx, gl):
        (g,) = ctx.saved_tensors
        sp, sl, sb = ctx.shapes
        gs = g * gl
        n0, n1 = sp.numel(), sl.numel()
        return (gs[:n0].view(sp), gs[n0:n0 + n1].view(sl), gs[n0 + n1:].view(sb), None, None, None, None, None, None)


def actor_loss_cont(pre: Tensor, lam: Tensor, base: Tensor, disc: Tensor, offset: Tensor, invscale: Tensor,
                    ent_coef: float, init_std: float, min_std: float) -> Optional[Tensor]:
    """DreamerV3 continuous (trunc-normal, bounds [-1, 1]) policy loss (reference ``dreamer_v3.py:258-301``) from the
    actor head outputs ``pre`` [T, M, 2A]: ``-mean_{t<T-1} disc (advantage + ent_coef H)`` with the closed-form
    truncated-normal entropy; one launch forward (+ a fixed-order sum), one backward.  None when the kernel does
    not apply (the caller keeps the eager distribution objective)."""
    if not (_native(pre) and pre.dim() == 3 and pre.shape[-1] % 2 == 0
            and all(t.dtype == torch.float32 for t in (pre, lam, base, disc, offset, invscale))):
        return None
    return _ActorLossCont.apply(pre, lam, base, disc.detach(), offset.detach(), invscale.detach(), float(ent_coef),
                                float(init_std), float(min_std))


# =============================================================== skinny weight-streaming GEMM
def skinny_ok(A: Tensor, W: Tensor) -> bool:
    """Shape/alignment gate of ``skinny_nt`` (M <= 16 rows, K % 128, N % 128, 16-byte strides)."""
    if not (_native(A) and A.dtype == torch.float32 and W.dtype == torch.float32 and A.dim() in (2, 3)
            and W.dim() == A.dim() and A.stride(-1) == 1 and W.stride(-1) == 1):
        return False
    M, K = A.shape[-2:]
    N = W.shape[-2]
    if not (1 <= M <= 16 and K % 128 == 0 and N % 128 == 0 and W.shape[-1] == K):
        return False
    strides = [A.stride(-2), W.stride(-2)] + ([A.stride(0), W.stride(0)] if A.dim() == 3 else [])
    return all(s % 4 == 0 for s in strides) and A.data_ptr() % 16 == 0 and W.data_ptr() % 16 == 0


def skinny_nt(A: Tensor, W: Tensor, out: Tensor, add: Optional[Tensor] = None) -> bool:
    """``out = A @ W^T (+ add)`` for a few activation rows against a large weight (``csrc/skinny.hip``:
    split-K weight streaming at HBM rate).  Batched when A / W / out are 3-D.  Returns False (nothing
    done) when the shapes are outside the kernel's gate - the caller keeps its library GEMM."""
    if not skinny_ok(A, W) or out.stride(-1) != 1 or out.data_ptr() % 16 or out.stride(-2) % 4:
        return False
    if add is not None and (add.stride(-1) != 1 or add.data_ptr() % 16 or (add.shape[-2] > 1 and add.stride(-2) % 4)):
        return False
    C = _ext()
    Z = A.shape[0] if A.dim() == 3 else 1
    need = C.skinny_workspace(W.shape[-2], A.shape[-1], Z)
    part = torch.empty(need, device=A.device, dtype=torch.float32) if need else None
    C.skinny_nt(A, W, out, add, part)
    return True


# Workspace of the one-launch column sums (LayerNorm parameter / bias gradients, csrc/norm.hip colsum_t_kernel):
# without it they run as a zero kernel + an atomic reduction (two launches, order-dependent float sums).  One per
# process, on the device it trains on (Runner sets it up before any step is captured).
_reduce_ws: dict = {}


def init_reduce_workspace(device, floats: int = 1 << 22, counters: int = 1 << 16) -> bool:
    if not (torch.cuda.is_available() and native_available()) or torch.cuda.is_current_stream_capturing():
        return False
    device = torch.device(device)
    if device.type != "cuda":
        return False
    if device.index is None:
        device = torch.device("cuda", torch.cuda.current_device())
    with torch.cuda.device(device):
        if device.index in _reduce_ws:  # one per device for the process: captured graphs keep its addresses
            ws, cnt = _reduce_ws[device.index]
        else:
            ws = torch.empty(floats, device=device, dtype=torch.float32)
            cnt = torch.zeros(counters, device=device, dtype=torch.int32)
            _reduce_ws[device.index] = (ws, cnt)  # never freed: a graph captured with it may replay at any time
        _ext().set_colsum_workspace(ws, cnt)
    return True


# =============================================================== P2E disagreement (K20)
def ensemble_disagreement(hidden: Tensor, weight: Tensor, bias: Optional[Tensor] = None) -> Tensor:
    """``mean_c var_i (hidden_i W_i^T + b_i)[m, c]`` per row (unbiased variance over the ``n`` members):
    the Plan2Explore intrinsic reward before its multiplier (reference ``p2e_dv2/p2e_dv2.py`` /
    ``p2e_dv1/p2e_dv1.py``).  ``hidden`` [n, M, H], ``weight`` [n, O, H], ``bias`` [n, O] -> [M].
    On the GPU the member head GEMMs and the variance are one kernel (``csrc/ensemble.hip``): the
    [n, M, O] predictions are never materialised."""
    n, M, H = hidden.shape
    if (_native(hidden) and hidden.dtype == torch.float32 and weight.dtype == torch.float32 and H % 4 == 0
            and n <= 64 and (bias is None or bias.dtype == torch.float32)):
        part = _ext().ens_disagreement(hidden.contiguous(), weight.contiguous(),
                                       bias.contiguous() if bias is not None else None)
        return part.sum(0) / weight.shape[1]
    wt = weight.transpose(1, 2)
    pred = torch.baddbmm(bias.unsqueeze(1), hidden, wt) if bias is not None else torch.bmm(hidden, wt)
    return pred.var(0).mean(-1)


# =============================================================== SAC twin-Q target (K15)
def sac_twin_q_target(ens, obs: Tensor, act: Tensor, logp: Tensor, rewards: Tensor, dones: Tensor, log_alpha: Tensor,
                      gamma: float) -> Optional[Tensor]:
    """``r + (1 - d) * gamma * (min_c Q'_c(s', a') - alpha * logp)`` for an ``EnsembleMLP`` target critic
    (2 ReLU hidden layers, scalar head, no dropout / LayerNorm) in one kernel (``csrc/sac_target.hip``).
    None when the critic or the tensors are outside the kernel's gate (the caller keeps the eager path)."""
    if not (_native(obs) and obs.dtype == torch.float32 and act.dtype == torch.float32 and obs.dim() == 2):
        return None
    if ens.norms is not None or (ens.dropout > 0 and ens.training) or ens.act_name != "relu" or len(ens.layers) != 2:
        return None
    if ens.head is None or ens.head.out_features != 1 or ens.layers[0].bias is None or ens.layers[1].bias is None:
        return None
    H = ens.layers[0].out_features
    if not (1 <= ens.n <= 4 and H % 128 == 0 and H <= 512 and ens.layers[1].out_features == H
            and obs.shape[1] + act.shape[1] <= 1024):
        return None
    l1, l2, hd = ens.layers[0], ens.layers[1], ens.head
    return _ext().sac_twin_q_target(obs.contiguous(), act.contiguous(), logp.reshape(-1).contiguous(),
                                    rewards.reshape(-1).contiguous().float(), dones.reshape(-1).contiguous().float(),
                                    log_alpha.detach().reshape(-1), l1.weight.detach(), l1.bias.detach(),
                                    l2.weight.detach(), l2.bias.detach(), hd.weight.detach(), hd.bias.detach(), float(gamma))


class _SACCriticLoss(torch.autograd.Function):
    """``csrc/sac_critic.hip``: forward + loss + data backward in one launch, weight gradients in one."""

    @staticmethod
    def forward(ctx, obs, act, y, W1, b1, W2, b2, W3, b3):
        ctx.set_materialize_grads(False)  # unused outputs: None, not a zero-filled tensor (one fill launch each)
        lossp, q, *saved = _ext().sac_critic_fwd(obs, act, y, W1, b1, W2, b2, W3, b3)
        ctx.save_for_backward(*saved)
        ctx.IN = W1.shape[2]
        ctx.mark_non_differentiable(q)
        return lossp.sum(), q

    @staticmethod
    def backward(ctx, g, _gq):
        if g is None:
            return (None,) * 9
        grads = _ext().sac_critic_wgrad(*ctx.saved_tensors, g.reshape(1).contiguous(), ctx.IN)
        return (None, None, None, *grads)


def sac_critic_loss(ens, obs: Tensor, act: Tensor, y: Tensor) -> Optional[Tuple[Tensor, Tensor]]:
    """(``sum_c mean_b (Q_c(s, a) - y)^2``, q [B, n]) for an ``EnsembleMLP`` critic (2 ReLU hidden layers,
    scalar head, no dropout / LayerNorm) as two kernels (K15, ``csrc/sac_critic.hip``) whose backward gives
    every critic parameter's gradient; None outside the kernels' gate (the caller keeps the eager path)."""
    if not (_native(obs) and obs.dtype == torch.float32 and act.dtype == torch.float32 and obs.dim() == 2):
        return None
    if ens.norms is not None or (ens.dropout > 0 and ens.training) or ens.act_name != "relu" or len(ens.layers) != 2:
        return None
    if ens.head is None or ens.head.out_features != 1 or ens.layers[0].bias is None or ens.layers[1].bias is None:
        return None
    H = ens.layers[0].out_features
    if not (1 <= ens.n <= 8 and H % 128 == 0 and H <= 512 and ens.layers[1].out_features == H
            and obs.shape[1] + act.shape[1] <= 1024):
        return None
    l1, l2, hd = ens.layers[0], ens.layers[1], ens.head
    return _SACCriticLoss.apply(obs.contiguous(), act.contiguous(), y.detach().reshape(-1).contiguous().float(), l1.weight,
                                l1.bias, l2.weight, l2.bias, hd.weight, hd.bias)


# =============================================================== DreamerV3 observation loss (K6)
class _ObsMSE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, rec, tgt, rows, scale, symlog):
        ctx.save_for_backward(rec, tgt)
        ctx.cfg = (rows, scale, symlog)
        return _ext().obs_mse_fwd(rec, tgt, rows, scale, symlog)

    @staticmethod
    def backward(ctx, g):
        rec, tgt = ctx.saved_tensors
        rows, scale, symlog = ctx.cfg
        return _ext().obs_mse_bwd(rec, tgt, rows, scale, symlog, g.contiguous()), None, None, None, None


def obs_mse(rec: Tensor, target: Tensor, scale: float = 1.0, symlog: bool = False) -> Tensor:
    """Per-(t, b) observation loss summed over the trailing dims of ``rec`` [T, B, ...] (K6):
    ``sum (rec - target * scale)^2`` for image keys (``target`` may be the raw uint8 frames), or the
    DreamerV3 symlog MSE with the ``d < 1e-8 -> 0`` rule for vector keys (reference
    ``dreamer_v3.py:186-196``).  One fused kernel each way on GPU; eager torch otherwise."""
    T, B = rec.shape[:2]
    n = rec[0, 0].numel()
    if (_native(rec) and rec.dtype == torch.float32 and target.dtype in (torch.uint8, torch.float32)
            and n % 4 == 0 and target.numel() == rec.numel()):
        return _ObsMSE.apply(rec.contiguous(), target.contiguous(), T * B, float(scale), int(bool(symlog))).view(T, B)
    tgt = target.float() * scale if target.dtype == torch.uint8 or scale != 1.0 else target
    dims = tuple(range(2, rec.dim()))
    if symlog:
        d = (rec - torch.sign(tgt) * torch.log1p(tgt.abs())) ** 2
        d = torch.where(d < 1e-8, torch.zeros_like(d), d)
        return d.sum(dim=dims)
    return ((rec - tgt) ** 2).sum(dim=dims)


def symlog_cat(xs: Sequence[Tensor]) -> Tensor:
    """``cat([symlog(x) for x in xs], -1)`` (the DreamerV3 vector encoder's input, reference
    ``dreamer_v3/agent.py`` MLPEncoder): one launch on GPU for inputs that need no gradient; eager torch otherwise."""
    xs = list(xs)
    if (xs and len(xs) <= 8 and _native(xs[0]) and all(x.dtype == torch.float32 and x.is_cuda and not x.requires_grad
                                                        for x in xs)):
        return _ext().symlog_cat([x.contiguous() for x in xs])
    from sheeprl_prey_amd.utils.utils import symlog

    return torch.cat([symlog(x) for x in xs], -1)


def imag_discount(continue_logits: Tensor, dones: Tensor, gamma: float, skip_first: bool = False):
    """``(c[1:] * gamma, cumprod(c * gamma) / gamma)`` with ``c_0 = 1 - done`` and ``c_t = [logit_t > 0]``
    (reference ``dreamer_v3.py:262-279``), one kernel on GPU; shapes [T, M, 1] / [T+1, M, 1].  ``skip_first``:
    ``continue_logits`` holds only the rows 1.. (row 0 is replaced by ``1 - done``, so it need not be computed)."""
    if _native(continue_logits) and continue_logits.dtype == torch.float32 and dones.dtype == torch.float32:
        cg, disc = _ext().imag_discount(continue_logits.detach().contiguous(), dones.reshape(-1).contiguous(), float(gamma),
                                        bool(skip_first))
        return cg, disc
    c = (continue_logits > 0).to(continue_logits.dtype)
    c = torch.cat(((1 - dones).reshape(1, -1, 1).to(c.dtype), c if skip_first else c[1:]))
    return c[1:] * gamma, torch.cumprod(c * gamma, dim=0) / gamma


# =============================================================== persistent LSTM (K18)
class _LSTMSeq(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, h0, c0, W_ih, W_hh, b_ih, b_hh):
        ctx.set_materialize_grads(False)  # unused outputs: None, not a zero-filled tensor (one fill launch each)
        T, B, D = x.shape
        H = W_hh.shape[1]
        C = _ext()
        bias = b_ih + b_hh if b_ih is not None else None
        x2 = x.reshape(T * B, D)
        xg = (torch.addmm(bias, x2, W_ih.t()) if bias is not None else x2.mm(W_ih.t())).view(T, B, 4 * H)
        h0c, c0c = h0.reshape(B, H).contiguous(), c0.reshape(B, H).contiguous()
        Whh = W_hh.contiguous()
        out, gates, cs, hT, cT = C.lstm_fwd(xg, Whh, h0c, c0c)
        ctx.save_for_backward(x, h0c, c0c, W_ih, Whh, out, gates, cs)
        ctx.has_bias = bias is not None
        return out, hT.unsqueeze(0), cT.unsqueeze(0)

    @staticmethod
    def backward(ctx, dout, dhT, dcT):
        x, h0, c0, W_ih, Whh, out, gates, cs = ctx.saved_tensors
        T, B, D = x.shape
        H = Whh.shape[1]
        dout = dout.contiguous() if dout is not None else torch.zeros_like(out)
        dg, dh0, dc0 = _ext().lstm_bwd(Whh, c0, gates, cs, dout, dhT.reshape(B, H).contiguous() if dhT is not None else None,
                                       dcT.reshape(B, H).contiguous() if dcT is not None else None)
        dg2 = dg.reshape(T * B, 4 * H)
        h_prev = torch.cat((h0.unsqueeze(0), out[:-1]), 0).reshape(T * B, H)
        dW_hh = dg2.t().mm(h_prev)
        dW_ih = dg2.t().mm(x.reshape(T * B, D))
        dx = dg2.mm(W_ih).view(T, B, D)
        db = dg2.sum(0) if ctx.has_bias else None
        return dx, dh0.unsqueeze(0), dc0.unsqueeze(0), dW_ih, dW_hh, db, db


def lstm_supported(lstm: torch.nn.LSTM, x: Tensor) -> bool:
    return (_native(x) and x.dtype == torch.float32 and x.dim() == 3 and lstm.num_layers == 1 and not lstm.batch_first
            and not lstm.bidirectional and getattr(lstm, "proj_size", 0) == 0 and lstm.hidden_size % 16 == 0
            and lstm.hidden_size <= 64 and (lstm.dropout == 0 or not lstm.training))


def lstm_seq(lstm: torch.nn.LSTM, x: Tensor, states):
    """``nn.LSTM`` (1 layer, seq-first) over the whole sequence as one persistent launch each way
    (``csrc/lstm.hip``); same outputs and gradients as the module (reference ppo_recurrent/agent.py:60-73)."""
    h0, c0 = states
    return_ = _LSTMSeq.apply(x, h0, c0, lstm.weight_ih_l0, lstm.weight_hh_l0, lstm.bias_ih_l0 if lstm.bias else None,
                             lstm.bias_hh_l0 if lstm.bias else None)
    out, hT, cT = return_
    return out, (hT, cT)


# =============================================================== plain GRU cell (K19)
class _GRUCellAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gi, gh, h):
        hn, rzn = _ext().gru_cell_fwd(gi, gh, h)
        ctx.save_for_backward(gh, h, rzn)
        return hn

    @staticmethod
    def backward(ctx, g):
        gh, h, rzn = ctx.saved_tensors
        return tuple(_ext().gru_cell_bwd(gh, h, rzn, g.contiguous()))


def gru_step(rnn: torch.nn.GRU, x: Tensor, h: Tensor):
    """One step of a 1-layer ``nn.GRU`` (``x`` [1, B, D] or [B, D], ``h`` [1, B, H]) with the gate math
    fused in one kernel each way (``csrc/gru_cell.hip``) and the two input/recurrent projections as
    library GEMMs; returns ``(out, h')`` like the module.  Falls back to the module off the GPU."""
    single_step = x.dim() == 3 and x.shape[0] == 1
    if not (single_step and _native(x) and x.dtype == torch.float32 and rnn.num_layers == 1 and not rnn.batch_first
            and not rnn.bidirectional and rnn.bias):
        return rnn(x, h)
    x2 = x.reshape(-1, x.shape[-1])
    h2 = h.reshape(-1, rnn.hidden_size)
    gi = torch.nn.functional.linear(x2, rnn.weight_ih_l0, rnn.bias_ih_l0).contiguous()
    gh = torch.nn.functional.linear(h2, rnn.weight_hh_l0, rnn.bias_hh_l0).contiguous()
    hn = _GRUCellAct.apply(gi, gh, h2.contiguous()).view(1, -1, rnn.hidden_size)
    return hn, hn
