"""Recorded MLP trunks: run an ``[Linear -> LayerNorm(+act)] * L`` stack step by step inside a rollout,
keep every step's activations in ``[R, M, N]`` slabs, and back-propagate through ALL R steps later as
one batch of ``R*M`` rows.

Why (DreamerV3 discrete imagination, reference ``dreamer_v3.py:235-301``): the reference runs the actor
on each imagined latent during the H=15 rollout (to pick the next action) and then AGAIN over the
stacked trajectories ``[H+1, B*T, latent]`` to build the policy loss - the same weights on the same
inputs.  Recording the rollout's forward (pre-LayerNorm GEMM outputs, row statistics, activations)
removes the second forward entirely (~35 GFLOP, 3 GEMMs + 2 LayerNorms at the Atari-100k shapes); the
backward is the usual per-layer chain at ``M = (H+1)*B*T`` rows: ``ln_act_bwd`` (HIP), ``dW = dpre^T x``
and ``dx = dpre W`` (library GEMMs), bias gradients by the column-sum kernel.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
from torch import Tensor, nn

from sheeprl_prey_amd import ops


def trunk_layers(mlp: nn.Module) -> Optional[List[Tuple[nn.Linear, nn.Module]]]:
    """``[(Linear, fused LayerNorm)]`` of an MLP built as ``[Linear, LayerNorm(act), Identity] * L``
    (``models.MLP`` after ``fuse_norm_act``); None for any other layout (dropout, no norm, ...)."""
    from sheeprl_prey_amd.utils.model import LayerNorm

    seq = getattr(mlp, "model", mlp)
    if getattr(mlp, "flatten_dim", None) is not None:
        return None
    mods = list(seq)
    if len(mods) % 3:
        return None
    out = []
    for i in range(0, len(mods), 3):
        lin, ln, ident = mods[i : i + 3]
        if not (isinstance(lin, nn.Linear) and type(ln) is LayerNorm and isinstance(ident, nn.Identity)):
            return None
        if len(ln.normalized_shape) != 1 or ln.weight is None or ln.bias is None or ln.normalized_shape[0] != lin.out_features:
            return None
        out.append((lin, ln))
    return out or None


class TrunkRecord:
    """Activation slabs of one recorded rollout: ``rows`` steps of ``M`` rows through ``layers``."""

    def __init__(self, layers: Sequence[Tuple[nn.Linear, nn.Module]], rows: int, M: int, device) -> None:
        self.layers = list(layers)
        self.R, self.M = rows, M
        self.pre = [torch.empty(rows, M, lin.out_features, device=device) for lin, _ in self.layers]
        self.y = [torch.empty(rows, M, lin.out_features, device=device) for lin, _ in self.layers]
        self.mean = [torch.empty(rows, M, device=device) for _ in self.layers]
        self.rstd = [torch.empty(rows, M, device=device) for _ in self.layers]
        self.inp: Optional[Tensor] = None  # [R, M, K0] (may be a row-strided view)
        # (idx [R, M, >= G], G, off, n_onehot) when the first layer's leading inputs are one-hots (gathered
        # forward): its weight gradient then scatters those columns instead of multiplying them (ops.wgrad)
        self.onehot = None

    @torch.no_grad()
    def step(self, t: int, x: Tensor, gather=None, tail=None, tail_tn=None) -> Optional[Tensor]:
        """Forward of step ``t`` on ``x`` [M, K0] (row stride allowed); returns the trunk output [M, N].
        ``gather`` = (idx, G, off, n_onehot, table[, Y]): the first ``n_onehot`` input columns are one-hot with hot
        columns ``idx - off`` - the first layer is then a GEMM over the dense columns (or ``Y``, that product
        precomputed by the caller) plus a row gather of ``table`` (its transposed one-hot weight columns) with the
        LayerNorm fused (``ops/onehot.py``).
        ``tail`` = (head Linear, uniforms [M], unimix, sample_out, idx_out, idx_off): the last LayerNorm, the head
        and the unimix one-hot sample run as one kernel (``csrc/actor_tail.hip``); returns None when it did (the
        sample is in ``sample_out``), else the trunk output as without ``tail``.
        ``tail_tn`` = (head Linear, uniforms [M, A], init_std, min_std, pre_out, loc, scale, sample_out): the continuous
        form - the last LayerNorm, the head and the truncated-normal sample as one kernel
        (``csrc/truncnorm.hip`` head_linear_sample_fwd); None when it did."""
        C = ops._ext()
        M = self.M
        for i, (lin, ln) in enumerate(self.layers):
            pre = self.pre[i][t]
            if i == 0 and gather is not None:
                from sheeprl_prey_amd.ops.onehot import gather_first_layer

                idx, G, off, n1, table = gather[:5]
                gather_first_layer(x, idx, G, off, lin, ln, n1, table=table, y_out=self.y[0][t], z_out=pre,
                                   mean=self.mean[0][t], rstd=self.rstd[0][t], Y=gather[5] if len(gather) > 5 else None)
                x = self.y[0][t]
                continue
            if lin.bias is not None:
                torch.addmm(lin.bias, x, lin.weight.t(), out=pre)
            else:
                torch.mm(x, lin.weight.t(), out=pre)
            N = pre.shape[-1]
            if tail is not None and i == len(self.layers) - 1:
                # the last LayerNorm + the actor head + the unimix sample as one launch (csrc/actor_tail.hip)
                head, uni, alpha, sample_out, idx_out, ioff = tail
                if C.actor_tail(pre, self.y[i][t], ln.weight, ln.bias, self.mean[i][t], self.rstd[i][t], float(ln.eps),
                                ops._act_code(ln.act), head.weight, head.bias, uni, float(alpha), sample_out, idx_out,
                                int(ioff)):
                    return None
            if tail_tn is not None and i == len(self.layers) - 1:
                head, u, init_std, min_std, pre_out, loc, scale, sample_out = tail_tn
                if C.tn_head_linear_sample_fwd(pre, head.weight, head.bias, u, float(init_std), float(min_std), -1.0, 1.0,
                                               pre_out, loc, scale, sample_out, ln_w=ln.weight, ln_b=ln.bias,
                                               ln_eps=float(ln.eps), act=ops._act_code(ln.act), y_out=self.y[i][t],
                                               mean=self.mean[i][t], rstd=self.rstd[i][t]):
                    return None
            C.ln_act_fwd_into(pre, N, self.y[i][t], N, ln.weight, ln.bias, self.mean[i][t], self.rstd[i][t], M, N, 1,
                              float(ln.eps), ops._act_code(ln.act))
            x = self.y[i][t]
        return x

    def backward(self, dy: Tensor) -> List[Optional[Tensor]]:
        """Parameter gradients ``[W, b, gamma, beta] * L`` (None where not required) of the recorded
        trunk for the output gradient ``dy`` [R, M, N] (``self.inp`` must hold the trunk inputs)."""
        C = ops._ext()
        RM = self.R * self.M
        L = len(self.layers)
        grads: List[Optional[Tensor]] = [None] * (4 * L)
        dy = dy.reshape(RM, -1)
        if dy.stride(-1) != 1 or dy.stride(0) != dy.shape[-1]:
            dy = dy.contiguous()
        for i in reversed(range(L)):
            lin, ln = self.layers[i]
            N = lin.out_features
            pre = self.pre[i].view(RM, N)
            dpre, dg, db = C.ln_act_bwd(pre, dy, ln.weight, ln.bias, self.mean[i].view(RM), self.rstd[i].view(RM),
                                        ops._act_code(ln.act))
            x = self.y[i - 1].view(RM, -1) if i > 0 else self.inp.reshape(RM, self.inp.shape[-1])
            want_b = lin.bias is not None and lin.bias.requires_grad
            if lin.weight.requires_grad and ops.wgrad_ok(dpre):
                oh = self.onehot if i == 0 else None
                if oh is not None and x.shape[1] > oh[3] and ops.wgrad_onehot_ok(dpre, oh[1], oh[3]):
                    grads[4 * i], grads[4 * i + 1] = ops.wgrad(dpre, x[:, oh[3]:], onehot=oh, bias=want_b)
                else:
                    grads[4 * i], grads[4 * i + 1] = ops.wgrad(dpre, x, bias=want_b)
            else:
                grads[4 * i] = dpre.t().mm(x) if lin.weight.requires_grad else None
                if want_b:
                    grads[4 * i + 1] = C.colsum(dpre)
            grads[4 * i + 2] = dg if ln.weight.requires_grad else None
            grads[4 * i + 3] = db if ln.bias.requires_grad else None
            if i > 0:
                dy = dpre.mm(lin.weight)
        return grads

    def params(self) -> List[Tensor]:
        """The trunk's parameters in ``backward``'s gradient order (a missing bias as an empty tensor)."""
        out = []
        for lin, ln in self.layers:
            out += [lin.weight, lin.bias if lin.bias is not None else _NONE, ln.weight, ln.bias]
        return out

    def output(self, inputs: Tensor) -> Tensor:
        """The recorded trunk output ``[R, M, N]`` as a tensor whose backward runs the batched chain.
        ``inputs`` [R, M, K0]: the rollout's trunk inputs (their gradient is not computed: the DV3
        actor reads detached latents)."""
        self.inp = inputs
        return _RecordedTrunk.apply(self, *self.params())


_NONE = torch.empty(0)


class _RecordedTrunk(torch.autograd.Function):
    @staticmethod
    def forward(ctx, rec: TrunkRecord, *params):
        ctx.rec = rec
        # a fresh alias of the last activation slab: autograd owns the returned tensor's grad_fn
        return rec.y[-1].view_as(rec.y[-1])

    @staticmethod
    def backward(ctx, dy):
        rec: TrunkRecord = ctx.rec
        ctx.rec = None
        return (None, *rec.backward(dy))
