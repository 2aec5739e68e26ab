"""Fused DreamerV3 posterior scan (forward + BPTT) for GPU tensors.

The reference runs ``rssm.dynamic`` T=64 times under autograd (``dreamer_v3.py:122-129``): every
step re-records ~20 kernels, and the backward adds a small-M weight-gradient GEMM plus a gradient
accumulation add per weight per step.  Here one autograd node owns the whole scan:

forward, per step (9 launches):
  mask(h,z | is_first) -> x = z'Wz^T + a_proj[t] -> LN+SiLU (written into the [h', feat] buffer)
  -> gx = [h', feat] Wg^T -> LN-GRU gates -> u = h [Wt1; Wr1]^T + P[t] (prior|posterior first layers
  as ONE GEMM) -> grouped LN+SiLU (two parameter sets, group-major output) -> two second-layer GEMMs as
  one batched GEMM -> unimix + straight-through sample for prior and posterior in one kernel.
backward, per step (9 launches): the adjoint chain only (activation gradients);
after the loop every weight gradient is ONE large GEMM over the stacked T*B rows and every LayerNorm
parameter gradient ONE column reduction over per-step partial slots.

Large recurrent states (XL, deter 4096: ~300 MB of weights per step for 16 rows) route every per-step
GEMM by size (``_nt``): ``skinny.hip`` split-K streaming for the smaller weights, the library's NT
kernels for the GRU weight, with transposed weight copies for the adjoint GEMMs.

The step-invariant work (action half of the recurrent input layer, embedding half of the posterior
layer) is hoisted by the caller (``RSSM.scan_dynamic``) and enters as ``a_proj`` / ``P`` inputs, so
autograd handles their (large, efficient) GEMM backward.
"""
from __future__ import annotations

import os
from typing import Tuple

import torch
from torch import Tensor

from sheeprl_prey_amd.ops import sidestream
from sheeprl_prey_amd.ops.reference import ACTS


def _use_skinny(B: int, H: int) -> bool:
    """Large recurrent states (XL: deter 4096): the per-step GEMMs take a weight-streaming route."""
    return B <= 16 and H >= 1024


# Measured on MI355X (scripts/skinny_sweep.py, 16 rows): hipBLASLt's NT kernels stream the big GRU
# weight at ~6.4 TB/s (16x12288x5120: 39 us) against 4.5 TB/s for skinny.hip, while skinny.hip wins
# below ~16 M weights (16x2048x4096: 13.8 us vs 17.7 us).  Route by size; the adjoint GEMMs use a
# transposed weight copy so they also run in the fast NT layout (16x5120x12288 A.W: 76 -> 42 us).
_SKINNY_MAX_WEIGHTS = 16 * 1024 * 1024


def _nt(A: Tensor, W: Tensor, out: Tensor, add: Tensor = None) -> None:
    """out = A @ W^T (+ add) for few rows against a large row-major weight W."""
    from sheeprl_prey_amd.ops import skinny_nt

    if W.shape[-2] * W.shape[-1] <= _SKINNY_MAX_WEIGHTS and skinny_nt(A, W, out, add):
        return
    Wt = W.transpose(-1, -2)
    if A.dim() == 3:
        if add is None:
            torch.bmm(A, Wt, out=out)
        else:
            torch.baddbmm(add, A, Wt, out=out)
    elif add is None:
        torch.mm(A, Wt, out=out)
    elif add.data_ptr() == out.data_ptr():
        out.addmm_(A, Wt)
    else:
        torch.addmm(add, A, Wt, out=out)


class RSSMScanFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a_proj, P, is_first, uniform, z0, Wz, ln1_w, ln1_b, Wg, lng_w, lng_b, W1, ln2_w, ln2_b, W2, b2, meta):
        ctx.set_materialize_grads(False)  # unused outputs: None, not a zero-filled tensor (one fill launch each)
        from sheeprl_prey_amd.ops import _ext

        C = _ext()
        T, B, D = a_proj.shape
        S = Wz.shape[1]
        H = lng_w.shape[0] // 3
        hid = W1.shape[0] // 2
        disc, alpha, eps1, epsg, eps2, act1, act2 = meta
        dev, f32 = a_proj.device, torch.float32
        HD = H + D
        first = is_first.reshape(T, B).contiguous()
        cat = torch.empty(T, B, HD, device=dev, dtype=f32)
        zm = torch.empty(T, B, S, device=dev, dtype=f32)
        xr = torch.empty(T, B, D, device=dev, dtype=f32)
        m1 = torch.empty(T, B, device=dev, dtype=f32)
        r1 = torch.empty(T, B, device=dev, dtype=f32)
        gx = torch.empty(T, B, 3 * H, device=dev, dtype=f32)
        mg = torch.empty(T, B, device=dev, dtype=f32)
        rg = torch.empty(T, B, device=dev, dtype=f32)
        hs = torch.empty(T, B, H, device=dev, dtype=f32)
        u = torch.empty(T, B, 2 * hid, device=dev, dtype=f32)
        v = torch.empty(T, 2, B, hid, device=dev, dtype=f32)
        m2 = torch.empty(T, 2 * B, device=dev, dtype=f32)
        r2 = torch.empty(T, 2 * B, device=dev, dtype=f32)
        logits = torch.empty(T, 2, B, S, device=dev, dtype=f32)
        mixed = torch.empty(T, 2, B, S, device=dev, dtype=f32)
        samples = torch.empty(T, 2, B, S, device=dev, dtype=f32)
        Wz_t, Wg_t, W1_t, W2_t = Wz.t(), Wg.t(), W1.t(), W2.transpose(1, 2)
        # XL shapes: split-K weight streaming instead of the library's skinny GEMMs (False -> library)
        sk = _use_skinny(B, H)
        Wzc = Wz.contiguous() if sk else None
        h_prev = None
        z_prev = None
        for t in range(T):
            C.rssm_mask_fwd(h_prev, H, z_prev, first[t], z0, cat[t], HD, zm[t], B, H, S)
            if sk:
                _nt(zm[t], Wzc, xr[t], a_proj[t])
            else:
                torch.addmm(a_proj[t], zm[t], Wz_t, out=xr[t])
            C.ln_act_fwd_into(xr[t], D, cat[t, :, H:], HD, ln1_w, ln1_b, m1[t], r1[t], B, D, 1, eps1, act1)
            if sk:
                _nt(cat[t], Wg, gx[t])
            else:
                torch.mm(cat[t], Wg_t, out=gx[t])
            C.ln_gru_fwd_into(gx[t], cat[t], HD, lng_w, lng_b, hs[t], mg[t], rg[t], B, H, epsg)
            if sk:
                _nt(hs[t], W1, u[t], P[t])
            else:
                torch.addmm(P[t], hs[t], W1_t, out=u[t])
            C.ln_act_fwd_into(u[t], hid, v[t], hid, ln2_w, ln2_b, m2[t], r2[t], 2 * B, hid, 2, eps2, act2)
            if sk:
                _nt(v[t], W2, logits[t], b2)
            else:
                torch.baddbmm(b2, v[t], W2_t, out=logits[t])
            C.unimix_sample_fwd_into(logits[t], uniform[t], mixed[t], samples[t], disc, alpha)
            h_prev = hs[t]
            z_prev = samples[t, 1]
        ctx.save_for_backward(first, Wz, ln1_w, ln1_b, Wg, lng_w, lng_b, W1, ln2_w, ln2_b, W2,
                              cat, zm, xr, m1, r1, gx, mg, rg, hs, u, v, m2, r2, logits)
        ctx.meta = meta
        ctx.dims = (T, B, D, S, H, hid)
        post = samples[:, 1].contiguous()
        return hs, post, mixed[:, 1].contiguous(), mixed[:, 0].contiguous()

    @staticmethod
    def backward(ctx, d_hs, d_post, d_post_mixed, d_prior_mixed):
        from sheeprl_prey_amd.ops import _ext

        C = _ext()
        (first, Wz, ln1_w, ln1_b, Wg, lng_w, lng_b, W1, ln2_w, ln2_b, W2,
         cat, zm, xr, m1, r1, gx, mg, rg, hs, u, v, m2, r2, logits) = ctx.saved_tensors
        disc, alpha, eps1, epsg, eps2, act1, act2 = ctx.meta
        T, B, D, S, H, hid = ctx.dims
        dev, f32 = hs.device, torch.float32
        HD = H + D
        DH = d_hs.clone() if d_hs is not None else torch.zeros(T, B, H, device=dev, dtype=f32)
        DH = DH.contiguous()
        dsamp = torch.zeros(T, 2, B, S, device=dev, dtype=f32)
        if d_post is not None:
            dsamp[:, 1].copy_(d_post)
        dmixed = torch.zeros(T, 2, B, S, device=dev, dtype=f32)
        if d_prior_mixed is not None:
            dmixed[:, 0].copy_(d_prior_mixed)
        if d_post_mixed is not None:
            dmixed[:, 1].copy_(d_post_mixed)
        dlog = torch.empty(T, 2, B, S, device=dev, dtype=f32)
        dv = torch.empty(T, 2, B, hid, device=dev, dtype=f32)
        du = torch.empty(T, B, 2 * hid, device=dev, dtype=f32)
        dgx = torch.empty(T, B, 3 * H, device=dev, dtype=f32)
        dx = torch.empty(T, B, D, device=dev, dtype=f32)
        dcat = torch.empty(B, HD, device=dev, dtype=f32)
        dhp = torch.empty(B, H, device=dev, dtype=f32)
        dzp = torch.empty(B, S, device=dev, dtype=f32)
        g1 = C.ln_bwd_grid(B, D, 1)
        g2 = C.ln_bwd_grid(2 * B, hid, 2)
        gg = C.ln_gru_bwd_grid(B)
        p1g = torch.empty(T, g1, D, device=dev, dtype=f32)
        p1b = torch.empty_like(p1g)
        p2g = torch.empty(T, g2 * 2, hid, device=dev, dtype=f32)
        p2b = torch.empty_like(p2g)
        pgg = torch.empty(T, gg, 3 * H, device=dev, dtype=f32)
        pgb = torch.empty_like(pgg)
        sidestream.flush(dev, inline=True)
        sk = _use_skinny(B, H)
        if sk:  # the adjoint GEMMs stream W^T: one transposed copy of each weight per backward
            WzT, WgT, W1T, W2T = (Wz.t().contiguous(), Wg.t().contiguous(), W1.t().contiguous(),
                                  W2.transpose(1, 2).contiguous())
        for t in range(T - 1, -1, -1):
            C.unimix_sample_bwd_into(logits[t], dmixed[t], dsamp[t], dlog[t], disc, alpha)
            if sk:
                _nt(dlog[t], W2T, dv[t])
            else:
                torch.bmm(dlog[t], W2, out=dv[t])
            C.ln_act_bwd_into(u[t], hid, dv[t], hid, du[t], hid, ln2_w, ln2_b, m2[t], r2[t], p2g[t], p2b[t], None, None,
                              2 * B, hid, 2, act2)
            if sk:
                _nt(du[t], W1T, DH[t], DH[t])
            else:
                DH[t].addmm_(du[t], W1)
            C.ln_gru_bwd_into(gx[t], cat[t], HD, lng_w, lng_b, mg[t], rg[t], DH[t], dgx[t], dhp, pgg[t], pgb[t], None, None,
                              B, H)
            if sk:
                _nt(dgx[t], WgT, dcat)
            else:
                torch.mm(dgx[t], Wg, out=dcat)
            C.ln_act_bwd_into(xr[t], D, dcat[:, H:], HD, dx[t], D, ln1_w, ln1_b, m1[t], r1[t], p1g[t], p1b[t], None, None,
                              B, D, 1, act1)
            if t > 0:
                if sk:
                    _nt(dx[t], WzT, dzp)
                else:
                    torch.mm(dx[t], Wz, out=dzp)
                C.rssm_mask_bwd(dhp, H, dcat, HD, dzp, first[t], DH[t - 1], dsamp[t - 1, 1], B, H, S)
        TB = T * B
        # ---- batched weight gradients: one GEMM / one reduction each
        dWz = dx.reshape(TB, D).t().mm(zm.reshape(TB, S))
        dWg = dgx.reshape(TB, 3 * H).t().mm(cat.reshape(TB, HD))
        dW1 = du.reshape(TB, 2 * hid).t().mm(hs.reshape(TB, H))
        dlog_g = dlog.transpose(0, 1).reshape(2, TB, S)
        v_g = v.transpose(0, 1).reshape(2, TB, hid)
        dW2 = torch.bmm(dlog_g.transpose(1, 2), v_g)
        db2 = dlog_g.sum(1, keepdim=True)
        dln1_w = torch.empty_like(ln1_w)
        dln1_b = torch.empty_like(ln1_b)
        C.colsum2(p1g, p1b, dln1_w, dln1_b, T * g1, D, 1)
        dlng_w = torch.empty_like(lng_w)
        dlng_b = torch.empty_like(lng_b)
        C.colsum2(pgg, pgb, dlng_w, dlng_b, T * gg, 3 * H, 1)
        dln2_w = torch.empty_like(ln2_w)
        dln2_b = torch.empty_like(ln2_b)
        C.colsum2(p2g, p2b, dln2_w, dln2_b, T * g2 * 2, hid, 2)
        return (dx, du, None, None, None, dWz, dln1_w, dln1_b, dWg, dlng_w, dlng_b, dW1, dln2_w, dln2_b, dW2, db2, None)


class RSSMScan4Fn(torch.autograd.Function):
    """Same contract as :class:`RSSMScanFn`, 4 + 4 launches per step (``csrc/rssm_scan.hip``):
    every launch is a 16-row MFMA GEMM whose prologue rebuilds its A operand from the previous
    launch's raw output (LN, LN-GRU, masking, their adjoints) and whose epilogue holds the bias /
    unimix sample / unimix adjoint.  Requires batch <= 16, classes dividing 32 (see
    :func:`scan4_supported`).  Buffers are group-major ([2, T, B, S]) so the prior half of the
    categorical adjoint is one launch for all steps."""

    @staticmethod
    def forward(ctx, a_proj, P, is_first, uniform, z0, Wz, ln1_w, ln1_b, Wg, lng_w, lng_b, W1, ln2_w, ln2_b, W2, b2, meta):
        ctx.set_materialize_grads(False)  # unused outputs: None, not a zero-filled tensor (one fill launch each)
        from sheeprl_prey_amd.ops import _ext

        C = _ext()
        T, B, D = a_proj.shape
        S = Wz.shape[1]
        H = lng_w.shape[0] // 3
        hid = W1.shape[0] // 2
        disc, alpha, eps1, epsg, eps2, act1, act2 = meta
        dev, f32 = a_proj.device, torch.float32
        e = lambda *shape: torch.empty(*shape, device=dev, dtype=f32)  # noqa: E731
        first = is_first.reshape(T, B).contiguous()
        Wz_c = Wz.contiguous()
        fwd = [a_proj, P, first, uniform.contiguous(), z0, Wz_c, ln1_w.contiguous(), ln1_b.contiguous(), Wg.contiguous(),
               lng_w.contiguous(), lng_b.contiguous(), W1.contiguous(), ln2_w.contiguous(), ln2_b.contiguous(),
               W2.contiguous(), b2.reshape(2, S).contiguous(),
               e(T, B, H + D), e(T, B, S), e(T, B, D), e(T, B), e(T, B), e(T, B, 3 * H), e(T, B), e(T, B), e(T, B, H),
               e(T, B, 2 * hid), e(2, T, B, hid), e(T, 2 * B), e(T, 2 * B), e(2, T, B, S), e(2, T, B, S), e(2, T, B, S)]
        dims = [T, B, S, D, H, hid, disc, act1, act2]
        fl = [alpha, eps1, epsg, eps2]
        WzT = Wz_c.t().contiguous()
        c0 = torch.mv(Wz_c, z0.reshape(-1))  # recurrent input of a reset row
        sel = torch.empty(T, 16, S // disc, device=dev, dtype=torch.int32)  # F4 -> FX selected WzT rows
        C.scan4_fwd(fwd, dims, fl, WzT, c0, sel)
        ctx.save_for_backward(*fwd[:32], WzT)
        ctx.dims, ctx.fl = dims, fl
        hs, mixed, samples = fwd[24], fwd[30], fwd[31]
        return hs, samples[1], mixed[1], mixed[0]

    @staticmethod
    def backward(ctx, d_hs, d_post, d_post_mixed, d_prior_mixed):
        from sheeprl_prey_amd.ops import _ext

        C = _ext()
        fwd = list(ctx.saved_tensors)
        WzT = fwd.pop()
        T, B, S, D, H, hid = ctx.dims[:6]
        dev, f32 = fwd[0].device, torch.float32
        e = lambda *shape: torch.empty(*shape, device=dev, dtype=f32)  # noqa: E731
        Wz, Wg, W1, W2 = fwd[5], fwd[8], fwd[11], fwd[14]
        dmixed = torch.zeros(2, T, B, S, device=dev, dtype=f32)
        if d_prior_mixed is not None:
            dmixed[0].copy_(d_prior_mixed)
        if d_post_mixed is not None:
            dmixed[1].copy_(d_post_mixed)
        DH = d_hs.contiguous().clone() if d_hs is not None else torch.zeros(T, B, H, device=dev, dtype=f32)
        dpost = d_post.contiguous() if d_post is not None else torch.empty(0, device=dev, dtype=f32)
        dlog, dv, du, dgx, dx = e(2, T, B, S), e(2, T, B, hid), e(T, B, 2 * hid), e(T, B, 3 * H), e(T, B, D)
        p1g, p1b, pgg, pgb, p2g, p2b = e(T, D), e(T, D), e(T, 3 * H), e(T, 3 * H), e(T, 2 * hid), e(T, 2 * hid)
        bwd = [WzT, Wg.t().contiguous(), W1.t().contiguous(), W2.transpose(1, 2).contiguous(), dpost,
               dmixed, DH, dlog, dv, du, dgx, dx, e(B, H + D), e(B, H), p1g, p1b, pgg, pgb, p2g, p2b]
        fork = sidestream.fork_point(dev)
        C.scan4_bwd(fwd + bwd, ctx.dims, ctx.fl)
        sidestream.flush(dev, fork=fork)
        cat, zm, hs, v = fwd[16], fwd[17], fwd[24], fwd[26]
        TB = T * B
        dWz = dx.reshape(TB, D).t().mm(zm.reshape(TB, S))
        dWg = dgx.reshape(TB, 3 * H).t().mm(cat.reshape(TB, H + D))
        dW1 = du.reshape(TB, 2 * hid).t().mm(hs.reshape(TB, H))
        dlog_g = dlog.reshape(2, TB, S)
        dW2 = torch.bmm(dlog_g.transpose(1, 2), v.reshape(2, TB, hid))
        db2 = dlog_g.sum(1, keepdim=True)
        return (dx, du, None, None, None, dWz, p1g.sum(0), p1b.sum(0), dWg, pgg.sum(0), pgb.sum(0), dW1,
                p2g.sum(0).view(2, hid), p2b.sum(0).view(2, hid), dW2, db2, None)


class RSSMPersistFn(torch.autograd.Function):
    """Posterior path of the scan as ONE persistent launch forward and ONE backward
    (``csrc/rssm_persist.hip``): every workgroup keeps its weight tile in registers for all T steps
    and the GEMM -> LayerNorm seams are in-launch hand-offs (write-through stores + arrival
    counters).  ``W1`` is the h-half of the representation input layer [hid, H], ``ln2_*`` / ``W2`` /
    ``b2`` the representation head, ``P`` its embedding projection (+ bias), ``uniform`` [T, B*S/C].
    Returns recurrent states, posterior samples and posterior unimix logits; the prior head runs
    batched on the returned states (``fused_scan``)."""

    @staticmethod
    def forward(ctx, a_proj, P, is_first, uniform, z0, Wz, ln1_w, ln1_b, Wg, lng_w, lng_b, W1, ln2_w, ln2_b, W2, b2, meta):
        ctx.set_materialize_grads(False)  # unused outputs: None, not a zero-filled tensor (one fill launch each)
        from sheeprl_prey_amd.ops import _ext

        C = _ext()
        T, B, D = a_proj.shape
        S = Wz.shape[1]
        H = lng_w.shape[0] // 3
        hid = W1.shape[0]
        disc, alpha, eps1, epsg, eps2, act1, act2 = meta
        dev, f32 = a_proj.device, torch.float32
        e = lambda *shape: torch.empty(*shape, device=dev, dtype=f32)  # noqa: E731
        first = is_first.reshape(T, B).contiguous()
        Wz_c = Wz.contiguous()
        z0 = z0.reshape(-1).contiguous()
        # recurrent input before the posterior gathers: action part + z0 Wz^T of reset rows
        xr = torch.addcmul(a_proj, first.unsqueeze(-1), torch.mv(Wz_c, z0))
        zm = e(T, B, S)
        torch.mul(first[0].unsqueeze(-1), z0, out=zm[0])
        ok, words, _, _, _ = C.scanp_info(B, S, D, H, hid, disc)
        assert ok, "scanp: unsupported shape"
        sync = torch.empty(words, device=dev, dtype=torch.int32)
        _scan_health_word(dev)
        # every transposed weight the scan needs (forward Wz^T; backward W2^T, W1^T, Wg^T) in one launch
        from sheeprl_prey_amd.ops import transpose_many

        train = any(ctx.needs_input_grad)
        W2c, W1c, Wgc = W2.contiguous(), W1.contiguous(), Wg.contiguous()
        trs = transpose_many([Wz_c, W2c, W1c, Wgc] if train else [Wz_c])
        fwd = [P.contiguous(), first, uniform.contiguous(), z0, Wz_c, trs[0], ln1_w.contiguous(),
               ln1_b.contiguous(), Wgc, lng_w.contiguous(), lng_b.contiguous(), W1c,
               ln2_w.contiguous(), ln2_b.contiguous(), W2c, b2.contiguous(),
               xr, e(T, B, H + D), zm, e(T, B), e(T, B), e(T, B, 3 * H), e(T, 3 * H // 16, 16, 2), e(T, B), e(T, B),
               e(T, B, H), e(T, B, hid), e(T, B, hid), e(T, B), e(T, B), e(T, B, S), e(T, B, S), e(T, B, S),
               torch.empty(T, B, S // disc, device=dev, dtype=torch.int32), sync]
        dims = [T, B, S, D, H, hid, disc, act1, act2]
        fl = [alpha, eps1, epsg, eps2]
        C.scanp_fwd(fwd, dims, fl)
        ctx.save_for_backward(*fwd, *trs[1:])
        ctx.dims, ctx.fl = dims, fl
        hs, mixed, samples = fwd[25], fwd[31], fwd[32]
        return hs, samples, mixed

    @staticmethod
    def backward(ctx, d_hs, d_post, d_post_mixed):
        from sheeprl_prey_amd.ops import _ext

        C = _ext()
        saved = list(ctx.saved_tensors)
        fwd, (W2T, W1T, WgT) = saved[:-3], saved[-3:]
        T, B, S, D, H, hid, disc = ctx.dims[:7]
        alpha = ctx.fl[0]
        dev, f32 = fwd[0].device, torch.float32
        e = lambda *shape: torch.empty(*shape, device=dev, dtype=f32)  # noqa: E731
        Wz, Wg, W1, W2 = fwd[4], fwd[8], fwd[11], fwd[14]
        logits = fwd[30]
        dmixed = d_post_mixed.contiguous() if d_post_mixed is not None else torch.zeros(T, B, S, device=dev, dtype=f32)
        DH = d_hs.contiguous().clone() if d_hs is not None else torch.zeros(T, B, H, device=dev, dtype=f32)
        dpost = d_post.contiguous() if d_post is not None else torch.empty(0, device=dev, dtype=f32)
        dlog = e(T, B, S)
        # the last step's categorical adjoint has no recurrent term: one launch before the scan
        C.unimix_sample_bwd_into(logits[T - 1], dmixed[T - 1], dpost[T - 1] if d_post is not None else None, dlog[T - 1],
                                 disc, alpha)
        dv, du, dgx, dcat, dx = e(T, B, hid), e(T, B, hid), e(T, B, 3 * H), e(T, B, H + D), e(T, B, D)
        # the six LayerNorm parameter partials as column slices of one buffer: one column sum for all of them
        widths = (D, D, 3 * H, 3 * H, hid, hid)
        lnp = e(T, sum(widths))
        p1g, p1b, pgg, pgb, p2g, p2b = torch.split(lnp, widths, dim=1)
        bwd = [W2T, W1T, WgT, dpost, dmixed, DH, dlog, dv, du, dgx, dcat,
               dx, p1g, p1b, pgg, pgb, p2g, p2b, e(T, B, 3 * H), e(T, H // 16, 16, 2)]
        _scan_health_word(dev)
        fork = sidestream.fork_point(dev)
        C.scanp_bwd(fwd + bwd, ctx.dims, ctx.fl)
        # the queued decoder / head parameter gradients run beside the scan backward (ops/sidestream.py)
        sidestream.flush(dev, fork=fork)
        cat, zm, hs, v = fwd[17], fwd[18], fwd[25], fwd[27]
        TB = T * B
        dWz = dx.reshape(TB, D).t().mm(zm.reshape(TB, S))
        dWg = dgx.reshape(TB, 3 * H).t().mm(cat.reshape(TB, H + D))
        dW1 = du.reshape(TB, hid).t().mm(hs.reshape(TB, H))
        dlog2 = dlog.reshape(TB, S)
        dW2 = dlog2.t().mm(v.reshape(TB, hid))
        db2 = dlog2.sum(0)
        g1w, g1b, ggw, ggb, g2w, g2b = torch.split(lnp.sum(0), widths)
        return (dx, du, None, None, None, dWz, g1w, g1b, dWg, ggw, ggb, dW1, g2w, g2b, dW2, db2, None)


def scanp_error(sync: Tensor) -> int:
    """Error word of a persistent-scan launch (0 = every hand-off completed; else the waiter's code)."""
    from sheeprl_prey_amd.ops import _ext

    return int(sync[_ext().scanp_info(1, 32, 16, 16, 16, 32)[2]].item())


# ---------------------------------------------------------------- persistent-scan health
# Every hand-off wait of the persistent scan is bounded; a wait that times out (a starved / not
# co-resident workgroup) makes the whole grid drain and or-s ``1 << code`` into this sticky device word,
# which every launch shares.  The host reads it off the hot path (log / checkpoint time, end of a bench)
# and raises, so a starved scan can never silently produce garbage gradients.
SCAN_WAIT_CODES = {
    1: "fwd A waits h_{t-1} (B; ag form: every A' h tile)", 2: "fwd A waits x_{t} (C gathers)",
    3: "fwd B waits gx (A; ag form: every A' h tile)", 4: "fwd C waits u (B)", 5: "fwd C waits every C sample",
    6: "fwd A' waits every A' row-statistics partial (ag form)", 11: "bwd G1 waits dlog (G4)", 12: "bwd G2 waits dv (G1)", 13: "bwd G3 waits dZ (G2)",
    14: "bwd G4 waits dcat (G3)",
}
_HEALTH: dict = {}
_SPIN_MAX = 0  # 0 = kernel default; tests force tiny bounds to exercise the timeout path


def _scan_health_word(device) -> Tensor:
    from sheeprl_prey_amd.ops import _ext

    from sheeprl_prey_amd.ops import fault_block

    key = str(device)
    w = _HEALTH.get(key)
    if w is None:
        # word 0 of the device's fault block: the flat optimisers skip the update of a step that set it
        w = _HEALTH[key] = fault_block(device)[0:1]
    _ext().set_scanp_health(w, _SPIN_MAX)
    return w


def set_scan_spin_max(n: int) -> None:
    """Debug: bound every persistent-scan hand-off wait to ``n`` polls (0 = the kernel default)."""
    global _SPIN_MAX
    _SPIN_MAX = int(n)
    for w in _HEALTH.values():
        from sheeprl_prey_amd.ops import _ext

        _ext().set_scanp_health(w, _SPIN_MAX)


def check_scan_health(raise_error: bool = True) -> int:
    """Host check of the sticky persistent-scan health word (syncs the device).  Returns the bit mask of
    the wait codes that timed out since the last check (0 = healthy) and raises when it is non-zero."""
    bad = 0
    for w in _HEALTH.values():
        v = int(w.item())
        if v:
            w.zero_()
            bad |= v
    if bad and raise_error:
        names = [f"{c}: {n}" for c, n in SCAN_WAIT_CODES.items() if bad & (1 << c)]
        raise RuntimeError("persistent RSSM scan: a hand-off wait timed out (workgroups starved or not co-resident); "
                           f"the affected steps' outputs are invalid. Timed-out waits: {names or hex(bad)}. "
                           "SRL_SCAN_IMPL=scan4 selects the multi-launch scan.")
    return bad


def scanp_supported(B: int, S: int, D: int, H: int, hid: int, classes: int) -> bool:
    """Shape gate of the persistent scan (register tiles, LDS, one resident workgroup per CU)."""
    from sheeprl_prey_amd.ops import _ext

    return bool(_ext().scanp_info(B, S, D, H, hid, classes)[0])


def scan4_supported(B: int, S: int, D: int, H: int, hid: int, classes: int) -> bool:
    """Shape gate of the 4-launch scan: 16-row tiles, 16/32-column tiles, whole categorical groups
    per 32-column tile, every A operand fits the 160 KiB LDS of one workgroup."""
    if not (1 <= B <= 16 and S % 32 == 0 and D % 16 == 0 and H % 16 == 0 and hid % 16 == 0 and H <= 512):
        return False
    if not (1 <= classes <= 32 and 32 % classes == 0):
        return False
    from sheeprl_prey_amd.ops import _ext

    return int(_ext().scan4_lds(S, D, H, hid)) <= 160 * 1024


def fused_scan_supported(rssm) -> bool:
    """The fused scan covers the DreamerV3 RSSM layout: LN+act MLPs, LN-GRU, equal prior/posterior widths."""
    import torch.nn as nn

    from sheeprl_prey_amd.utils.model import LayerNorm

    try:
        rec = rssm.recurrent_model.mlp.model
        tr = rssm.transition_model.model
        rep = rssm.representation_model.model
        gru = rssm.recurrent_model.rnn
    except AttributeError:
        return False
    ok = (
        len(rec) == 3 and isinstance(rec[1], LayerNorm) and rec[1].act in ACTS and rec[0].bias is None
        and len(tr) == 4 and isinstance(tr[1], LayerNorm) and len(rep) == 4 and isinstance(rep[1], LayerNorm)
        and tr[1].act == rep[1].act and tr[1].eps == rep[1].eps
        and tr[0].out_features == rep[0].out_features and tr[0].bias is not None and rep[0].bias is not None
        and isinstance(gru.layer_norm, nn.LayerNorm) and gru.linear.bias is None
        and rssm.discrete <= 64 and gru.hidden_size <= 4096 and rec[0].out_features <= 2048 and tr[0].out_features <= 2048
    )
    return bool(ok)


class _SplitCols(torch.autograd.Function):
    """``W[:, :k], W[:, k:]`` whose backward assembles the full-weight gradient with ONE concatenation
    (autograd's slice backward zero-fills the full weight for each part, copies the part in and adds
    the two: five launches per split weight per step)."""

    @staticmethod
    def forward(ctx, W: Tensor, k: int):
        ctx.set_materialize_grads(False)  # unused outputs: None, not a zero-filled tensor (one fill launch each)
        ctx.k, ctx.n, ctx.m = k, W.shape[0], W.shape[1]
        return W[:, :k], W[:, k:]

    @staticmethod
    def backward(ctx, g1, g2):
        k, n, m = ctx.k, ctx.n, ctx.m
        ref = g1 if g1 is not None else g2
        if g1 is None:
            g1 = torch.zeros(n, k, device=ref.device, dtype=ref.dtype)
        if g2 is None:
            g2 = torch.zeros(n, m - k, device=ref.device, dtype=ref.dtype)
        return torch.cat((g1, g2), 1), None


def _split_cols(W: Tensor, k: int):
    if W.requires_grad and torch.is_grad_enabled():
        return _SplitCols.apply(W, k)
    return W[:, :k], W[:, k:]


def fused_scan(rssm, embedded_obs: Tensor, actions: Tensor, is_first: Tensor, z0: Tensor,
               uniform: Tensor = None) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """Returns recurrent_states [T,B,H], posteriors [T,B,S], posteriors_logits [T,B,S], priors_logits [T,B,S]."""
    T, B = embedded_obs.shape[:2]
    rec = rssm.recurrent_model.mlp.model
    gru = rssm.recurrent_model.rnn
    tr = rssm.transition_model.model
    rep = rssm.representation_model.model
    H = gru.hidden_size
    S = tr[3].out_features
    rec_lin = rec[0]
    Wz, Wa = _split_cols(rec_lin.weight, S)
    a_proj = torch.nn.functional.linear(torch.addcmul(actions, is_first, actions, value=-1.0), Wa)  # (1 - first) a
    Wh_rep, We = _split_cols(rep[0].weight, H)
    e_proj = torch.nn.functional.linear(embedded_obs, We, rep[0].bias)
    hid = tr[0].out_features
    meta = (rssm.discrete, float(rssm.unimix), float(rec[1].eps), float(gru.layer_norm.eps), float(tr[1].eps),
            ACTS[rec[1].act], ACTS[tr[1].act])
    impl = getattr(rssm, "scan_impl", os.environ.get("SRL_SCAN_IMPL", "persist"))
    nseg = S // rssm.discrete
    if impl == "persist" and scanp_supported(B, S, rec_lin.out_features, H, hid, rssm.discrete):
        # posterior path in one persistent launch; the prior head is off the recurrence: batched
        uni_post = uniform.view(T, 2, B * nseg)[:, 1] if uniform is not None else torch.rand(
            T, B * nseg, device=embedded_obs.device)
        hs, post, post_mixed = RSSMPersistFn.apply(
            a_proj.contiguous(), e_proj.contiguous(), is_first.contiguous(), uni_post.contiguous(), z0.reshape(-1).contiguous(),
            Wz, rec[1].weight, rec[1].bias, gru.linear.weight, gru.layer_norm.weight, gru.layer_norm.bias,
            Wh_rep, rep[1].weight, rep[1].bias, rep[3].weight, rep[3].bias, meta)
        prior_mixed = rssm._uniform_mix_fused(rssm.transition_model(hs))
        return hs, post, post_mixed, prior_mixed
    if uniform is None:
        uniform = torch.rand(T, 2 * B * nseg, device=embedded_obs.device)
    P = torch.cat((tr[0].bias.expand(T, B, hid), e_proj), -1)
    W1 = torch.cat((tr[0].weight, Wh_rep), 0)
    ln2_w = torch.stack((tr[1].weight, rep[1].weight))
    ln2_b = torch.stack((tr[1].bias, rep[1].bias))
    W2 = torch.stack((tr[3].weight, rep[3].weight))
    b2 = torch.stack((tr[3].bias, rep[3].bias)).unsqueeze(1)
    fn = RSSMScanFn
    if impl in ("scan4", "persist") and scan4_supported(B, S, rec_lin.out_features, H, hid, rssm.discrete):
        fn = RSSMScan4Fn
    return fn.apply(a_proj.contiguous(), P.contiguous(), is_first.contiguous(), uniform, z0.reshape(-1).contiguous(),
                            Wz, rec[1].weight, rec[1].bias, gru.linear.weight, gru.layer_norm.weight, gru.layer_norm.bias,
                            W1, ln2_w, ln2_b, W2, b2, meta)
