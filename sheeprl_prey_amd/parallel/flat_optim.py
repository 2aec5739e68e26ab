"""Optimisers that own ONE contiguous fp32 slab of parameters and gradients.

Why (MI355X): the reference runs ``torch.optim.Adam`` per tensor behind 9 DDP wrappers
(``dreamer_v3/agent.py:1054-1063``).  Here every parameter of an optimiser is re-pointed into
a flat buffer (16-byte aligned chunks) and every ``.grad`` is a view of a flat gradient slab,
so that

* gradient sync is one RCCL all-reduce (or a few large buckets sized for xGMI),
* global-norm clipping is one reduction kernel (``ops.flat_grad_norm``) and the clip factor
  stays on the device (no host sync - hipGraph-capturable),
* the Adam/AdamW/SGD update is one fused, float4-vectorised HIP kernel (``ops.flat_adam``).

Optimiser state is exposed in ``torch.optim`` ``state_dict`` format so checkpoints keep the
reference's layout (``{"state": {i: {step, exp_avg, exp_avg_sq}}, "param_groups": [...]}``).
"""
from __future__ import annotations

import weakref

import math
from typing import Any, Dict, Iterable, List, Optional

import torch
import torch.distributed as dist
from torch import Tensor

_ALIGN = 4  # floats -> 16 B


_LIVE: "weakref.WeakSet[FlatOptimizer]" = weakref.WeakSet()


def gather_all_pending() -> None:
    """Rebuild every live optimiser's gradient slab whose grads still sit outside it (see
    ``FlatOptimizer.zero_grad``).  ``SegmentedGraph`` calls this at the end of each captured phase,
    so the copies are recorded in the phase that ran the backward - before the eager RCCL
    all-reduce that follows it between graph replays."""
    for opt in list(_LIVE):
        opt._gather()


def _aligned(n: int) -> int:
    return (n + _ALIGN - 1) // _ALIGN * _ALIGN


def _side_join() -> None:
    from sheeprl_prey_amd.ops import sidestream

    sidestream.join()


class FlatOptimizer:
    kind = "base"

    def __init__(self, params: Iterable, lr: float, weight_decay: float = 0.0, **defaults):
        plist: List[Tensor] = []
        seen = set()
        for p in params:
            if isinstance(p, dict):  # param group dicts: take the params (single group semantics)
                for q in p["params"]:
                    if id(q) not in seen and q.requires_grad:
                        seen.add(id(q))
                        plist.append(q)
                continue
            if id(p) in seen or not p.requires_grad:
                continue
            seen.add(id(p))
            plist.append(p)
        if not plist:
            raise ValueError("optimizer got an empty parameter list")
        self.params = plist
        device = plist[0].device
        self.offsets: List[int] = []
        total = 0
        for p in plist:
            self.offsets.append(total)
            total += _aligned(p.numel())
        self.numel = total
        owner = self._shared_owner(plist)
        if owner is not None:
            # every param already lives, in this order, in a contiguous run of another optimiser's
            # slab (e.g. SAC-AE's encoder: in both the critic and the encoder optimiser): share it,
            # keep separate optimiser state
            slab, base = owner
            self.flat_param = slab.flat_param[base : base + total]
            self.flat_grad = slab.flat_grad[base : base + total]
        else:
            self.flat_param = torch.zeros(total, device=device, dtype=torch.float32)
            self.flat_grad = torch.zeros(total, device=device, dtype=torch.float32)
            with torch.no_grad():
                for p, off in zip(plist, self.offsets):
                    n = p.numel()
                    self.flat_param[off : off + n].copy_(p.detach().reshape(-1))
                    p.data = self.flat_param[off : off + n].view_as(p)
                    p.grad = self.flat_grad[off : off + n].view_as(p)
                    p._flat_slab = (weakref.ref(self), off)
        # [step, clip_coef, last_norm, pad]
        self.scalars = torch.tensor([0.0, 1.0, 0.0, 0.0], device=device, dtype=torch.float32)
        self.param_groups = [dict(params=self.params, lr=lr, weight_decay=weight_decay, **defaults)]
        self.defaults = dict(lr=lr, weight_decay=weight_decay, **defaults)
        self._advanced = False
        self._detached = False  # grads live outside the slab until ``_gather`` (see zero_grad)
        _LIVE.add(self)
        self._init_state()

    def _shared_owner(self, plist: List[Tensor]):
        tags = [getattr(p, "_flat_slab", None) for p in plist]
        if all(t is None for t in tags):
            return None
        if any(t is None for t in tags) or len({id(t[0]()) for t in tags}) != 1:
            raise ValueError("FlatOptimizer: parameters are partly owned by another optimiser's flat slab; "
                             "a shared slab must cover exactly a contiguous run of the owner's parameters")
        slab = tags[0][0]()
        if slab is None:
            return None
        base = tags[0][1]
        for t, off in zip(tags, self.offsets):
            if t[1] - base != off:
                raise ValueError("FlatOptimizer: shared parameters are not contiguous/in order in the owner's slab")
        return slab, base

    # ------------------------------------------------------------------ to override
    def _init_state(self) -> None:
        pass

    def _update(self) -> None:
        raise NotImplementedError

    # ------------------------------------------------------------------ common
    @property
    def device(self) -> torch.device:
        return self.flat_param.device

    @property
    def lr(self) -> float:
        return self.param_groups[0]["lr"]

    def _relink(self) -> None:
        """Re-attach grads to the slab if user code set them to None."""
        for p, off in zip(self.params, self.offsets):
            if p.grad is None or p.grad.data_ptr() != self.flat_grad[off:].data_ptr():
                p.grad = self.flat_grad[off : off + p.numel()].view_as(p)

    def grad_views(self, params: Iterable[Tensor]) -> List[Tensor]:
        """The slab views of ``params``' gradients, with every ``.grad`` linked to its view: for kernels that
        write complete gradients straight into the slab (the fused SAC update) - nothing is zeroed or gathered
        before the optimiser reads it."""
        self.wait_grads()
        self._relink()
        self._detached = False
        index = {id(p): i for i, p in enumerate(self.params)}
        return [self._ov_view(index[id(p)]) for p in params]

    def zero_grad(self, set_to_none: bool = True, arm: bool = True) -> None:
        """``set_to_none`` (default): the next backward lets autograd hand each parameter its freshly
        computed gradient (AccumulateGrad steals the buffer: no per-parameter accumulate kernel), and
        the slab is rebuilt by ``_gather`` - one memset + multi-tensor copies - before anything reads
        it.  Otherwise the slab is zeroed and grads accumulate into it in place.

        ``arm`` starts an overlapped all-reduce round (``enable_overlap``): pass ``False`` for a
        clean-up zero that is not followed by the backward its sync belongs to - a backward of another
        loss reaching these parameters must not launch collectives."""
        self.wait_grads()
        ov = getattr(self, "_ov", None)
        if ov is not None:
            if arm:
                self.arm_overlap()
            else:
                for w in ov["works"]:
                    w.wait()
                ov.update(armed=False, works=[])
        if set_to_none:
            for p in self.params:
                p.grad = None
            self._detached = True
            return
        self.flat_grad.zero_()
        self._relink()
        self._detached = False

    def _gather(self) -> None:
        _side_join()
        if not self._detached:
            return
        self._detached = False
        views, grads, missing, in_slab = [], [], [], False
        for p, off in zip(self.params, self.offsets):
            v = self.flat_grad[off : off + p.numel()].view_as(p)
            g = p.grad
            if g is None:
                missing.append(v)
            elif g.data_ptr() != v.data_ptr():
                views.append(v)
                grads.append(g if g.dtype == v.dtype else g.to(v.dtype))
            else:
                in_slab = True
            p.grad = v
        if missing:
            if in_slab:
                torch._foreach_zero_(missing)
            else:
                self.flat_grad.zero_()  # one memset (also clears the alignment padding)
        if grads:
            torch._foreach_copy_(views, grads)

    def _guard(self) -> Optional[Tensor]:
        """The device fault block (``ops.fault_block``) the update kernels check: a step during which a kernel
        recorded a fault (persistent-scan hand-off timeout, out-of-range replay index) leaves the parameters and
        the Adam moments untouched.  GPU slabs only (the CPU path has no such kernels)."""
        from sheeprl_prey_amd import ops

        return ops.fault_block(self.flat_param.device) if self.flat_param.is_cuda else None

    def clip_grad_norm_(self, max_norm: float) -> Tensor:
        from sheeprl_prey_amd import ops

        self.wait_grads()
        self._gather()
        norm = ops.flat_grad_norm(self.flat_grad, self.scalars, float(max_norm), self._guard())
        self._advanced = True
        return norm

    # ------------------------------------------------------------------ overlapped gradient all-reduce
    def enable_overlap(self, group=None, world_size: int = 1, bucket_mb: float = 32) -> bool:
        """Bucketed all-reduce overlapped with the backward (eager multi-rank paths).

        The slab is cut into buckets from its tail (parameters are laid out in forward order, so
        the backward produces the tail first).  A post-accumulate-grad hook per parameter moves its
        fresh gradient into the slab and, once every parameter of a bucket has reported, launches
        that bucket's async all-reduce while autograd keeps computing earlier layers.  Buckets are
        launched strictly in index order, so every rank issues the same collective sequence
        whatever the hook order.  Hooks act only between ``arm_overlap()`` and the following
        ``all_reduce_grads`` (``Runner.backward`` / ``Runner.sync_gradients`` pair them), so extra
        backward passes that accumulate into the same slab never trigger a collective.  Contract: ONE
        backward between ``zero_grad`` (which arms) and the sync, as every algorithm here does.
        Reference counterpart: the per-model DDP reducers of ``dreamer_v3/agent.py:1054-1063``.

        Collectives never enter a hipGraph: inside a capture the hooks do nothing (the segmented graph
        mode issues the whole-slab all-reduce eagerly between phase replays)."""
        if world_size <= 1 or getattr(self, "_ov", None) is not None:
            return getattr(self, "_ov", None) is not None
        if self.flat_grad._base is not None or any(
                getattr(p, "_flat_slab", (None,))[0] is not None and p._flat_slab[0]() is not self for p in self.params):
            return False  # slab shared with another optimiser: keep the plain path
        cap = max(_ALIGN, int(bucket_mb * (1 << 20) // 4))
        buckets: List[List[int]] = []  # param indices, tail first
        cur, size = [], 0
        for i in reversed(range(len(self.params))):
            cur.append(i)
            size += _aligned(self.params[i].numel())
            if size >= cap:
                buckets.append(cur)
                cur, size = [], 0
        if cur:
            buckets.append(cur)
        ranges = []
        for b in buckets:
            lo = min(self.offsets[i] for i in b)
            hi = max(self.offsets[i] + _aligned(self.params[i].numel()) for i in b)
            ranges.append((lo, hi))
        bucket_of = {}
        for bi, b in enumerate(buckets):
            for i in b:
                bucket_of[i] = bi
        g = self.flat_grad
        use_avg = g.is_cuda and dist.get_backend(group) == "nccl"
        self._ov = dict(group=group, ws=world_size, buckets=buckets, ranges=ranges, bucket_of=bucket_of,
                        op=dist.ReduceOp.AVG if use_avg else dist.ReduceOp.SUM, avg=use_avg, armed=False,
                        pending=[], seen=[], works=[], next=0)
        self._ov_handles = [p.register_post_accumulate_grad_hook(self._make_ov_hook(i)) for i, p in enumerate(self.params)]
        return True

    def _make_ov_hook(self, i: int):
        ref = weakref.ref(self)

        def hook(p: Tensor) -> None:
            self_ = ref()
            # no collective inside a hipGraph capture: the segmented mode issues them between replays
            if self_ is None or not self_._ov["armed"]:
                return
            if p.is_cuda and torch.cuda.is_current_stream_capturing():
                return
            self_._ov_ready(i, p)

        return hook

    def arm_overlap(self) -> None:
        """Start a new gradient round (``zero_grad`` calls this).  A round that launched buckets and
        was never synced (no ``all_reduce_grads``) is drained and dropped - every rank does the same."""
        ov = getattr(self, "_ov", None)
        if ov is None:
            return
        for w in ov["works"]:
            w.wait()
        ov.update(armed=True, pending=[len(b) for b in ov["buckets"]], seen=[False] * len(self.params), works=[], next=0)

    def _ov_view(self, i: int) -> Tensor:
        p = self.params[i]
        return self.flat_grad[self.offsets[i] : self.offsets[i] + p.numel()].view_as(p)

    def _ov_ready(self, i: int, p: Tensor) -> None:
        ov = self._ov
        if ov["seen"][i]:
            return
        _side_join()  # the gradient may still be in flight on the side stream
        v = self._ov_view(i)
        g = p.grad
        if g is not None and g.data_ptr() != v.data_ptr():
            v.copy_(g)
            p.grad = v
        elif g is None:
            v.zero_()
            p.grad = v
        ov["seen"][i] = True
        b = ov["bucket_of"][i]
        ov["pending"][b] -= 1
        self._ov_launch_ready()

    def _ov_launch_ready(self) -> None:
        ov = self._ov
        while ov["next"] < len(ov["buckets"]) and ov["pending"][ov["next"]] == 0:
            lo, hi = ov["ranges"][ov["next"]]
            ov["works"].append(dist.all_reduce(self.flat_grad[lo:hi], op=ov["op"], group=ov["group"], async_op=True))
            ov["next"] += 1

    def _ov_finish(self, wait: bool = True) -> None:
        ov = self._ov
        _side_join()  # deferred parameter gradients (ops/sidestream.py) land in .grad without a hook
        # parameters whose hook did not fire in this backward: no gradient (a zero slab view), a deferred one set
        # by the side stream, or the accumulated one already in the slab
        for i, p in enumerate(self.params):
            if not ov["seen"][i]:
                v = self._ov_view(i)
                if p.grad is None:
                    v.zero_()
                elif p.grad.data_ptr() != v.data_ptr():
                    v.copy_(p.grad)
                p.grad = v
                ov["seen"][i] = True
                ov["pending"][ov["bucket_of"][i]] -= 1
        self._detached = False
        self._ov_launch_ready()
        works = ov["works"]
        ov.update(armed=False, works=[])
        self._pending = (works, None if ov["avg"] else ov["ws"])
        if wait:
            self.wait_grads()

    def all_reduce_grads(self, group=None, world_size: int = 1, bucket_mb: int = 32, wait: bool = True) -> None:
        """Average the gradient slab over ``group`` (bucketed for xGMI).  ``wait=False`` leaves the
        collectives in flight: ``wait_grads`` - called by ``clip_grad_norm_`` / ``step`` before they read
        the slab - joins them, so the caller may run independent work meanwhile (on a graph-captured
        step the join is a stream dependency, the overlap is recorded in the graph)."""
        ov = getattr(self, "_ov", None)
        if ov is not None and ov["armed"]:
            self._ov_finish(wait)
            return
        self._gather()
        if world_size <= 1:
            return
        g = self.flat_grad
        use_avg = g.is_cuda and dist.get_backend(group) == "nccl"
        op = dist.ReduceOp.AVG if use_avg else dist.ReduceOp.SUM
        bucket = max(1, int(bucket_mb * (1 << 20) // 4))
        works = [dist.all_reduce(g[i : i + bucket], op=op, group=group, async_op=True) for i in range(0, g.numel(), bucket)]
        self._pending = (works, None if use_avg else world_size)
        if wait:
            self.wait_grads()

    def wait_grads(self) -> None:
        """Join the gradient collectives ``all_reduce_grads(wait=False)`` left in flight (and any side-stream
        gradient work, ``ops/sidestream.py``)."""
        _side_join()
        pending = getattr(self, "_pending", None)
        if pending is None:
            return
        self._pending = None
        works, div = pending
        for w in works:
            w.wait()
        if div is not None:
            self.flat_grad.div_(div)

    @torch.no_grad()
    def step(self, closure=None):
        from sheeprl_prey_amd import ops

        self.wait_grads()
        self._gather()
        if not self._advanced:
            ops.flat_advance(self.scalars, self._guard())
        self._advanced = False
        self._update()
        return None

    # ------------------------------------------------------------------ state dict (torch format)
    def _state_tensors(self) -> Dict[str, Tensor]:
        return {}

    def state_dict(self) -> Dict[str, Any]:
        step = self.scalars[0].detach().cpu().clone()
        state = {}
        bufs = self._state_tensors()
        for i, (p, off) in enumerate(zip(self.params, self.offsets)):
            n = p.numel()
            st = {"step": step.clone()}
            for name, b in bufs.items():
                st[name] = b[off : off + n].view_as(p).detach().cpu().clone()
            state[i] = st
        groups = []
        for g in self.param_groups:
            gg = {k: v for k, v in g.items() if k != "params"}
            gg["params"] = list(range(len(self.params)))
            groups.append(gg)
        return {"state": state, "param_groups": groups}

    def load_state_dict(self, sd: Dict[str, Any]) -> None:
        bufs = self._state_tensors()
        st = sd.get("state", {})
        with torch.no_grad():
            for i, (p, off) in enumerate(zip(self.params, self.offsets)):
                s = st.get(i, st.get(str(i)))
                if s is None:
                    continue
                n = p.numel()
                for name, b in bufs.items():
                    if name in s:
                        b[off : off + n].copy_(torch.as_tensor(s[name]).reshape(-1).to(b.device))
                if "step" in s:
                    self.scalars[0] = float(torch.as_tensor(s["step"]).item())
        if sd.get("param_groups"):
            for g, sg in zip(self.param_groups, sd["param_groups"]):
                for k, v in sg.items():
                    if k != "params":
                        g[k] = v


class FlatAdam(FlatOptimizer):
    """``torch.optim.Adam`` semantics (L2 weight decay added to the gradient); ``decoupled``
    gives AdamW."""

    kind = "adam"

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 amsgrad: bool = False, decoupled: bool = False, **_ignored):
        if amsgrad:
            raise ValueError("amsgrad is not supported by the fused flat Adam")
        self.decoupled = decoupled
        super().__init__(params, lr=lr, weight_decay=weight_decay, betas=tuple(betas), eps=eps)

    def _init_state(self) -> None:
        self.exp_avg = torch.zeros_like(self.flat_param)
        self.exp_avg_sq = torch.zeros_like(self.flat_param)

    def _state_tensors(self):
        return {"exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq}

    def _update(self) -> None:
        from sheeprl_prey_amd import ops

        g = self.param_groups[0]
        b1, b2 = g["betas"]
        ops.flat_adam(self.flat_param, self.flat_grad, self.exp_avg, self.exp_avg_sq, self.scalars,
                      float(g["lr"]), float(b1), float(b2), float(g["eps"]), float(g["weight_decay"]), self.decoupled)


class FlatAdamW(FlatAdam):
    kind = "adamw"

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 1e-2, **kw):
        kw.pop("decoupled", None)
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, decoupled=True, **kw)


class FlatSGD(FlatOptimizer):
    kind = "sgd"

    def __init__(self, params, lr: float = 1e-3, momentum: float = 0.0, dampening: float = 0.0,
                 weight_decay: float = 0.0, nesterov: bool = False, **_ignored):
        super().__init__(params, lr=lr, weight_decay=weight_decay, momentum=momentum, dampening=dampening, nesterov=nesterov)

    def _init_state(self) -> None:
        self.momentum_buffer = torch.zeros_like(self.flat_param)

    def _state_tensors(self):
        return {"momentum_buffer": self.momentum_buffer}

    def _update(self) -> None:
        g = self.param_groups[0]
        coef = self.scalars[1]
        grad = self.flat_grad * coef
        if g["weight_decay"]:
            grad = grad + g["weight_decay"] * self.flat_param
        if g["momentum"]:
            first = self.scalars[0] <= 1
            self.momentum_buffer.mul_(g["momentum"]).add_(grad, alpha=1 - g["dampening"])
            self.momentum_buffer.copy_(torch.where(first, grad, self.momentum_buffer))
            grad = grad + g["momentum"] * self.momentum_buffer if g["nesterov"] else self.momentum_buffer
        self.flat_param.add_(grad, alpha=-g["lr"])


_TARGETS = {
    "torch.optim.Adam": FlatAdam,
    "torch.optim.AdamW": FlatAdamW,
    "torch.optim.SGD": FlatSGD,
    "sheeprl_prey_amd.parallel.flat_optim.FlatAdam": FlatAdam,
    "sheeprl_prey_amd.parallel.flat_optim.FlatAdamW": FlatAdamW,
    "sheeprl_prey_amd.parallel.flat_optim.FlatSGD": FlatSGD,
}


def flatten_like(target: torch.nn.Module, source_opt: FlatOptimizer) -> Tensor:
    """Re-point ``target``'s parameters (e.g. a target network) into a flat slab laid out like
    ``source_opt.flat_param``, so Polyak averaging is one ``lerp_`` over the slab."""
    flat = torch.zeros_like(source_opt.flat_param)
    tparams = list(target.parameters())
    assert len(tparams) == len(source_opt.params), "target/source parameter count mismatch"
    with torch.no_grad():
        for sp, tp, off in zip(source_opt.params, tparams, source_opt.offsets):
            n = tp.numel()
            assert sp.shape == tp.shape, "target/source parameter layout mismatch"
            flat[off : off + n].copy_(tp.detach().reshape(-1))
            tp.data = flat[off : off + n].view_as(tp)
    return flat


def build_optimizer(cfg: Dict[str, Any], params) -> FlatOptimizer:
    """Instantiate an optimiser from a Hydra-style ``{_target_: torch.optim.Adam, lr: ...}``
    node.  The torch targets map onto the flat fused implementations."""
    cfg = dict(cfg)
    target = cfg.pop("_target_", "torch.optim.Adam")
    cls = _TARGETS.get(target)
    if cls is None:
        raise ValueError(f"Unsupported optimizer target '{target}'. Supported: {sorted(_TARGETS)}")
    return cls(params, **cfg)
