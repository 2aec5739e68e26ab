"""The distributed runner: one process per GPU, RCCL over xGMI (gloo on CPU).

Replaces Lightning Fabric in the reference (``sheeprl/cli.py:83-84``, ``fabric.launch``,
``setup_module``, ``backward``, ``clip_gradients``, ``all_gather``, ``all_reduce``, ``barrier``,
``save``/``load``, ``log``/``log_dict``, ``call``).  Design choices for MI355X:

* no DDP wrapper per sub-module: every optimiser owns ONE flat fp32 gradient slab
  (:class:`~sheeprl_prey_amd.parallel.flat_optim.FlatOptimizer`), reduced by one RCCL
  all-reduce (or a few large buckets) per backward instead of 9 DDP instances;
* global-norm clipping and the Adam update run as two fused HIP kernels on that slab;
* launch: torchrun env (``RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*``) or local spawn of
  ``devices`` processes (the multi-process CPU tests use gloo).
"""
from __future__ import annotations

import datetime
import os
import pickle
import random
import socket
from contextlib import closing
from typing import Any, Callable, Dict, Iterable, List, Optional, Sequence, Union

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn
from torch import Tensor


# Fabric precision strings -> autocast dtype of the forward passes of set-up modules (None: plain fp32).
# "16-mixed" needs a loss scaler the flat-slab optimisers do not implement; "64-true" would need every
# buffer and env tensor in fp64: both are rejected up front rather than silently run in fp32.
_PRECISIONS = {"32-true": None, "32": None, "bf16-mixed": torch.bfloat16}
# Lightning Fabric's spellings of the same two modes (``fabric.precision=bf16`` / ``32`` in the reference)
_PRECISION_ALIASES = {"bf16": "bf16-mixed", "32-true": "32-true", "32": "32-true"}


def _autocast_dtype(precision: Any) -> Optional[torch.dtype]:
    key = str(precision).strip().lower()
    key = _PRECISION_ALIASES.get(key, key)
    if key not in _PRECISIONS:
        raise ValueError(f"fabric.precision={precision!r} is not supported; use one of "
                         f"{sorted(set(_PRECISIONS) | set(_PRECISION_ALIASES))} (16-mixed needs a loss scaler, "
                         "bf16-true / 64-true a non-fp32 parameter store: neither is implemented)")
    return _PRECISIONS[key]


def _autocast_targets(module: nn.Module) -> List[nn.Module]:
    """The modules whose ``forward`` the algorithms actually call.  A container without a forward of its
    own (DreamerV3's ``WorldModel`` and ``RSSM``, SAC's agent) is never called itself: its children are
    (the reference sets each of them up separately, ``dreamer_v3/agent.py:1054-1063``)."""
    if type(module).forward is not nn.Module.forward:
        return [module]
    out: List[nn.Module] = []
    for child in module.children():
        out += _autocast_targets(child)
    return out


def _to_fp32(out: Any) -> Any:
    if isinstance(out, Tensor):
        return out.float() if out.is_floating_point() and out.dtype != torch.float32 else out
    if isinstance(out, (tuple, list)):
        return type(out)(_to_fp32(o) for o in out)
    if isinstance(out, dict):
        return {k: _to_fp32(v) for k, v in out.items()}
    return out


class _AutocastHooks:
    """Forward pre/post hooks that run a module's ``forward`` under ``torch.autocast`` and hand fp32
    outputs back, like Fabric's mixed-precision ``_FabricModule`` (reference ``fabric.precision``,
    ``configs/fabric/default.yaml:5``).  Hooks, not a patched ``forward``: a deep-copied module (the
    target critics) keeps calling its OWN weights.  Our fused ops take fp32 only, so bf16 activations
    route through the eager reference ops (``ops/__init__.py`` dtype checks)."""

    def __init__(self, device_type: str, dtype: torch.dtype) -> None:
        self.device_type, self.dtype = device_type, dtype
        self._stack: List[Any] = []

    def pre(self, module, args):
        ctx = torch.autocast(self.device_type, dtype=self.dtype)
        ctx.__enter__()
        self._stack.append(ctx)

    def post(self, module, args, out):
        if self._stack:
            self._stack.pop().__exit__(None, None, None)
        return _to_fp32(out)


def _free_port() -> int:
    with closing(socket.socket(socket.AF_INET, socket.SOCK_STREAM)) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _resolve_accelerator(accelerator: str) -> str:
    acc = os.environ.get("LT_ACCELERATOR", accelerator) or "cpu"
    acc = str(acc).lower()
    if acc in ("gpu", "cuda", "rocm", "hip"):
        return "cuda"
    if acc == "auto":
        return "cuda" if torch.cuda.is_available() else "cpu"
    return "cpu"


def _resolve_devices(devices: Any, accelerator: str) -> int:
    dev = os.environ.get("LT_DEVICES", devices)
    if isinstance(dev, str):
        if dev in ("auto", "-1"):
            if "WORLD_SIZE" in os.environ:
                return int(os.environ["LOCAL_WORLD_SIZE"]) if "LOCAL_WORLD_SIZE" in os.environ else int(os.environ["WORLD_SIZE"])
            return max(torch.cuda.device_count(), 1) if accelerator == "cuda" else 1
        dev = int(dev)
    if isinstance(dev, (list, tuple)):
        return len(dev)
    if dev is None or int(dev) <= 0:
        # `devices: 0` in ddp presets means "all visible"
        return max(torch.cuda.device_count(), 1) if accelerator == "cuda" else 1
    return int(dev)


def _spawn_entry(local_rank: int, world_size: int, port: int, fn, cfg, runner_kwargs) -> None:
    os.environ["RANK"] = str(local_rank)
    os.environ["LOCAL_RANK"] = str(local_rank)
    os.environ["WORLD_SIZE"] = str(world_size)
    os.environ["LOCAL_WORLD_SIZE"] = str(world_size)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    runner = Runner(**runner_kwargs)
    runner._init_distributed()
    try:
        fn(runner, cfg)
    except BaseException:
        # no final barrier after a failure: the other ranks may sit in another collective; dropping
        # the process group makes theirs fail too instead of every rank hanging
        runner.teardown(clean=False)
        raise
    runner.teardown()


class Runner:
    """Process/device/collective layer used by every algorithm."""

    def __init__(
        self,
        devices: Any = 1,
        num_nodes: int = 1,
        strategy: str = "auto",
        accelerator: str = "cpu",
        precision: str = "32-true",
        callbacks: Optional[Sequence[Any]] = None,
        loggers: Optional[Sequence[Any]] = None,
        cuda_graphs: bool = False,
        fused_ops: bool = True,
        bucket_mb: float = 32,
        tunable_gemm: str = "use",
        overlap_grad_sync: bool = True,
        pg_timeout_s: float = 1800,
        process_group=None,
        **_unused,
    ) -> None:
        self.accelerator = _resolve_accelerator(accelerator)
        if self.accelerator == "cuda" and not torch.cuda.is_available():
            self.accelerator = "cpu"
        self.devices = _resolve_devices(devices, self.accelerator)
        self.num_nodes = int(num_nodes)
        self.strategy = strategy
        self.precision = precision
        self._amp_dtype = _autocast_dtype(precision)
        self._amp_hooks: Optional[_AutocastHooks] = None
        self.callbacks = list(callbacks or [])
        self._loggers = list(loggers or [])
        self.cuda_graphs = bool(cuda_graphs) and self.accelerator == "cuda"
        # fabric.fused_ops=False routes every op through the eager fp32 oracles (ops/reference.py)
        self.fused_ops = bool(fused_ops)
        from sheeprl_prey_amd import ops as _ops

        _ops.set_fused(self.fused_ops)
        self.bucket_mb = float(bucket_mb)
        # bucketed all-reduce launched from backward hooks (FlatOptimizer.enable_overlap)
        self.overlap_grad_sync = bool(overlap_grad_sync)
        # process-group timeout: a stalled collective ends the run with an error instead of holding the node
        self.pg_timeout_s = float(pg_timeout_s)
        # library-GEMM solution choice (parallel/gemm_tuning.py): committed TunableOp results
        self.tunable_gemm = str(tunable_gemm)
        self._kwargs = dict(
            devices=devices, num_nodes=num_nodes, strategy=strategy, accelerator=accelerator,
            precision=precision, callbacks=callbacks, cuda_graphs=cuda_graphs, fused_ops=fused_ops, bucket_mb=bucket_mb,
            tunable_gemm=tunable_gemm, overlap_grad_sync=overlap_grad_sync,
            pg_timeout_s=pg_timeout_s,
        )
        self.group = process_group  # None == WORLD
        if str(strategy).lower() in ("fsdp",):
            raise ValueError("FSDP is not supported: SheepRL-style RL models are replicated (data parallel only)")

    # ------------------------------------------------------------------ topology
    @property
    def world_size(self) -> int:
        if dist.is_available() and dist.is_initialized():
            return dist.get_world_size(self.group)
        return 1

    @property
    def global_rank(self) -> int:
        if dist.is_available() and dist.is_initialized():
            return dist.get_rank(self.group) if self.group is not None else dist.get_rank()
        return 0

    @property
    def local_rank(self) -> int:
        return int(os.environ.get("LOCAL_RANK", 0))

    @property
    def node_rank(self) -> int:
        return int(os.environ.get("GROUP_RANK", 0))

    @property
    def is_global_zero(self) -> bool:
        return self.global_rank == 0

    @property
    def device(self) -> torch.device:
        if self.accelerator == "cuda":
            n = torch.cuda.device_count()
            return torch.device("cuda", self.local_rank % max(n, 1))
        return torch.device("cpu")

    @property
    def backend(self) -> str:
        # On ROCm the "nccl" backend string IS RCCL.  SRL_DIST_BACKEND=gloo forces gloo with GPU
        # tensors (rehearsing the multi-rank GPU code path with several ranks on ONE GPU, where RCCL
        # would refuse the duplicate device).
        forced = os.environ.get("SRL_DIST_BACKEND")
        if forced:
            return forced
        return "nccl" if self.accelerator == "cuda" else "gloo"

    @property
    def logger(self):
        return self._loggers[0] if self._loggers else None

    @property
    def loggers(self):
        return self._loggers

    # ------------------------------------------------------------------ launch
    def _device_setup(self) -> None:
        """Per-process GPU setup after set_device: TunableOp mode, the one-launch column-sum workspace."""
        from sheeprl_prey_amd.parallel.gemm_tuning import configure

        configure(self.tunable_gemm)
        if self.fused_ops:
            from sheeprl_prey_amd import ops

            ops.init_reduce_workspace(self.device)

    def _init_distributed(self) -> None:
        ws = int(os.environ.get("WORLD_SIZE", "1"))
        if self.accelerator == "cuda":
            torch.cuda.set_device(self.device)
            self._device_setup()
        if ws > 1 and not dist.is_initialized():
            # RCCL errors / timeouts tear the process down (non-zero exit) rather than leaving it blocked
            os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
            kwargs = dict(backend=self.backend, timeout=datetime.timedelta(seconds=max(10.0, self.pg_timeout_s)))
            if self.accelerator == "cuda" and self.backend == "nccl":
                kwargs["device_id"] = self.device
            dist.init_process_group(**kwargs)

    def launch(self, fn: Callable[["Runner", Any], Any], cfg: Any) -> Any:
        """Run ``fn(runner, cfg)`` on every rank."""
        already = "WORLD_SIZE" in os.environ and int(os.environ.get("WORLD_SIZE", "1")) > 1
        if already or self.devices * self.num_nodes <= 1:
            if already or dist.is_initialized():
                self._init_distributed()
            elif self.accelerator == "cuda":
                torch.cuda.set_device(self.device)
                self._device_setup()
            return fn(self, cfg)
        import torch.multiprocessing as mp

        port = _free_port()
        mp.start_processes(
            _spawn_entry,
            args=(self.devices, port, fn, cfg, self._kwargs),
            nprocs=self.devices,
            join=True,
            start_method="spawn",
        )
        return None

    def teardown(self, clean: bool = True) -> None:
        for lg in self._loggers:
            try:
                lg.finalize("success" if clean else "failed")
            except Exception:
                pass
        if dist.is_available() and dist.is_initialized():
            if clean:
                try:
                    dist.barrier()
                except Exception:
                    pass
            dist.destroy_process_group()

    # ------------------------------------------------------------------ utils
    def seed_everything(self, seed: int) -> int:
        random.seed(seed)
        np.random.seed(seed % (2**32))
        torch.manual_seed(seed)
        if torch.cuda.is_available():
            torch.cuda.manual_seed_all(seed)
        return seed

    def print(self, *args, **kwargs) -> None:
        if self.is_global_zero:
            print(*args, **kwargs, flush=True)

    def to_device(self, x):
        if isinstance(x, Tensor):
            return x.to(self.device, non_blocking=x.is_pinned() or x.device.type != "cpu")
        if isinstance(x, dict):
            return {k: self.to_device(v) for k, v in x.items()}
        return x

    def setup_module(self, module: nn.Module) -> nn.Module:
        """Move to device, make every rank start from rank 0's weights and, with
        ``precision=bf16-mixed``, run the module's forward under autocast."""
        module = module.to(self.device)
        if self._amp_dtype is not None:
            if self._amp_hooks is None:
                self._amp_hooks = _AutocastHooks(self.device.type, self._amp_dtype)
            for m in _autocast_targets(module):
                m.register_forward_pre_hook(self._amp_hooks.pre)
                m.register_forward_hook(self._amp_hooks.post, always_call=True)
            # fp32-only fast paths that read weights without calling forwards (fused RSSM scan,
            # buffer-resident imagination, fused PPO rollout/update) check this flag and step aside
            for m in module.modules():
                m._srl_autocast = True
        if self.world_size > 1:
            with torch.no_grad():
                tensors = [p.data for p in module.parameters()] + [b for b in module.buffers()]
                if tensors:
                    flat = torch.cat([t.reshape(-1).float() for t in tensors])
                    dist.broadcast(flat, src=self._global_src(0), group=self.group)
                    off = 0
                    for t in tensors:
                        n = t.numel()
                        t.copy_(flat[off : off + n].view_as(t).to(t.dtype))
                        off += n
        return module

    def setup_optimizers(self, *optimizers):
        return optimizers[0] if len(optimizers) == 1 else optimizers

    def _global_src(self, src: int) -> int:
        if self.group is None:
            return src
        return dist.get_global_rank(self.group, src)

    # ------------------------------------------------------------------ grads
    def backward(self, loss: Tensor, optimizer=None, **kwargs) -> None:
        """``loss.backward()`` then average the optimiser's flat gradient slab across ranks."""
        loss.backward(**kwargs)
        if optimizer is not None:
            self.sync_gradients(optimizer)

    def agree_faults(self, device) -> None:
        """Make the device-side skip decision collective: all-reduce (max) words 0/1 of the device fault block
        (persistent-scan hand-off timeout, replay-gather error; ``ops.fault_block``) so that when ONE rank's
        kernels recorded a fault every rank skips the same optimiser update (the flat optimisers' norm /
        advance kernels read those words) and every rank raises at its next host health check, instead of the
        faulted rank keeping its parameters while the others step and the replicas silently diverging."""
        if self.world_size <= 1 or torch.device(device).type != "cuda":
            return
        from sheeprl_prey_amd import ops

        dist.all_reduce(ops.fault_block(device)[:2], op=dist.ReduceOp.MAX, group=self.group)

    def sync_gradients(self, optimizer, wait: bool = True, faults: bool = False) -> None:
        """Average ``optimizer``'s gradients over the ranks.  ``wait=False`` (flat optimisers): the
        collectives stay in flight until the optimiser's next ``clip_grad_norm_`` / ``step`` joins them.
        ``faults=True``: first agree on the device fault words (``agree_faults``) - pass it on the step's first
        sync, after the kernels that can record a fault (replay gather, scan) and before any optimiser reads
        them."""
        if self.world_size <= 1:
            return
        from sheeprl_prey_amd.parallel.flat_optim import FlatOptimizer

        if faults:
            dev = optimizer.flat_param.device if isinstance(optimizer, FlatOptimizer) else next(
                (p.device for g in optimizer.param_groups for p in g["params"]), torch.device("cpu"))
            self.agree_faults(dev)
        if isinstance(optimizer, FlatOptimizer):
            optimizer.all_reduce_grads(self.group, self.world_size, bucket_mb=self.bucket_mb, wait=wait)
            if self.overlap_grad_sync:
                # from the next zero_grad on, buckets launch from the backward hooks (same call on every rank)
                optimizer.enable_overlap(self.group, self.world_size, bucket_mb=self.bucket_mb)
            return
        grads = [p.grad for g in optimizer.param_groups for p in g["params"] if p.grad is not None]
        if not grads:
            return
        flat = torch.cat([g.reshape(-1) for g in grads])
        dist.all_reduce(flat, group=self.group)
        flat.div_(self.world_size)
        off = 0
        for g in grads:
            n = g.numel()
            g.copy_(flat[off : off + n].view_as(g))
            off += n

    def clip_gradients(
        self,
        module: Optional[nn.Module] = None,
        optimizer=None,
        max_norm: float = 1.0,
        norm_type: float = 2.0,
        error_if_nonfinite: bool = False,
    ) -> Tensor:
        """Global-norm clip.  On a flat slab: one fused norm kernel; the scaling is folded into
        the next optimiser step (no host sync).  Returns the pre-clip norm (device tensor)."""
        from sheeprl_prey_amd.parallel.flat_optim import FlatOptimizer

        if isinstance(optimizer, FlatOptimizer):
            return optimizer.clip_grad_norm_(max_norm)
        params = [p for p in (module.parameters() if module is not None else []) if p.grad is not None]
        return torch.nn.utils.clip_grad_norm_(params, max_norm, norm_type=norm_type, error_if_nonfinite=error_if_nonfinite)

    # ------------------------------------------------------------------ uneven inputs (DDP ``Join``)
    def max_steps(self, n_local: int) -> int:
        """Ranks with different numbers of optimisation steps (uneven data) agree on the max; the
        ranks that run out shadow the remaining gradient all-reduces (``shadow_step``) like
        ``torch.distributed.algorithms.Join`` does for DDP (reference ``ppo_recurrent.py:54``)."""
        if self.world_size <= 1:
            return n_local
        dev = self.device if self.backend == "nccl" else torch.device("cpu")
        t = torch.tensor([n_local], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return int(t.item())

    def shadow_step(self, optimizer) -> None:
        """Contribute zero gradients to a collective the other ranks are running (no update)."""
        optimizer.zero_grad()
        self.sync_gradients(optimizer)

    def sync_from_last_joiner(self, module: nn.Module, n_local: int, n_max: int) -> None:
        """After uneven training every rank takes the weights of a rank that ran all ``n_max``
        steps (DDP Join's final model sync)."""
        if self.world_size <= 1:
            return
        dev = self.device if self.backend == "nccl" else torch.device("cpu")
        cand = torch.tensor([self.global_rank if n_local == n_max else 1 << 30], dtype=torch.int64, device=dev)
        dist.all_reduce(cand, op=dist.ReduceOp.MIN, group=self.group)
        src = int(cand.item())
        with torch.no_grad():
            flat = torch.cat([p.data.reshape(-1) for p in module.parameters()])
            self.broadcast(flat, src=src)
            off = 0
            for p in module.parameters():
                n = p.numel()
                p.data.copy_(flat[off : off + n].view_as(p))
                off += n

    # ------------------------------------------------------------------ collectives
    def barrier(self, *_args, **_kw) -> None:
        if self.world_size > 1:
            if self.backend == "nccl":
                dist.barrier(group=self.group, device_ids=[self.device.index])
            else:
                dist.barrier(group=self.group)

    def all_reduce(self, x: Tensor, reduce_op: str = "mean", group=None) -> Tensor:
        group = group if group is not None else self.group
        if self.world_size <= 1:
            return x
        x = x.clone()
        dist.all_reduce(x, group=group)
        if reduce_op in ("mean", "avg"):
            x = x / dist.get_world_size(group)
        return x

    def all_gather(self, data: Union[Tensor, Dict[str, Tensor]], group=None, sync_grads: bool = False):
        """Gather tensors (or dicts of tensors) into a new leading [world] dim.  A dict is packed
        into ONE byte buffer and gathered with a single collective (instead of one per key)."""
        group = group if group is not None else self.group
        if isinstance(data, dict):
            if self.world_size <= 1:
                return {k: v.unsqueeze(0) for k, v in data.items()}
            return self._all_gather_packed(data, group)
        if self.world_size <= 1:
            return data.unsqueeze(0)
        ws = dist.get_world_size(group)
        t = data.contiguous()
        if self.backend == "gloo" and t.is_cuda:
            t = t.cpu()
        if t.is_cuda:
            out = torch.empty((ws,) + tuple(t.shape), dtype=t.dtype, device=t.device)
            dist.all_gather_into_tensor(out, t, group=group)
        else:
            parts = [torch.empty_like(t) for _ in range(ws)]
            dist.all_gather(parts, t, group=group)
            out = torch.stack(parts)
        return out.to(data.device)

    def _all_gather_packed(self, data: Dict[str, Tensor], group) -> Dict[str, Tensor]:
        keys = list(data.keys())
        tensors = [data[k].contiguous() for k in keys]
        dev = tensors[0].device
        parts = [t.to(dev).reshape(-1).view(torch.uint8) for t in tensors]
        sizes = [p.numel() for p in parts]
        packed = torch.cat(parts) if len(parts) > 1 else parts[0]
        gathered = self.all_gather(packed, group=group)  # [ws, nbytes]
        out, off = {}, 0
        for k, t, n in zip(keys, tensors, sizes):
            chunk = gathered[:, off : off + n].contiguous()
            out[k] = chunk.view(t.dtype).view((gathered.shape[0],) + tuple(t.shape)).to(data[k].device)
            off += n
        return out

    def broadcast(self, x: Tensor, src: int = 0, group=None) -> Tensor:
        group = group if group is not None else self.group
        if self.world_size > 1:
            dist.broadcast(x, src=src if group is None else dist.get_global_rank(group, src), group=group)
        return x

    def broadcast_object(self, obj: Any, src: int = 0, group=None) -> Any:
        group = group if group is not None else self.group
        if self.world_size <= 1:
            return obj
        lst = [obj]
        dist.broadcast_object_list(lst, src=src if group is None else dist.get_global_rank(group, src), group=group)
        return lst[0]

    def gather_object(self, obj: Any, dst: int = 0, group=None) -> Optional[List[Any]]:
        group = group if group is not None else self.group
        if self.world_size <= 1:
            return [obj]
        out = [None] * dist.get_world_size(group) if self.global_rank == dst else None
        if self.backend == "nccl":
            # object collectives over RCCL would pickle into device tensors: use a gloo side group
            group = self.cpu_group(group)
        dist.gather_object(obj, out, dst=dst, group=group)
        return out

    _cpu_groups: Dict[Any, Any] = {}

    def cpu_group(self, group=None):
        key = id(group)
        if key not in Runner._cpu_groups:
            ranks = None if group is None else dist.get_process_group_ranks(group)
            Runner._cpu_groups[key] = dist.new_group(ranks=ranks, backend="gloo")
        return Runner._cpu_groups[key]

    # ------------------------------------------------------------------ io / logging
    def save(self, path: str, state: Dict[str, Any]) -> None:
        if self.is_global_zero:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
            tmp = path + ".tmp"
            torch.save(state, tmp)
            os.replace(tmp, path)
        self.barrier()

    def load(self, path: str, map_location: Any = "cpu") -> Dict[str, Any]:
        return torch.load(path, map_location=map_location, weights_only=True)

    def log(self, name: str, value: Any, step: int) -> None:
        if self.is_global_zero:
            for lg in self._loggers:
                lg.log_metrics({name: float(value)}, step)

    def log_dict(self, metrics: Dict[str, Any], step: int) -> None:
        if self.is_global_zero and metrics:
            for lg in self._loggers:
                lg.log_metrics(metrics, step)

    def call(self, hook: str, **kwargs) -> None:
        for cb in self.callbacks:
            fn = getattr(cb, hook, None)
            if fn is not None:
                fn(runner=self, **kwargs)
