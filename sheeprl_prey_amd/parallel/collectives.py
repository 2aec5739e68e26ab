"""Collective-sequence recording and a host-side hang watchdog for multi-rank runs.

A data-parallel step deadlocks (RCCL) or errors (gloo) as soon as two ranks issue their collectives
in different orders or with different sizes: hook-launched gradient buckets, the lambda all-gather of
``Moments`` (reference ``dreamer_v3/utils.py:35``) and a deferred actor all-reduce must line up on
every rank.  ``CollectiveLog`` wraps the ``torch.distributed`` entry points the framework calls and
records ``(phase, op, numel, dtype)`` per call, so tests can assert that every rank's sequence is
identical and ``bench.py`` can report how many collectives each phase of a step issues.

``Heartbeat`` is the guard for the driver's multi-GPU runs: a collective that never completes inside
a replayed hipGraph is invisible to the process group's own timeout (the watchdog tracks eagerly
launched works), so a daemon thread ends the process with a non-zero status when the main loop stops
beating, instead of letting it hold the node until an outer time limit.
"""
from __future__ import annotations

import os
import sys
import threading
import time
from collections import Counter, OrderedDict
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

_PHASE = ["-"]
_OPS = ("all_reduce", "all_gather", "all_gather_into_tensor", "reduce_scatter_tensor", "broadcast", "all_to_all_single",
        "all_gather_object", "broadcast_object_list", "scatter_object_list", "gather_object", "barrier")


def set_phase(name: str) -> None:
    """Tag the collectives issued from now on (a training step calls this at each of its phases)."""
    _PHASE[0] = name


def current_phase() -> str:
    return _PHASE[0]


def _numel(args, kwargs) -> int:
    for a in list(args) + list(kwargs.values()):
        if torch.is_tensor(a):
            return int(a.numel())
        if isinstance(a, (list, tuple)) and a and torch.is_tensor(a[0]):
            return int(sum(t.numel() for t in a))
    return 0


def _dtype(args, kwargs) -> str:
    for a in list(args) + list(kwargs.values()):
        if torch.is_tensor(a):
            return str(a.dtype).replace("torch.", "")
        if isinstance(a, (list, tuple)) and a and torch.is_tensor(a[0]):
            return str(a[0].dtype).replace("torch.", "")
    return "-"


class CollectiveLog:
    """Context manager: while active, every call of the wrapped ``torch.distributed`` collectives is
    appended to ``records`` as ``(step, phase, op, numel, dtype)``.  ``new_step()`` advances the step
    index (``DreamerV3Trainer.train_step`` calls it through ``step_boundary``)."""

    _active: Optional["CollectiveLog"] = None

    def __init__(self):
        self.records: List[Tuple[int, str, str, int, str]] = []
        self.step = 0
        self._orig = {}

    def __enter__(self) -> "CollectiveLog":
        for name in _OPS:
            fn = getattr(dist, name, None)
            if fn is None:
                continue
            self._orig[name] = fn
            setattr(dist, name, self._wrap(name, fn))
        CollectiveLog._active = self
        return self

    def __exit__(self, *exc) -> None:
        for name, fn in self._orig.items():
            setattr(dist, name, fn)
        self._orig.clear()
        CollectiveLog._active = None

    def _wrap(self, name, fn):
        def wrapped(*args, **kwargs):
            self.records.append((self.step, _PHASE[0], name, _numel(args, kwargs), _dtype(args, kwargs)))
            return fn(*args, **kwargs)

        wrapped.__wrapped__ = fn
        return wrapped

    def new_step(self) -> None:
        self.step += 1

    def sequence(self, step: Optional[int] = None) -> List[Tuple[str, str, int, str]]:
        return [r[1:] for r in self.records if step is None or r[0] == step]

    def per_phase(self, step: int) -> Dict[str, Dict[str, int]]:
        """``{phase: {op: count}}`` of one step (insertion-ordered by first use)."""
        out: "OrderedDict[str, Counter]" = OrderedDict()
        for s, ph, op, _, _ in self.records:
            if s == step:
                out.setdefault(ph, Counter())[op] += 1
        return {ph: dict(c) for ph, c in out.items()}


def step_boundary() -> None:
    """Called once per training step; advances the active ``CollectiveLog`` (no-op otherwise)."""
    log = CollectiveLog._active
    if log is not None:
        log.new_step()


class Heartbeat:
    """Daemon watchdog: if ``beat()`` is not called for ``timeout_s`` seconds the process prints the
    last beat's label and exits with status 3 (``os._exit``: a rank stuck in a device wait never
    returns to Python).  ``timeout_s <= 0`` disables it.  Until the first ``beat()`` the limit is
    ``max(timeout_s, startup_grace_s)``: model / env construction, the first graph captures, TunableOp
    tuning and diagnostic passes run before any step completes and must not trip a short step timeout.
    The grace defaults to ``grace_factor * timeout_s`` (scaled to the run: a short step timeout keeps a short
    start-up limit), and callers re-arm it around long passes with ``grace()``."""

    def __init__(self, timeout_s: float, label: str = "start", startup_grace_s: Optional[float] = None,
                 grace_factor: float = 4.0):
        self.timeout_s = float(timeout_s)
        self.startup_grace_s = float(startup_grace_s) if startup_grace_s is not None else grace_factor * self.timeout_s
        self._beaten = False
        self.label = label
        self._last = time.monotonic()
        self._stop = threading.Event()
        self._thread = None
        if self.timeout_s > 0:
            self._thread = threading.Thread(target=self._run, name="srl-heartbeat", daemon=True)
            self._thread.start()

    def beat(self, label: str = "") -> None:
        self._last = time.monotonic()
        self._beaten = True
        if label:
            self.label = label

    def grace(self, label: str = "") -> None:
        """Re-arm the start-up grace until the next ``beat()`` (long diagnostic passes, e.g. a rank-0 profile
        that the other ranks wait for at a barrier)."""
        self._last = time.monotonic()
        self._beaten = False
        if label:
            self.label = label

    def stop(self) -> None:
        self._stop.set()

    def _run(self) -> None:
        while not self._stop.wait(min(5.0, self.timeout_s / 4)):
            idle = time.monotonic() - self._last
            limit = self.timeout_s if self._beaten else max(self.timeout_s, self.startup_grace_s)
            if idle > limit:
                rank = os.environ.get("RANK", "0")
                print(f"[rank {rank}] heartbeat: no progress for {idle:.0f} s after '{self.label}' "
                      f"(a collective or kernel never completed); exiting", file=sys.stderr, flush=True)
                os._exit(3)
