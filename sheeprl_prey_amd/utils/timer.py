"""Named wall-clock timers (reference: ``sheeprl/utils/timer.py:15-82``).

``with timer("Time/train_time"):`` accumulates seconds into a class-level registry;
``timer.compute()`` returns ``{name: seconds}`` and ``timer.reset()`` clears it.
Optionally synchronises the GPU at region boundaries so asynchronous launches are
charged to the right region (``sync_cuda``).
"""
from __future__ import annotations

import time
from contextlib import ContextDecorator
from typing import Dict, Optional

import torch


class SumMetric:
    """Tiny replacement for ``torchmetrics.SumMetric`` (host float accumulation)."""

    def __init__(self, sync_on_compute: bool = False, **_):
        self.sync_on_compute = sync_on_compute
        self.value = 0.0

    def update(self, v) -> None:
        self.value += float(v)

    def compute(self) -> float:
        if self.sync_on_compute and torch.distributed.is_available() and torch.distributed.is_initialized():
            t = torch.tensor([self.value], dtype=torch.float64)
            torch.distributed.all_reduce(t)
            return float(t.item())
        return self.value

    def reset(self) -> None:
        self.value = 0.0

    def to(self, *_args, **_kw):
        return self


class timer(ContextDecorator):
    disabled: bool = False
    sync_cuda: bool = False
    timers: Dict[str, SumMetric] = {}
    _start_time: Optional[float] = None

    def __init__(self, name: str, metric: Optional[SumMetric] = None) -> None:
        self.name = name
        if not timer.disabled and name not in timer.timers:
            timer.timers[name] = metric if metric is not None else SumMetric()

    def start(self) -> None:
        if self._start_time is not None:
            raise RuntimeError("timer is running. Use .stop() to stop it")
        if timer.sync_cuda and torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize()
        self._start_time = time.perf_counter()

    def stop(self) -> float:
        if self._start_time is None:
            raise RuntimeError("timer is not running. Use .start() to start it")
        if timer.sync_cuda and torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize()
        elapsed = time.perf_counter() - self._start_time
        self._start_time = None
        if self.name in timer.timers:
            timer.timers[self.name].update(elapsed)
        return elapsed

    @classmethod
    def to(cls, device="cpu") -> None:
        return None

    @classmethod
    def add(cls, name: str, seconds: float) -> None:
        """Charge ``seconds`` measured elsewhere (e.g. GPU event time of asynchronously launched work)."""
        if cls.disabled:
            return
        if name not in cls.timers:
            cls.timers[name] = SumMetric()
        cls.timers[name].update(seconds)

    @classmethod
    def reset(cls) -> None:
        for t in cls.timers.values():
            t.reset()

    @classmethod
    def compute(cls) -> Dict[str, float]:
        return {k: v.compute() for k, v in cls.timers.items()}

    def __enter__(self):
        if not timer.disabled:
            self.start()
        return self

    def __exit__(self, *exc_info):
        if not timer.disabled:
            self.stop()
        return False
