"""Metric aggregation (reference: ``sheeprl/utils/metric.py:17-173``).

Values may be host numbers or device tensors.  Device scalars are accumulated *on the
device* (no per-update host sync - important when the train step is hipGraph-captured);
the host sees them only at ``compute()`` time, once per log interval.
"""
from __future__ import annotations

import math
import warnings
from typing import Any, Dict, Optional, Union

import torch
from torch import Tensor


class MeanMetric:
    def __init__(self, sync_on_compute: bool = False, **_):
        self.sync_on_compute = sync_on_compute
        self._acc: Optional[Tensor] = None
        self.reset()

    def attach(self, acc: Tensor) -> None:
        """A device accumulator ``[sum, count]`` (float64) that kernels add to every step (the fused SAC update,
        ``algos/sac/fused.py``): ``compute`` adds it, ``reset`` zeroes it - no per-step copy launch."""
        self._acc = acc

    SLOTS = 512  # device scalars staged before one NaN-filtered reduction

    def reset(self) -> None:
        self._host_sum = 0.0
        self._host_n = 0
        self._dev_sum: Optional[Tensor] = None
        self._dev_n: Optional[Tensor] = None
        self._slots: Optional[Tensor] = None
        self._used = 0
        if self._acc is not None:
            self._acc.zero_()

    def _flush(self) -> None:
        if not self._used:
            return
        v = self._slots[: self._used]
        finite = torch.isfinite(v)
        self._dev_sum += torch.where(finite, v, torch.zeros_like(v)).sum().double()
        self._dev_n += finite.sum().double()
        self._used = 0

    def update(self, value: Union[float, int, Tensor, Any]) -> None:
        if isinstance(value, Tensor):
            v = value.detach()
            if v.is_cuda:
                if self._dev_sum is None:
                    self._dev_sum = torch.zeros((), device=v.device, dtype=torch.float64)
                    self._dev_n = torch.zeros((), device=v.device, dtype=torch.float64)
                if v.numel() == 1:
                    # a per-step device scalar (e.g. a graph's static loss output): one copy kernel into
                    # a staging slot, no host sync; the NaN-filtered sum runs once per SLOTS updates
                    if self._slots is None:
                        self._slots = torch.empty(self.SLOTS, device=v.device, dtype=torch.float32)
                    self._slots[self._used].copy_(v.reshape(()))
                    self._used += 1
                    if self._used == self.SLOTS:
                        self._flush()
                    return
                v = v.float().reshape(-1)
                finite = torch.isfinite(v)
                self._dev_sum += torch.where(finite, v, torch.zeros_like(v)).sum().double()
                self._dev_n += finite.sum().double()
                return
            vals = v.float().reshape(-1).tolist()
        elif hasattr(value, "__len__"):
            vals = [float(x) for x in value]
        else:
            vals = [float(value)]
        for x in vals:
            if math.isfinite(x):
                self._host_sum += x
                self._host_n += 1

    def compute(self) -> float:
        s, n = self._host_sum, float(self._host_n)
        if self._dev_sum is not None:
            self._flush()
            s += float(self._dev_sum.item())
            n += float(self._dev_n.item())
        if self._acc is not None:
            a_s, a_n = self._acc.tolist()
            s += a_s
            n += a_n
        if self.sync_on_compute and torch.distributed.is_available() and torch.distributed.is_initialized():
            t = torch.tensor([s, n], dtype=torch.float64)
            torch.distributed.all_reduce(t)
            s, n = float(t[0]), float(t[1])
        return s / n if n > 0 else float("nan")

    def to(self, *_args, **_kw):
        return self


class MetricAggregator:
    """Dict of named metrics; NaN results are dropped at compute (reference ``metric.py:110-114``)."""

    disabled: bool = False

    def __init__(self, metrics: Optional[Dict[str, Any]] = None, raise_on_missing: bool = False):
        self.metrics: Dict[str, Any] = {}
        if metrics is not None:
            self.metrics = dict(metrics)
        self._raise_on_missing = raise_on_missing

    def __iter__(self):
        return iter(self.metrics.keys())

    def __contains__(self, name: str) -> bool:
        return name in self.metrics

    def add(self, name: str, metric: Any) -> None:
        if self.disabled:
            return
        if name in self.metrics:
            raise ValueError(f"Metric {name} already exists")
        self.metrics[name] = metric

    def update(self, name: str, value: Any) -> None:
        if self.disabled:
            return
        if name not in self.metrics:
            if self._raise_on_missing:
                raise ValueError(f"Metric {name} does not exist")
            warnings.warn(f"The key '{name}' is missing from the `MetricAggregator` keys.", UserWarning)
            return
        self.metrics[name].update(value)

    def pop(self, name: str) -> None:
        if name in self.metrics:
            self.metrics.pop(name)

    def reset(self) -> None:
        for m in self.metrics.values():
            m.reset()

    def to(self, device="cpu") -> "MetricAggregator":
        return self

    def compute(self) -> Dict[str, float]:
        out: Dict[str, float] = {}
        if self.disabled:
            return out
        for k, m in self.metrics.items():
            v = m.compute()
            if isinstance(v, Tensor):
                v = float(v.item())
            if not (isinstance(v, float) and math.isnan(v)):
                out[k] = v
        return out


class RankIndependentMetricAggregator:
    """Per-rank metric dicts gathered with ``all_gather_object`` (reference ``metric.py:118-173``)."""

    def __init__(self, metrics: Dict[str, Any], process_group=None):
        self._aggregator = MetricAggregator(metrics)
        self._process_group = process_group

    def update(self, name: str, value: Any) -> None:
        self._aggregator.update(name, value)

    def compute(self):
        local = self._aggregator.compute()
        if torch.distributed.is_available() and torch.distributed.is_initialized():
            ws = torch.distributed.get_world_size(self._process_group)
            out = [None] * ws
            torch.distributed.all_gather_object(out, local, group=self._process_group)
            return out
        return [local]

    def reset(self) -> None:
        self._aggregator.reset()

    def to(self, device="cpu"):
        return self
