"""Observation/action spaces with the gymnasium 0.29 API surface used by the framework
(``Box``, ``Discrete``, ``MultiDiscrete``, ``Dict``): ``shape``, ``dtype``, ``sample()``,
``seed()``, ``contains()``, ``low/high``, ``n``, ``nvec``.  gymnasium is not part of the image."""
from __future__ import annotations

from collections import OrderedDict
from typing import Any, Dict as TDict, Optional, Sequence, Tuple, Union

import numpy as np


class Space:
    def __init__(self, shape: Optional[Tuple[int, ...]] = None, dtype=None, seed: Optional[int] = None):
        self._shape = None if shape is None else tuple(int(s) for s in shape)
        self.dtype = None if dtype is None else np.dtype(dtype)
        self._np_random: Optional[np.random.Generator] = None
        if seed is not None:
            self.seed(seed)

    @property
    def np_random(self) -> np.random.Generator:
        if self._np_random is None:
            self.seed()
        return self._np_random

    @property
    def shape(self):
        return self._shape

    def seed(self, seed: Optional[int] = None):
        self._np_random = np.random.default_rng(seed)
        return [seed]

    def sample(self, mask=None):
        raise NotImplementedError

    def contains(self, x) -> bool:
        raise NotImplementedError

    def __contains__(self, x) -> bool:
        return self.contains(x)


class Box(Space):
    def __init__(self, low, high, shape: Optional[Sequence[int]] = None, dtype=np.float32, seed=None):
        dtype = np.dtype(dtype)
        if shape is None:
            shape = np.shape(low) if np.ndim(low) > 0 else np.shape(high)
        shape = tuple(int(s) for s in shape)
        lo = np.broadcast_to(np.asarray(low, dtype=np.float64), shape)
        hi = np.broadcast_to(np.asarray(high, dtype=np.float64), shape)
        if dtype.kind in "uib":
            info = np.iinfo(dtype) if dtype.kind != "b" else None
            if info is not None:
                lo = np.clip(lo, info.min, info.max)
                hi = np.clip(hi, info.min, info.max)
        self.low = lo.astype(dtype)
        self.high = hi.astype(dtype)
        super().__init__(shape, dtype, seed)

    def is_bounded(self, manner: str = "both") -> bool:
        below = bool(np.all(np.isfinite(self.low)))
        above = bool(np.all(np.isfinite(self.high)))
        return {"both": below and above, "below": below, "above": above}[manner]

    def sample(self, mask=None):
        if self.dtype.kind in "ui":
            return self.np_random.integers(self.low, self.high.astype(np.int64) + 1, size=self.shape).astype(self.dtype)
        low = np.where(np.isfinite(self.low), self.low, -1.0)
        high = np.where(np.isfinite(self.high), self.high, 1.0)
        unb = ~np.isfinite(self.low) & ~np.isfinite(self.high)
        s = self.np_random.uniform(low, high, size=self.shape)
        if unb.any():
            s = np.where(unb, self.np_random.normal(size=self.shape), s)
        return s.astype(self.dtype)

    def contains(self, x) -> bool:
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low)) and bool(np.all(x <= self.high))

    def __repr__(self):
        return f"Box({self.low.min() if self.low.size else ''}, {self.high.max() if self.high.size else ''}, {self.shape}, {self.dtype})"

    def __eq__(self, other):
        return isinstance(other, Box) and self.shape == other.shape and np.allclose(self.low, other.low) and np.allclose(self.high, other.high)


class Discrete(Space):
    def __init__(self, n: int, seed=None, start: int = 0):
        self.n = int(n)
        self.start = int(start)
        super().__init__((), np.int64, seed)

    def sample(self, mask=None):
        return np.int64(self.start + self.np_random.integers(self.n))

    def contains(self, x) -> bool:
        try:
            x = int(x)
        except (TypeError, ValueError):
            return False
        return self.start <= x < self.start + self.n

    def __repr__(self):
        return f"Discrete({self.n})"

    def __eq__(self, other):
        return isinstance(other, Discrete) and self.n == other.n


class MultiDiscrete(Space):
    def __init__(self, nvec, dtype=np.int64, seed=None):
        self.nvec = np.asarray(nvec, dtype=dtype)
        super().__init__(self.nvec.shape, dtype, seed)

    def sample(self, mask=None):
        return (self.np_random.random(self.nvec.shape) * self.nvec).astype(self.dtype)

    def contains(self, x) -> bool:
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= 0)) and bool(np.all(x < self.nvec))

    def __repr__(self):
        return f"MultiDiscrete({self.nvec.tolist()})"


class Dict(Space):
    def __init__(self, spaces: Optional[Union[TDict[str, Space], Sequence[Tuple[str, Space]]]] = None, seed=None, **kw):
        if spaces is None:
            spaces = {}
        if isinstance(spaces, dict) and not isinstance(spaces, OrderedDict):
            spaces = OrderedDict(spaces.items())
        elif not isinstance(spaces, OrderedDict):
            spaces = OrderedDict(spaces)
        spaces.update(kw)
        self.spaces: "OrderedDict[str, Space]" = spaces
        super().__init__(None, None, seed)

    def seed(self, seed: Optional[int] = None):
        super().seed(seed)
        for i, s in enumerate(self.spaces.values()):
            s.seed(None if seed is None else seed + i)
        return [seed]

    def sample(self, mask=None):
        return OrderedDict((k, s.sample()) for k, s in self.spaces.items())

    def contains(self, x) -> bool:
        return isinstance(x, dict) and all(k in x and s.contains(x[k]) for k, s in self.spaces.items())

    def __getitem__(self, k: str) -> Space:
        return self.spaces[k]

    def __setitem__(self, k: str, v: Space) -> None:
        self.spaces[k] = v

    def __iter__(self):
        return iter(self.spaces)

    def __len__(self):
        return len(self.spaces)

    def keys(self):
        return self.spaces.keys()

    def items(self):
        return self.spaces.items()

    def values(self):
        return self.spaces.values()

    def __repr__(self):
        return "Dict(" + ", ".join(f"{k!r}: {s}" for k, s in self.spaces.items()) + ")"


def batch_space(space: Space, n: int) -> Space:
    """The space of ``n`` stacked samples (vector-env ``observation_space``/``action_space``)."""
    if isinstance(space, Box):
        return Box(np.repeat(space.low[None], n, 0), np.repeat(space.high[None], n, 0), (n, *space.shape), space.dtype)
    if isinstance(space, Discrete):
        return MultiDiscrete(np.full((n,), space.n))
    if isinstance(space, MultiDiscrete):
        return MultiDiscrete(np.repeat(space.nvec[None], n, 0))
    if isinstance(space, Dict):
        return Dict(OrderedDict((k, batch_space(s, n)) for k, s in space.spaces.items()))
    raise TypeError(f"cannot batch {space}")


def from_external(space) -> Space:
    """Convert a gymnasium/gym space (duck-typed by class name) into the native space classes, so
    third-party envs (DMC, Crafter, DIAMBRA, MineDojo, MineRL) plug into the native wrappers."""
    name = type(space).__name__
    if isinstance(space, Space):
        return space
    if name == "Box":
        return Box(space.low, space.high, tuple(space.shape), space.dtype)
    if name == "Discrete":
        return Discrete(int(space.n))
    if name == "MultiDiscrete":
        return MultiDiscrete(list(np.asarray(space.nvec).tolist()))
    if name == "Dict":
        return Dict({k: from_external(v) for k, v in space.spaces.items()})
    raise TypeError(f"Unsupported external space: {space!r}")
