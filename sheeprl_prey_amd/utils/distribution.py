"""Distributions used by the algorithms (reference: ``sheeprl/utils/distribution.py:25-398``).

``TwoHotEncodingDistribution`` routes ``log_prob`` / ``mean`` through the fused two-hot HIP
kernels; the others are thin, torch.distributions-compatible classes.
"""
from __future__ import annotations

import math
from numbers import Number
from typing import Callable, Optional

import torch
import torch.nn.functional as F
from torch import Tensor
from torch.distributions import Categorical, Distribution, constraints
from torch.distributions.kl import _kl_categorical_categorical, register_kl
from torch.distributions.utils import broadcast_all

from sheeprl_prey_amd import ops
from sheeprl_prey_amd.utils.utils import symexp, symlog

_LOG_SQRT_2PI_E = 0.5 * math.log(2.0 * math.pi * math.e)
_INV_SQRT_2PI = 1.0 / math.sqrt(2.0 * math.pi)


def _std_pdf(x: Tensor) -> Tensor:
    return torch.exp(-0.5 * x * x) * _INV_SQRT_2PI


def _finite_times(x: Tensor, y: Tensor) -> Tensor:
    """x * y with the x = +-inf, y = 0 products of unbounded tails taken as 0."""
    return torch.where(torch.isfinite(x), x * y, torch.zeros_like(y))


class TruncatedNormal(Distribution):
    """Normal(loc, scale) restricted to [low, high] (reference ``distribution.py:97-147``).

    Sampling is by inverse CDF: ``loc + scale * Phi^-1(Phi(alpha) + u Z)`` with ``u ~ U(eps, 1-eps)``,
    ``alpha = (low - loc) / scale``, ``Z = max(Phi(beta) - Phi(alpha), eps)`` (float32 eps), exactly the
    reference's semantics: the icdf argument is not clamped and samples are not clipped to the bounds.
    On the GPU ``rsample`` and ``log_prob`` are single fused HIP launches forward and backward
    (``csrc/truncnorm.hip``); moments, entropy and cdf are closed forms in eager torch.  Unlike the
    reference, the ``low < high`` check runs only with ``validate_args`` (it is a host sync)."""

    arg_constraints = {"loc": constraints.real, "scale": constraints.positive}
    has_rsample = True

    def __init__(self, loc, scale, low, high, validate_args=None):
        # the un-broadcast bounds go to the kernels (scalar bounds stay scalars)
        self._low_arg = low if isinstance(low, Tensor) else torch.as_tensor(float(low))
        self._high_arg = high if isinstance(high, Tensor) else torch.as_tensor(float(high))
        self.loc, self.scale, self.low, self.high = broadcast_all(loc, scale, low, high)
        batch_shape = torch.Size() if all(isinstance(v, Number) for v in (loc, scale, low, high)) else self.loc.size()
        super().__init__(batch_shape, validate_args=validate_args)
        if self.low.dtype != self.high.dtype:
            raise ValueError("Truncation bounds types are different")
        if validate_args and bool((self.low >= self.high).any()):
            raise ValueError("Incorrect truncation range")
        self._alpha = (self.low - self.loc) / self.scale
        self._beta = (self.high - self.loc) / self.scale

    # ---- standardised quantities
    @property
    def a(self) -> Tensor:
        return self._alpha

    @property
    def b(self) -> Tensor:
        return self._beta

    def _mass(self) -> Tensor:
        eps = torch.finfo(self.loc.dtype).eps
        return (self._phi_cdf(self._beta) - self._phi_cdf(self._alpha)).clamp_min(eps)

    @staticmethod
    def _phi_cdf(x: Tensor) -> Tensor:
        return 0.5 * (1.0 + torch.erf(x / math.sqrt(2.0)))

    @property
    def auc(self) -> Tensor:
        return self._mass()

    @constraints.dependent_property
    def support(self):
        return constraints.interval(self.low, self.high)

    # ---- moments / entropy (closed forms of the truncated normal)
    @property
    def mean(self) -> Tensor:
        return self.loc + self.scale * (_std_pdf(self._alpha) - _std_pdf(self._beta)) / self._mass()

    @property
    def variance(self) -> Tensor:
        Z = self._mass()
        pa, pb = _std_pdf(self._alpha), _std_pdf(self._beta)
        tail = (_finite_times(self._alpha, pa) - _finite_times(self._beta, pb)) / Z
        return self.scale**2 * (1.0 + tail - ((pa - pb) / Z) ** 2)

    def entropy(self) -> Tensor:
        Z = self._mass()
        tail = (_finite_times(self._beta, _std_pdf(self._beta)) - _finite_times(self._alpha, _std_pdf(self._alpha))) / Z
        return _LOG_SQRT_2PI_E + Z.log() - 0.5 * tail + self.scale.log()

    # ---- cdf / icdf / densities / samples
    def cdf(self, value: Tensor) -> Tensor:
        if self._validate_args:
            self._validate_sample(value)
        z = (value - self.loc) / self.scale
        return ((self._phi_cdf(z) - self._phi_cdf(self._alpha)) / self._mass()).clamp(0, 1)

    def icdf(self, value: Tensor) -> Tensor:
        return self.loc + self.scale * (math.sqrt(2.0) * torch.erfinv(2.0 * (self._phi_cdf(self._alpha) + value * self._mass()) - 1.0))

    def log_prob(self, value: Tensor) -> Tensor:
        if self._validate_args:
            self._validate_sample(value)
        lo, hi = self._bounds_for(value.device)
        return ops.truncnorm_log_prob(value, self.loc, self.scale, lo, hi)

    def rsample(self, sample_shape=torch.Size()) -> Tensor:
        shape = self._extended_shape(sample_shape)
        eps = torch.finfo(self.loc.dtype).eps
        u = torch.empty(shape, device=self.loc.device, dtype=self.loc.dtype).uniform_(eps, 1.0 - eps)
        loc, scale = self.loc.expand(shape), self.scale.expand(shape)
        lo, hi = self._bounds_for(self.loc.device)
        if lo.numel() != 1:
            lo, hi = self.low.expand(shape), self.high.expand(shape)
        return ops.truncnorm_rsample(loc, scale, lo, hi, u)

    def _bounds_for(self, device) -> tuple:
        lo, hi = self._low_arg, self._high_arg
        if lo.numel() == 1 and hi.numel() == 1:
            return lo.to(device=device, dtype=self.loc.dtype), hi.to(device=device, dtype=self.loc.dtype)
        return self.low, self.high


class TruncatedStandardNormal(TruncatedNormal):
    """Standard normal truncated to [a, b] (reference ``distribution.py:25-94``)."""

    def __init__(self, a, b, validate_args=None):
        a_t = a if isinstance(a, Tensor) else torch.as_tensor(float(a))
        super().__init__(torch.zeros_like(a_t, dtype=torch.get_default_dtype() if not a_t.is_floating_point() else a_t.dtype),
                         torch.ones_like(a_t, dtype=torch.get_default_dtype() if not a_t.is_floating_point() else a_t.dtype),
                         a, b, validate_args=validate_args)


class SymlogDistribution:
    """MSE/abs error in symlog space, summed over the event dims (reference ``distribution.py:152-193``)."""

    def __init__(self, mode: Tensor, dims: int, dist: str = "mse", agg: str = "sum", tol: float = 1e-8):
        self._mode = mode
        self._dims = tuple([-x for x in range(1, dims + 1)])
        self._dist = dist
        self._agg = agg
        self._tol = tol
        self._batch_shape = mode.shape[: len(mode.shape) - dims]
        self._event_shape = mode.shape[len(mode.shape) - dims :]

    @property
    def mode(self) -> Tensor:
        return symexp(self._mode)

    @property
    def mean(self) -> Tensor:
        return symexp(self._mode)

    def log_prob(self, value: Tensor) -> Tensor:
        assert self._mode.shape == value.shape, (self._mode.shape, value.shape)
        if self._dist == "mse":
            distance = (self._mode - symlog(value)) ** 2
        elif self._dist == "abs":
            distance = torch.abs(self._mode - symlog(value))
        else:
            raise NotImplementedError(self._dist)
        distance = torch.where(distance < self._tol, 0, distance)
        if self._agg == "mean":
            loss = distance.mean(self._dims)
        elif self._agg == "sum":
            loss = distance.sum(self._dims)
        else:
            raise NotImplementedError(self._agg)
        return -loss


class MSEDistribution:
    """Sum/mean squared error over the event dims (reference ``distribution.py:196-221``)."""

    def __init__(self, mode: Tensor, dims: int, agg: str = "sum"):
        self._mode = mode
        self._dims = tuple([-x for x in range(1, dims + 1)])
        self._agg = agg
        self._batch_shape = mode.shape[: len(mode.shape) - dims]
        self._event_shape = mode.shape[len(mode.shape) - dims :]

    @property
    def mode(self) -> Tensor:
        return self._mode

    @property
    def mean(self) -> Tensor:
        return self._mode

    def log_prob(self, value: Tensor) -> Tensor:
        assert self._mode.shape == value.shape, (self._mode.shape, value.shape)
        distance = (self._mode - value) ** 2
        if self._agg == "mean":
            return -distance.mean(self._dims)
        if self._agg == "sum":
            return -distance.sum(self._dims)
        raise NotImplementedError(self._agg)


class TwoHotEncodingDistribution:
    """Two-hot distribution over ``num_bins`` symlog-spaced bins (reference ``distribution.py:224-270``).

    ``dims=1``: ``logits [..., K]``, ``log_prob(x [..., 1]) -> [...]``, ``mean -> [..., 1]``.
    Both run as single fused kernels on GPU."""

    def __init__(self, logits: Tensor, dims: int = 0, low: int = -20, high: int = 20,
                 transfwd: Callable[[Tensor], Tensor] = symlog, transbwd: Callable[[Tensor], Tensor] = symexp):
        self.logits = logits
        self.dims = tuple([-x for x in range(1, dims + 1)])
        self.low = low
        self.high = high
        self.transfwd = transfwd
        self.transbwd = transbwd
        self._batch_shape = logits.shape[: len(logits.shape) - dims]
        self._event_shape = logits.shape[len(logits.shape) - dims : -1] + (1,)

    @property
    def probs(self) -> Tensor:
        return F.softmax(self.logits, dim=-1)

    @property
    def bins(self) -> Tensor:
        return ops.twohot_bins(self.logits.shape[-1], self.low, self.high, device=self.logits.device)

    @property
    def mean(self) -> Tensor:
        if self.transbwd is symexp and len(self.dims) == 1:
            return ops.twohot_mean(self.logits, self.low, self.high)
        return self.transbwd((self.probs * self.bins).sum(dim=self.dims, keepdim=True))

    @property
    def mode(self) -> Tensor:
        return self.mean

    def log_prob(self, x: Tensor) -> Tensor:
        if self.transfwd is symlog and len(self.dims) == 1:
            return -ops.twohot_nll(self.logits, x, self.low, self.high)
        # generic transform: two-hot target built on transfwd(x) (reference semantics)
        x = self.transfwd(x)
        bins = self.bins
        K = bins.numel()
        below = ((bins <= x).to(torch.int32).sum(-1, keepdim=True) - 1).clamp(0, K - 1).long()
        above = (K - (bins > x).to(torch.int32).sum(-1, keepdim=True)).clamp(0, K - 1).long()
        equal = below == above
        d_b = torch.where(equal, torch.ones_like(x), (bins[below] - x).abs())
        d_a = torch.where(equal, torch.ones_like(x), (bins[above] - x).abs())
        tot = d_b + d_a
        target = F.one_hot(below, K) * (d_a / tot)[..., None] + F.one_hot(above, K) * (d_b / tot)[..., None]
        log_pred = self.logits - torch.logsumexp(self.logits, dim=-1, keepdim=True)
        return (target.squeeze(-2) * log_pred).sum(dim=self.dims)


class OneHotCategoricalValidateArgs(Distribution):
    """One-hot categorical with ``validate_args`` plumbing (reference ``distribution.py:275-377``)."""

    arg_constraints = {"probs": constraints.simplex, "logits": constraints.real_vector}
    support = constraints.one_hot
    has_enumerate_support = True

    def __init__(self, probs=None, logits=None, validate_args=None):
        self._categorical = Categorical(probs, logits, validate_args=validate_args)
        batch_shape = self._categorical.batch_shape
        event_shape = self._categorical.param_shape[-1:]
        super().__init__(batch_shape, event_shape, validate_args=validate_args)

    def expand(self, batch_shape, _instance=None):
        new = self._get_checked_instance(OneHotCategoricalValidateArgs, _instance)
        batch_shape = torch.Size(batch_shape)
        new._categorical = self._categorical.expand(batch_shape)
        super(OneHotCategoricalValidateArgs, new).__init__(batch_shape, self.event_shape, validate_args=False)
        new._validate_args = self._validate_args
        return new

    def _new(self, *args, **kwargs):
        return self._categorical._new(*args, **kwargs)

    @property
    def _param(self):
        return self._categorical._param

    @property
    def probs(self):
        return self._categorical.probs

    @property
    def logits(self):
        return self._categorical.logits

    @property
    def mean(self):
        return self._categorical.probs

    @property
    def mode(self):
        probs = self._categorical.probs
        return F.one_hot(probs.argmax(dim=-1), num_classes=probs.shape[-1]).to(probs)

    @property
    def variance(self):
        return self._categorical.probs * (1 - self._categorical.probs)

    @property
    def param_shape(self):
        return self._categorical.param_shape

    def sample(self, sample_shape=torch.Size()):
        sample_shape = torch.Size(sample_shape)
        probs = self._categorical.probs
        indices = self._categorical.sample(sample_shape)
        return F.one_hot(indices, self._categorical._num_events).to(probs)

    def log_prob(self, value):
        if self._validate_args:
            self._validate_sample(value)
        return self._categorical.log_prob(value.max(-1)[1])

    def entropy(self):
        return self._categorical.entropy()

    def enumerate_support(self, expand=True):
        n = self.event_shape[0]
        values = torch.eye(n, dtype=self._param.dtype, device=self._param.device)
        values = values.view((n,) + (1,) * len(self.batch_shape) + (n,))
        if expand:
            values = values.expand((n,) + self.batch_shape + (n,))
        return values


class OneHotCategoricalStraightThroughValidateArgs(OneHotCategoricalValidateArgs):
    """Reparameterised one-hot categorical: ``rsample = sample + p - sg(p)`` (reference ``:380-393``)."""

    has_rsample = True

    def rsample(self, sample_shape=torch.Size()):
        samples = self.sample(sample_shape)
        probs = self._categorical.probs
        return samples + (probs - probs.detach())


@register_kl(OneHotCategoricalValidateArgs, OneHotCategoricalValidateArgs)
def _kl_onehot_onehot(p, q):
    return _kl_categorical_categorical(p._categorical, q._categorical)


class BernoulliSafeMode(torch.distributions.Bernoulli):
    @property
    def mode(self):
        return (self.probs > 0.5).to(self.probs)
