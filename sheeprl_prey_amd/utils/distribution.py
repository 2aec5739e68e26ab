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

CONST_SQRT_2 = math.sqrt(2)
CONST_INV_SQRT_2PI = 1 / math.sqrt(2 * math.pi)
CONST_INV_SQRT_2 = 1 / math.sqrt(2)
CONST_LOG_INV_SQRT_2PI = math.log(CONST_INV_SQRT_2PI)
CONST_LOG_SQRT_2PI_E = 0.5 * math.log(2 * math.pi * math.e)


class TruncatedStandardNormal(Distribution):
    """Standard normal truncated to [a, b]; rsample by inverse CDF (erfinv)."""

    arg_constraints = {"a": constraints.real, "b": constraints.real}
    has_rsample = True
    eps = 1e-6

    def __init__(self, a, b, validate_args=None):
        self.a, self.b = broadcast_all(a, b)
        batch_shape = torch.Size() if isinstance(a, Number) and isinstance(b, Number) else self.a.size()
        super().__init__(batch_shape, validate_args=validate_args)
        if self.a.dtype != self.b.dtype:
            raise ValueError("Truncation bounds types are different")
        if any((self.a >= self.b).view(-1).tolist()) if validate_args else False:
            raise ValueError("Incorrect truncation range")
        eps = torch.finfo(self.a.dtype).eps
        self._dtype_min_gt_0 = eps
        self._dtype_max_lt_1 = 1 - eps
        self._little_phi_a = self._little_phi(self.a)
        self._little_phi_b = self._little_phi(self.b)
        self._big_phi_a = self._big_phi(self.a)
        self._big_phi_b = self._big_phi(self.b)
        self._Z = (self._big_phi_b - self._big_phi_a).clamp(eps, 1 - eps)
        self._log_Z = self._Z.log()
        little_phi_coeff_a = torch.nan_to_num(self.a, nan=math.nan)
        little_phi_coeff_b = torch.nan_to_num(self.b, nan=math.nan)
        self._lpbb_m_lpaa_d_Z = (self._little_phi_b * little_phi_coeff_b - self._little_phi_a * little_phi_coeff_a) / self._Z
        self._mean = -(self._little_phi_b - self._little_phi_a) / self._Z
        self._variance = 1 - self._lpbb_m_lpaa_d_Z - ((self._little_phi_b - self._little_phi_a) / self._Z) ** 2
        self._entropy = CONST_LOG_SQRT_2PI_E + self._log_Z - 0.5 * self._lpbb_m_lpaa_d_Z

    @constraints.dependent_property
    def support(self):
        return constraints.interval(self.a, self.b)

    @property
    def mean(self):
        return self._mean

    @property
    def variance(self):
        return self._variance

    def entropy(self):
        return self._entropy

    @property
    def auc(self):
        return self._Z

    @staticmethod
    def _little_phi(x):
        return (-(x**2) * 0.5).exp() * CONST_INV_SQRT_2PI

    @staticmethod
    def _big_phi(x):
        phi = 0.5 * (1 + (x * CONST_INV_SQRT_2).erf())
        return phi.clamp(TruncatedStandardNormal.eps, 1 - TruncatedStandardNormal.eps)

    @staticmethod
    def _inv_big_phi(x):
        return CONST_SQRT_2 * (2 * x - 1).erfinv()

    def cdf(self, value):
        if self._validate_args:
            self._validate_sample(value)
        return ((self._big_phi(value) - self._big_phi_a) / self._Z).clamp(0, 1)

    def icdf(self, value):
        y = self._big_phi_a + value * self._Z
        y = y.clamp(self.eps, 1 - self.eps)
        return self._inv_big_phi(y)

    def log_prob(self, value):
        if self._validate_args:
            self._validate_sample(value)
        return CONST_LOG_INV_SQRT_2PI - self._log_Z - (value**2) * 0.5

    def rsample(self, sample_shape=torch.Size()):
        shape = self._extended_shape(sample_shape)
        p = torch.empty(shape, device=self.a.device).uniform_(self._dtype_min_gt_0, self._dtype_max_lt_1)
        return self.icdf(p)


class TruncatedNormal(TruncatedStandardNormal):
    """Normal(loc, scale) truncated to [a, b] (reference ``distribution.py:97-147``)."""

    has_rsample = True

    def __init__(self, loc, scale, a, b, validate_args=None):
        self.loc, self.scale, a, b = broadcast_all(loc, scale, a, b)
        self._non_std_a = a
        self._non_std_b = b
        a = (a - self.loc) / self.scale
        b = (b - self.loc) / self.scale
        super().__init__(a, b, validate_args=validate_args)
        self._log_scale = self.scale.log()
        self._mean = self._mean * self.scale + self.loc
        self._variance = self._variance * self.scale**2
        self._entropy = self._entropy + self._log_scale

    def _to_std_rv(self, value):
        return (value - self.loc) / self.scale

    def _from_std_rv(self, value):
        return value * self.scale + self.loc

    def cdf(self, value):
        return super().cdf(self._to_std_rv(value))

    def icdf(self, value):
        sample = self._from_std_rv(super().icdf(value))
        clipped = torch.max(torch.min(sample, self._non_std_b), self._non_std_a)
        return sample + (clipped - sample).detach()

    def log_prob(self, value):
        value = self._to_std_rv(value)
        if self._validate_args:
            self._validate_sample(value)
        return super().log_prob(value) - self._log_scale


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
