"""TruncatedNormal (K16): parity with the reference class and the fused HIP kernels vs the eager oracle.

Parity is pinned against the reference's own implementation (``sheeprl/utils/distribution.py:25-147``),
loaded straight from the read-only reference tree with its one package import stubbed; the test skips
when that tree is absent (e.g. on a GPU box)."""
import importlib.util
import math
import os
import sys
import types

import pytest
import torch

from sheeprl_prey_amd import ops
from sheeprl_prey_amd.ops import reference as ref
from sheeprl_prey_amd.utils.distribution import TruncatedNormal, TruncatedStandardNormal

REF = "/root/reference/sheeprl/utils/distribution.py"


def _reference_module():
    if not os.path.exists(REF):
        pytest.skip("reference tree not available")
    stub = types.ModuleType("sheeprl.utils.utils")
    stub.symlog = lambda x: torch.sign(x) * torch.log1p(x.abs())
    stub.symexp = lambda x: torch.sign(x) * (torch.exp(x.abs()) - 1)
    saved = {k: sys.modules.get(k) for k in ("sheeprl", "sheeprl.utils", "sheeprl.utils.utils")}
    sys.modules.update({"sheeprl": types.ModuleType("sheeprl"), "sheeprl.utils": types.ModuleType("sheeprl.utils"),
                        "sheeprl.utils.utils": stub})
    try:
        spec = importlib.util.spec_from_file_location("_ref_distribution", REF)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    return mod


def _params(n=64, seed=0, device="cpu"):
    g = torch.Generator().manual_seed(seed)
    loc = torch.tanh(torch.randn(n, 3, generator=g) * 2)
    scale = 2 * torch.sigmoid(torch.randn(n, 3, generator=g) / 2) + 0.1
    return loc.to(device), scale.to(device)


def test_matches_reference_class():
    R = _reference_module()
    loc, scale = _params()
    lo, hi = torch.tensor(-1.0), torch.tensor(1.0)
    mine = TruncatedNormal(loc, scale, lo, hi)
    theirs = R.TruncatedNormal(loc, scale, lo, hi)
    for name in ("mean", "variance"):
        torch.testing.assert_close(getattr(mine, name), getattr(theirs, name), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(mine.entropy(), theirs.entropy(), rtol=1e-5, atol=1e-6)
    u = torch.rand(loc.shape) * 0.98 + 0.01
    torch.testing.assert_close(mine.icdf(u), theirs.icdf(u), rtol=1e-5, atol=1e-6)
    v = torch.rand(loc.shape) * 1.8 - 0.9
    torch.testing.assert_close(mine.log_prob(v), theirs.log_prob(v), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(mine.cdf(v), theirs.cdf(v), rtol=1e-5, atol=1e-6)
    std_m, std_r = TruncatedStandardNormal(-0.5, 2.0), R.TruncatedStandardNormal(-0.5, 2.0)
    torch.testing.assert_close(std_m.mean, std_r.mean)
    torch.testing.assert_close(std_m.entropy(), std_r.entropy())


def test_gradients_match_reference_class():
    R = _reference_module()
    loc, scale = _params(seed=1)
    lo, hi = torch.tensor(-1.0), torch.tensor(1.0)
    u = torch.rand(loc.shape) * 0.98 + 0.01
    v = torch.rand(loc.shape) * 1.8 - 0.9
    grads = []
    for cls in (TruncatedNormal, R.TruncatedNormal):
        l, s = loc.clone().requires_grad_(), scale.clone().requires_grad_()
        d = cls(l, s, lo, hi)
        (d.icdf(u).sum() + d.log_prob(v).sum() + d.entropy().sum()).backward()
        grads.append((l.grad, s.grad))
    torch.testing.assert_close(grads[0][0], grads[1][0], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(grads[0][1], grads[1][1], rtol=1e-4, atol=1e-5)


def test_rsample_inside_bounds_and_moments():
    torch.manual_seed(0)
    loc = torch.full((200000,), 0.7)
    scale = torch.full((200000,), 0.5)
    d = TruncatedNormal(loc, scale, torch.tensor(-1.0), torch.tensor(1.0))
    x = d.rsample()
    assert float(x.min()) >= -1.0 - 1e-6 and float(x.max()) <= 1.0 + 1e-6
    assert abs(float(x.mean()) - float(d.mean[0])) < 5e-3
    assert abs(float(x.var()) - float(d.variance[0])) < 5e-3
    # the density integrates to one over the support
    grid = torch.linspace(-1, 1, 20001)
    dens = TruncatedNormal(torch.tensor(0.7), torch.tensor(0.5), -1.0, 1.0).log_prob(grid).exp()
    assert abs(float(torch.trapz(dens, grid)) - 1.0) < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("n", [7, 4096])
def test_truncnorm_kernels_match_oracle(n):
    assert ops.native_available()
    loc, scale = _params(n=n, seed=3, device="cuda")
    loc[:5] = torch.tensor([0.999, -0.999, 0.0, 0.5, -0.3], device="cuda")[: min(5, n)].unsqueeze(-1)  # near-bound means
    scale[:3] = 1e-3  # tiny scales: the mass clamp path
    lo, hi = torch.tensor(-1.0, device="cuda"), torch.tensor(1.0, device="cuda")
    u = torch.rand(loc.shape, device="cuda") * 0.998 + 0.001
    g = torch.randn(loc.shape, device="cuda")
    out, grads = [], []
    for fn in (ops.truncnorm_rsample, ref.truncnorm_rsample):
        l, s = loc.clone().requires_grad_(), scale.clone().requires_grad_()
        x = fn(l, s, lo, hi, u)
        (x * g).sum().backward()
        out.append(x.detach())
        grads.append((l.grad, s.grad))
    torch.testing.assert_close(out[0], out[1], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(grads[0][0], grads[1][0], rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(grads[0][1], grads[1][1], rtol=1e-3, atol=1e-4)
    # log-density with a leading sample dimension broadcast over the parameters
    v = (torch.rand(5, *loc.shape, device="cuda") * 1.8 - 0.9)
    g = torch.randn(v.shape, device="cuda")
    out, grads = [], []
    for fn in (ops.truncnorm_log_prob, ref.truncnorm_log_prob):
        vv, l, s = v.clone().requires_grad_(), loc.clone().requires_grad_(), scale.clone().requires_grad_()
        lp = fn(vv, l, s, lo, hi)
        (lp * g).sum().backward()
        out.append(lp.detach())
        grads.append((vv.grad, l.grad, s.grad))
    torch.testing.assert_close(out[0], out[1], rtol=1e-4, atol=1e-3)
    for a, b in zip(*grads):
        torch.testing.assert_close(a, b, rtol=1e-3, atol=1e-2)


@pytest.mark.gpu
def test_truncnorm_distribution_uses_kernels():
    from sheeprl_prey_amd.ops import _TruncNormRsample, _TruncNormLogProb  # noqa: F401

    loc, scale = _params(n=32, device="cuda")
    d = TruncatedNormal(loc.requires_grad_(), scale, torch.tensor(-1.0, device="cuda"), torch.tensor(1.0, device="cuda"))
    x = d.rsample()
    assert type(x.grad_fn).__name__ == "_TruncNormRsampleBackward"
    assert type(d.log_prob(x).grad_fn).__name__ == "_TruncNormLogProbBackward"
    assert math.isfinite(float(d.entropy().sum()))
