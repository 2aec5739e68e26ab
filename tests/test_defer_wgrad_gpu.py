"""Deferred world-model parameter gradients (``ops/sidestream.py``) change WHEN the decoder / head weight
gradients run (beside the scan backward, on a side stream), not WHAT they compute: at the headline bench shape
the clipped gradient slab of the world model (= Adam's first moment after one step from a zero state) must match
with deferral on and off, eager and graph-replayed - to within the run-to-run spread of the in-line step itself (a
few float-atomic reductions make the step not bitwise reproducible) and 1e-5 of the slab's largest entry."""
import pytest
import torch

from tests.test_dv3_step_oracle_gpu import _build, _data, _state

pytestmark = pytest.mark.gpu


def test_deferred_wgrad_bit_identical():
    from sheeprl_prey_amd.ops import sidestream

    tr, opts, moments = _build([9])
    data = _data([9])
    tr.update_target(1.0)
    snap = {k: v.detach().clone() for k, v in _state(tr, opts, moments).items()}

    def restore():
        for k, v in _state(tr, opts, moments).items():
            v.copy_(snap[k])

    def run(enabled: bool, graphed: bool):
        restore()
        sidestream.ENABLED = enabled
        tr.graphed.enabled = graphed
        torch.cuda.manual_seed(5)
        out = tr.train_step(data)
        torch.cuda.synchronize()
        return float(out["Loss/world_model_loss"]), opts[0].exp_avg.clone()

    old = sidestream.ENABLED
    try:
        run(False, False)  # first step of the process: one-time workspace set-up (column-sum tickets, tuning)
        l_off, m_off = run(False, False)
        _, m_off2 = run(False, False)
        spread = float((m_off2 - m_off).abs().max())
        tol = max(4 * spread, 1e-5 * float(m_off.abs().max()))
        print("in-line run-to-run spread", spread, "tolerance", tol)
        l_on, m_on = run(True, False)
        assert l_on == l_off
        assert float((m_on - m_off).abs().max()) <= tol, float((m_on - m_off).abs().max())
        # graph-captured with deferral (2 warm-up steps, capture, replay)
        for _ in range(3):
            restore()
            sidestream.ENABLED = True
            tr.graphed.enabled = True
            tr.train_step(data)
        assert tr.graphed.graph is not None
        l_g, m_g = run(True, True)
        assert l_g == l_off
        assert float((m_g - m_off).abs().max()) <= tol, float((m_g - m_off).abs().max())
    finally:
        sidestream.ENABLED = old
        tr.graphed.enabled = True
