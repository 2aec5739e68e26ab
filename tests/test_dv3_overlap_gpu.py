"""The DreamerV3 step with its actor phase on a side stream beside the critic phase (``DreamerV3Trainer.overlap_ac``,
the one-rank discrete default) against the same fused step with the two phases in line: the graph-replayed overlapped
step vs the eager in-line step, from the same weights, optimiser state, batch and random seed.  Same metrics and the
same updated parameters up to float-summation order (profiles/r5_ac_overlap.md)."""
import pytest
import torch

from tests.test_dv3_step_oracle_gpu import _build, _data, _rel, _state

pytestmark = pytest.mark.gpu


def test_overlapped_actor_critic_phases_match_in_line_step():
    from sheeprl_prey_amd.algos.dreamer_v3.dreamer_v3 import METRIC_KEYS

    adim = [9]
    tr, opts, moments = _build(adim)
    assert tr.overlap_ac and tr.graph_mode == "single"
    data = _data(adim)
    tr.update_target(1.0)
    snap = {k: v.detach().clone() for k, v in _state(tr, opts, moments).items()}
    for _ in range(3):  # 2 warm-up steps, then capture (+ one replay)
        tr.train_step(data)
    assert tr.graphed.graph is not None

    def restore():
        for k, v in _state(tr, opts, moments).items():
            v.copy_(snap[k])

    def run():
        restore()
        torch.cuda.manual_seed(5)
        out = {k: v.detach().clone() for k, v in tr.train_step(data).items()}
        torch.cuda.synchronize()
        return out, [o.flat_param.clone() for o in opts], [o.exp_avg.clone() for o in opts]

    out_on, p_on, m_on = run()  # graph replay, actor phase on the side stream
    tr.overlap_ac = False
    tr.graphed.enabled = False
    try:
        out_off, p_off, m_off = run()  # eager, phases in line
    finally:
        tr.overlap_ac = True
        tr.graphed.enabled = True
    for k in METRIC_KEYS:
        a, b = float(out_on[k]), float(out_off[k])
        assert abs(a - b) <= 1e-3 * max(abs(b), 1e-2), (k, a, b)
    for name, a, b in zip(("world_model", "actor", "critic"), m_on, m_off):
        assert _rel(a, b) < 1e-3, (name, _rel(a, b))
    for name, a, b in zip(("world_model", "actor", "critic"), p_on, p_off):
        assert _rel(a, b) < 1e-6, (name, _rel(a, b))
