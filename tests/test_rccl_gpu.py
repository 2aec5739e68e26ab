"""RCCL on the real device (one rank: the multi-GPU runs are the driver's).  Every case runs in its own
child process (``tests/rccl_child.py``): a process-group abort fails that case, not the GPU suite.

The framework's gradient collectives - the bucketed flat-slab all-reduce, the per-bucket all-reduce
launched from post-accumulate-grad hooks, the all-gather of the DreamerV3 lambda path - and the segmented
DreamerV3 step (one hipGraph per phase, collectives eagerly between replays, the N>1 default) over a
1-rank ``nccl`` (= RCCL) group; the optimiser / trainer is told there are 2 ranks so the multi-rank
code paths run."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("case", ["flat_slab_all_reduce_and_overlap", "all_gather_into_tensor",
                                  "hooks_silent_inside_capture", "dv3_segmented_step"])
def test_rccl_case(case):
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["PYTHONUNBUFFERED"] = "1"
    r = subprocess.run([sys.executable, os.path.join(HERE, "rccl_child.py"), case], capture_output=True, text=True,
                       timeout=300, env=env, cwd=os.path.dirname(HERE))
    tail = (r.stdout[-3000:] + "\n--- stderr ---\n" + r.stderr[-6000:])
    assert r.returncode == 0 and f"__RCCL_CASE_OK__ {case}" in r.stdout, f"rc={r.returncode}\n{tail}"
