import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP kernels / RCCL)")
    config.addinivalue_line("markers", "slow: long-running integration test")
    config.addinivalue_line("markers", "benchmark: performance test")


@pytest.fixture(autouse=True)
def _chdir_tmp(tmp_path, monkeypatch, request):
    # runs write logs/ relative to cwd: keep them out of the repo
    if "no_chdir" not in request.keywords:
        monkeypatch.chdir(tmp_path)
    yield


@pytest.fixture(autouse=True)
def _gpu_teardown(request):
    """GPU tests: objects of a finished test (trainers hold reference cycles through their graphed
    step functions, so their captured hipGraphs, graph memory pools and tensors are otherwise freed
    by the cyclic GC at an arbitrary point of a LATER test) are collected while the device is idle."""
    yield
    if "gpu" in request.keywords:
        import gc

        import torch

        gc.collect()
        if torch.cuda.is_available():
            torch.cuda.synchronize()
            torch.cuda.empty_cache()


if os.environ.get("SRL_ANOMALY"):
    # diagnostics (scripts/diag_fault2.sh): a failing backward node reports the forward stack that made it
    import torch

    torch.autograd.set_detect_anomaly(True)
