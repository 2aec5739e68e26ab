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
