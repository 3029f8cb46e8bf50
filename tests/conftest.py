import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long running")


@pytest.fixture
def cpu_config():
    from systemml_amd.conf import DMLConfig
    return DMLConfig(gpu=False)


@pytest.fixture
def gpu_config():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from systemml_amd.conf import DMLConfig
    return DMLConfig(gpu=True, precision="single")


@pytest.fixture(autouse=True)
def _isolated_cwd(tmp_path, monkeypatch):
    """Scripts write their $-named outputs relative to the working directory; keep them
    out of the repository."""
    monkeypatch.chdir(tmp_path)
