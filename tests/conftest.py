import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "vit-project_amd"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm MI355X GPU (run with -m gpu)")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
