import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

REFERENCE = "/root/reference"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X GPU (HIP kernels, RCCL)")
    config.addinivalue_line("markers", "slow: long-running test")


def has_gpu():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if has_gpu():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture
def manager(tmp_path):
    from katib_amd.controller.manager import Manager

    m = Manager(state_dir=str(tmp_path / "state"), num_devices=0, journal=False)
    m.config.amd.warm_workers = True
    yield m
    m.shutdown()


@pytest.fixture
def gpu_manager(tmp_path):
    from katib_amd.controller.manager import Manager

    m = Manager(state_dir=str(tmp_path / "state"), journal=False)
    yield m
    m.shutdown()
