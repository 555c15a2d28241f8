import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built libclipk.so")


@pytest.fixture(scope="session")
def dev():
    import torch
    assert torch.cuda.is_available(), "GPU test run without a visible GPU"
    from fsp_amd import _native
    _native.load()
    assert _native.load().clipk_device_arch_ok() == 1, "device 0 is not gfx950"
    return torch.device("cuda:0")
