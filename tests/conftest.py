import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP) device")
    config.addinivalue_line("markers", "multiproc: spawns several gloo ranks on the CPU")


@pytest.fixture(params=[True, False], ids=["batching", "no_batching"])
def toggle_batching(request):
    from hipsnapshot import knobs

    with knobs.override_is_batching_disabled(not request.param):
        yield request.param


@pytest.fixture
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from hipsnapshot.ops import native

    native.require_gpu_lib()
    return torch.device("cuda:0")
