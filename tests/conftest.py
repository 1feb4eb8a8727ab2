import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_addoption(parser):
    parser.addoption("--run-slow", action="store_true", default=False,
                     help="also run the tests marked slow (sanitizer builds of the native "
                          "engines; CI runs them, the default CPU run stays under 5 minutes)")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP) device")
    config.addinivalue_line("markers", "multiproc: spawns several gloo ranks on the CPU")
    config.addinivalue_line("markers", "slow: minutes of CPU (sanitizer builds); needs --run-slow")


def pytest_collection_modifyitems(config, items):
    if config.getoption("--run-slow") or os.environ.get("HIPSNAPSHOT_RUN_SLOW_TESTS") == "1":
        return
    skip = pytest.mark.skip(reason="slow: run with --run-slow")
    for item in items:
        if "slow" in item.keywords:
            item.add_marker(skip)


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
