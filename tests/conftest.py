import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built HIP library")
    config.addinivalue_line("markers", "slow: long-running CPU test")


import pytest  # noqa: E402


@pytest.fixture(scope="module", params=["4-wave", "8-wave"])
def kernel_instance(request):
    """Run a module's tests on both instances of the fused <= 32-atom flow
    kernel: the 4-wave throughput build (2 workgroups per CU, the one bench.py
    times) and the 8-wave latency build (enflow_latency.hip), selected through
    the latency threshold (0: never the latency build; 2^30: every batch).
    The previous setting is restored afterwards."""
    from enflow_amd import _lib
    prev = _lib.set_latency_threshold(0 if request.param == "4-wave" else 1 << 30)
    yield request.param
    _lib.set_latency_threshold(-1 if prev is None else prev)
