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


@pytest.fixture(scope="module", params=["4-wave", "8-wave", "coop"])
def kernel_instance(request):
    """Run a module's tests on the three instances of the fused <= 32-atom flow
    kernel: the 4-wave throughput build (2 workgroups per CU, the one bench.py
    times), the 8-wave latency build (enflow_latency.hip) and the cooperative
    build (enflow_coop.hip: two 8-wave workgroups per molecule; inference
    launches of default-flag layers, batches small enough for a cooperative
    launch -- others fall back to the 8-wave build), selected through the
    latency threshold and the cooperative limit (0: never; 2^30: every batch).
    The previous settings are restored afterwards."""
    from enflow_amd import _lib
    prev = _lib.set_latency_threshold(0 if request.param == "4-wave" else 1 << 30)
    prev_c = _lib.set_coop_max(1 << 30 if request.param == "coop" else 0)
    yield request.param
    _lib.set_latency_threshold(-1 if prev is None else prev)
    _lib.set_coop_max(-1 if prev_c is None else prev_c)
