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


@pytest.fixture(scope="module", params=["4-wave", "8-wave", "split", "split1"])
def kernel_instance(request):
    """Run a module's tests on every instance of the fused <= 32-atom flow
    kernel: the 4-wave throughput build (2 workgroups per CU, the one bench.py
    times), the 8-wave whole-tile latency build (enflow_latency.hip) and the
    feature-split latency build (enflow_split.hip: "split" two workgroups per
    molecule where they fit, else one; "split1" one workgroup per molecule; H =
    128 f16x3 inference only, other launches of these params run the 4-wave
    build), selected through the thresholds (0: never; 2^30: every batch).  The
    previous settings are restored afterwards."""
    from enflow_amd import _lib
    p = request.param
    prev = (_lib.set_latency_threshold(1 << 30 if p == "8-wave" else 0),
            _lib.set_split_threshold(1 << 30 if p == "split" else 0),
            _lib.set_fs_threshold(1 << 30 if p in ("split", "split1") else 0))
    yield p
    _lib.set_latency_threshold(-1 if prev[0] is None else prev[0])
    _lib.set_split_threshold(-1 if prev[1] is None else prev[1])
    _lib.set_fs_threshold(-1 if prev[2] is None else prev[2])
