import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")


def gpu_available():
    try:
        from blenderraytracer_amd import capi
        import ctypes as C
        lib = capi.load_library()
        n = C.c_int(0)
        return lib.rt_device_count(C.byref(n)) == 0 and n.value > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def lib():
    from blenderraytracer_amd import capi
    return capi.load_library()


@pytest.fixture(scope="session")
def gpu(lib):
    """On a GPU box the HIP path must be there: a missing device is a failure, not a skip."""
    if not gpu_available():
        pytest.fail("GPU test collected but no HIP device is visible to librt_hip.so")
    return lib
