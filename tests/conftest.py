import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

_LIB = os.path.join(ROOT, "udpdk_amd", "libudpdk_amd.so")
_ORACLE = os.path.join(ROOT, "oracle", "liboracle.so")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")
    # build the libraries once if they are missing (the driver normally runs build() first)
    if not (os.path.exists(_LIB) and os.path.exists(_ORACLE)):
        subprocess.run(["make", "-j8"], cwd=ROOT, check=True)


def _gpu_count() -> int:
    try:
        from udpdk_amd import abi
        return abi.device_count()
    except Exception:
        return 0


@pytest.fixture(scope="session")
def gpu_ctx():
    from udpdk_amd import abi
    if _gpu_count() < 1:
        pytest.fail("GPU test selected but no GPU is visible to libudpdk_amd.so")
    ctx = abi.GpuContext(0, max_frames=1 << 22, max_lanes=4096)
    yield ctx
    ctx.close()


@pytest.fixture()
def host_api():
    from udpdk_amd import abi
    api = abi.HostApi()
    api.reset()
    yield api
    api.reset()
