import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the C ABI on the GPU)")


def _ensure_built():
    lib = os.path.join(ROOT, "jepsen", "etcd_amd", "liblincheck.so")
    orc = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(orc):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    if not os.path.exists(lib):
        subprocess.check_call(["make", "-s", "-j8", "-C",
                               os.path.join(ROOT, "jepsen", "etcd_amd", "csrc")])


_ensure_built()


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:  # noqa: BLE001
        return False


@pytest.fixture(scope="session")
def ctx():
    from jepsen.etcd_amd import abi
    c = abi.Context(device_mask=1)
    yield c
    c.close()
