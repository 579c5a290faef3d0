import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the C ABI on the GPU)")


def _built_id(lib):
    """The build id baked into the library file, read without loading it
    (loading it here would bring up its HIP runtime before torch's)."""
    import re
    try:
        m = re.search(rb"LC_BUILD_ID:([0-9a-f]{16})", open(lib, "rb").read())
    except OSError:
        return None
    return m.group(1).decode() if m else None


def _ensure_built():
    """Build whatever is missing or stale: the oracle's make is incremental;
    the HIP library is rebuilt when its lc_build_id() differs from this
    tree's sources (abi.lib() refuses a mismatch anyway, so a stale binary
    can never be tested)."""
    sys.path.insert(0, ROOT)
    from jepsen.etcd_amd import abi
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    if os.environ.get("LINCHECK_LIB"):  # a dev A/B build (tools/build_variants.sh): test it as is
        return
    if _built_id(abi.LIB_PATH) != abi.source_build_id():
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
