import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


# torch (device tensors for the device-pointer entry points) bundles its own HIP runtime
# under the same soname as /opt/rocm's; load it before liborbslam_gpu.so so that both use
# torch's copy, as bench.py does (the library only needs the soname).
try:
    import torch  # noqa: F401,E402
except Exception:  # pragma: no cover
    torch = None


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP library)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def _ensure_built():
    lib = ROOT / "c_orb_slam_amd" / "liborbslam_gpu.so"
    orc = ROOT / "oracle" / "liborb_oracle.so"
    if not orc.exists():
        subprocess.run(["make", "-s", "-C", str(ROOT / "oracle")], check=True)
    if not lib.exists():
        subprocess.run(["make", "-s", "-C", str(ROOT), "lib"], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def gpu():
    import c_orb_slam_amd as orb
    assert orb.device_available(), "GPU test collected on a machine without a HIP device"
    return orb
