import os
import subprocess
import sys

import numpy as np
import pytest

try:  # torch first: one HIP runtime per process (see quadruped_pympc_amd/_lib.py)
    import torch  # noqa: F401
except ImportError:  # pragma: no cover
    torch = None

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "quadruped-pympc-tamols_amd")
for p in (PKG_DIR, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

# Build the native artifacts when they are missing (they normally ship prebuilt to the GPU box).
if not os.path.exists(os.path.join(PKG_DIR, "quadruped_pympc_amd", "libsrbd_hip.so")):
    subprocess.run(["make", "-j8", "-C", PKG_DIR], check=True)
if not os.path.exists(os.path.join(ROOT, "oracle", "libsrbd_oracle.so")):
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "libsrbd_oracle.so"], check=True)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture
def rng():
    return np.random.default_rng(12345)
