"""Shared pytest setup.

``-m "not gpu"`` tests run anywhere (oracle vs golden fixtures, host logic, C-ABI exports).
``-m gpu`` tests need an MI355X and call the HIP path through the C ABI.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "cc-mpc_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests proper")
    if os.environ.get("CCMPC_SEGV_BT") == "1":      # debug aid: native backtrace on SIGSEGV
        import ctypes
        import faulthandler
        faulthandler.enable()
        ctypes.CDLL(os.path.join(ROOT, "tools", "libsegvbt.so")).segv_bt_install()


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    return load


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test collected on a host without a HIP device")
    return torch.device("cuda:0")
