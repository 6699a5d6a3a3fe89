"""pytest configuration: the `gpu` marker and shared fixtures.

CPU tests (-m "not gpu") cover the oracle against the reference's recorded
outputs, the host logic and the C ABI exports; GPU tests (-m gpu) are the
parity tests proper and run through the native libraries on an MI355X.
"""
import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libpinc_hip)")


@pytest.fixture(scope="session")
def built():
    import subprocess
    # torch (device memory for the kernel-level tests) brings up the HIP
    # runtime first, whichever test file runs first: with the native
    # library initialised before it, the process aborted at exit in the
    # runtimes' teardown (a double free after all tests had passed)
    import torch  # noqa: F401
    from pinc_amd.build import build
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle"), "-j4"], check=True)
    return build()
