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
    # no import-order workaround: pinc_amd loads its libraries RTLD_LOCAL
    # (pinc_amd/_lib.py), and tests/test_abi_gpu.py checks that a process
    # importing pinc_amd before torch exits cleanly
    from pinc_amd.build import build
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle"), "-j4"], check=True)
    out = build()
    # the checker's stencil and per-rank loops use the job's CPU share
    # (results are bit-identical for any thread count, oracle/orc.h)
    import orc
    orc.LIB.orc_set_threads(max(1, min(16, len(os.sched_getaffinity(0)))))
    return out
