"""pytest configuration: the `gpu` marker and the CPU oracle build (test infrastructure)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, TESTS):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP library's C ABI)")


@pytest.fixture(scope="session", autouse=True)
def oracle_built():
    """Build oracle/_build/*.so when absent (gcc only; the product never links these)."""
    so = os.path.join(ROOT, "oracle", "_build", "libkb_oracle.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    return so
