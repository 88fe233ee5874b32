"""pytest configuration: the `gpu` marker and import paths.

`-m "not gpu"` (CPU container): oracle-vs-golden/KAT tests, host logic, and the
C-ABI library's symbol table.  `-m gpu` (MI355X box): parity of the HIP path
against the oracle and the golden fixtures, through the C-ABI.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "oracle"), os.path.join(ROOT, "quill-zkvm_amd"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); runs the gfx950 kernels")


@pytest.fixture(scope="session")
def dev():
    import quill_amd
    d = quill_amd.Device(0)
    yield d
    d.close()
