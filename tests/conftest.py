"""pytest configuration: the `gpu` marker and shared helpers.

`-m "not gpu"` (CPU container): oracle vs golden vectors, host logic, the
C-ABI library's exports, gloo multi-process tests.  `-m gpu` (MI355X box):
parity of the HIP path against the oracle through the C ABI.  GPU tests FAIL
(never skip) when no device is visible, so a silent CPU run cannot pass them.
"""
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "oracle"), str(ROOT / "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests of the HIP path")


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a HIP device (wireglider_amd has no CPU path)")
    import wireglider_amd as wga

    assert wga.device_count() > 0
    return torch.device("cuda:0")
