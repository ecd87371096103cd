"""pytest configuration: the `gpu` marker and import paths.

`-m "not gpu"` tests run anywhere (oracle vs golden vectors, host logic, C-ABI symbols,
kernel-algorithm emulation, gloo multi-rank); `-m gpu` tests call the HIP engine through
the C-ABI on a real MI355X and compare with the oracle.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "open-rdma-driver_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")


def gpu_available() -> bool:
    try:
        import icrc_amd

        return icrc_amd.device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def engine():
    import icrc_amd

    if icrc_amd.device_count() <= 0:
        pytest.fail("gpu test selected but no GPU is visible to the ICRC engine")
    e = icrc_amd.Engine(0)
    yield e
    e.close()


@pytest.fixture(scope="session")
def ab_engine():
    """An engine of the A/B library (diagnostics), for the variant-validation test."""
    import icrc_amd

    if icrc_amd.device_count() <= 0:
        pytest.fail("gpu test selected but no GPU is visible to the ICRC engine")
    e = icrc_amd.Engine(0, lib=icrc_amd.ab_library())
    yield e
    e.close()

