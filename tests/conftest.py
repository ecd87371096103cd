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


# Kernel variants only the A/B library accepts (libicrc_amd_ab.so, built with ICRC_AB_BUILD): the
# quad kernels (result-exact, kept for A/B) and their hybrid forms.  Diagnostics (wrong results by
# design) are not listed: no parity test runs them.
AB_ONLY_VARIANTS = {20, 24, 25, 26, 120, 124, 125, 126, 220, 224, 225, 226}


@pytest.fixture(scope="session")
def ab_engine():
    """An engine of the A/B library (quad kernels + diagnostics), for the A/B variants' parity."""
    import icrc_amd

    if icrc_amd.device_count() <= 0:
        pytest.fail("gpu test selected but no GPU is visible to the ICRC engine")
    e = icrc_amd.Engine(0, lib=icrc_amd.ab_library())
    yield e
    e.close()


def engine_for(variant, engine, ab_engine):
    return ab_engine if variant in AB_ONLY_VARIANTS else engine
