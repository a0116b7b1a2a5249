import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


# The simd = 1 host API keeps small calls on the host (a GPU round trip costs
# more than the work).  The suite's small shapes are meant for the device
# kernels, so the tests switch that policy off; tests/test_host_fast.py covers
# the policy itself in child processes with the default environment.
os.environ.setdefault("VELES_HOST_SMALL_SCALE", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")
    # Build the native library once if this checkout does not have it yet.
    from veles.simd_amd import _lib, build
    if os.environ.get("VELES_SIMD_LIB"):
        # An explicit override is never rebuilt: fail fast and say which path.
        if not os.path.exists(_lib.LIB_PATH):
            raise pytest.UsageError(
                f"VELES_SIMD_LIB={_lib.LIB_PATH} does not exist")
    elif not os.path.exists(_lib.LIB_PATH):
        build.build()


def pytest_collection_modifyitems(config, items):
    from veles.simd_amd import _lib
    # A library that exists but does not load is a build error, never a
    # reason to skip the GPU tests (they would pass as "skipped").
    if os.path.exists(_lib.LIB_PATH) and not _lib.available():
        raise pytest.UsageError(f"native library failed to load: {_lib._load_error}")
    if _lib.gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU visible to the native library")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(autouse=True)
def _default_tuning_knobs():
    """Every test starts from and leaves behind the default tuning knobs
    (vs_tune_set is per thread; a test that fails between a set and its
    restore must not leak into the next test)."""
    yield
    from veles.simd_amd import _lib
    if _lib.available():
        _lib.lib().vs_tune_reset()
