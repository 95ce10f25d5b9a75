import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "consistent-viterbi_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device; runs the HIP kernels")


def _build_once():
    import __graft_entry__ as g

    g.build()


@pytest.fixture(scope="session", autouse=True)
def built():
    _build_once()


def has_gpu():
    try:
        import cviterbi._lib as L

        return L.lib().cv_device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    if not has_gpu():
        pytest.fail("GPU test selected but no HIP device is visible")
    return 0


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}
