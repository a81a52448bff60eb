import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")

# every model the tests build NaN-fills its workspace blocks on allocation and its output tensors
# (mlic_set_poison): a kernel that reads memory its producer never wrote, or leaves an output element
# unwritten, then fails the equality / finiteness checks instead of passing on stale data.
# MLIC_POISON=0 in the environment turns it off.
os.environ.setdefault("MLIC_POISON", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return np.load(os.path.join(GOLDEN, name), allow_pickle=False)
    return load
