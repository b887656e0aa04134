import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def golden():
    import json

    import numpy as np

    gdir = os.path.join(ROOT, "tests", "golden")
    with open(os.path.join(gdir, "golden_v1.json")) as f:
        manifest = json.load(f)
    arrays = np.load(os.path.join(gdir, "golden_v1.npz"), allow_pickle=False)
    return manifest, arrays
