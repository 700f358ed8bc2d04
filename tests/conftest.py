import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden():
    import json

    import numpy as np

    d = os.path.join(ROOT, "tests", "golden")
    cases = np.load(os.path.join(d, "cases.npz"), allow_pickle=False)
    with open(os.path.join(d, "meta.json")) as f:
        meta = json.load(f)
    return cases, meta


@pytest.fixture(scope="session")
def golden_blocks():
    """Reference outputs for block sizes 6, 10, 12, 14 (gen_golden.py --blocks)."""
    import json

    import numpy as np

    d = os.path.join(ROOT, "tests", "golden")
    cases = np.load(os.path.join(d, "cases_blocks.npz"), allow_pickle=False)
    with open(os.path.join(d, "meta_blocks.json")) as f:
        meta = json.load(f)
    return cases, meta


@pytest.fixture(scope="session")
def golden_alpha():
    """Reference outputs across the app's alpha slider, up to 1.0 (gen_golden.py --alpha)."""
    import json

    import numpy as np

    d = os.path.join(ROOT, "tests", "golden")
    cases = np.load(os.path.join(d, "cases_alpha.npz"), allow_pickle=False)
    with open(os.path.join(d, "meta_alpha.json")) as f:
        meta = json.load(f)
    return cases, meta


@pytest.fixture(scope="session")
def stages():
    import numpy as np

    return np.load(os.path.join(ROOT, "tests", "golden", "stages.npz"), allow_pickle=False)
