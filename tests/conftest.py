import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "hockey-env_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (run with -m gpu on the MI355X box)")
    config.addinivalue_line("markers", "slow: longer statistical test")


@pytest.fixture(scope="session")
def oracle():
    import oracle as O  # noqa: E402  (tests/ is allowed to load the checker)
    O.build()
    return O


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    cache = {}

    def load(name):
        if name not in cache:  # NpzFile re-decompresses on every key access: materialise once
            with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
                cache[name] = {k: z[k] for k in z.files}
        return cache[name]

    return load
