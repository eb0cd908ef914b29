import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device) and libhorreum_gpu.so")


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "format_vectors.json"), encoding="utf-8") as f:
        return json.load(f)["cases"]


@pytest.fixture(scope="session")
def engine():
    from horreum_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()
