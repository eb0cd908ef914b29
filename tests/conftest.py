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
    if os.environ.get("HG_TEST_POISON") == "1":
        # every new device buffer of the library filled with 0xA5: a read of
        # memory no call wrote cannot pass on zero-filled fresh pages
        from horreum_amd import abi
        abi.set_knob("HG_DEBUG_POISON", 1)
    e = Engine(0)
    yield e
    e.close()


@pytest.fixture
def knobs():
    """knobs(name, value): set a library knob (hg_set_knob) for this test;
    every knob set is cleared afterwards."""
    from horreum_amd import abi
    touched = []

    def set_knob(name, value):
        abi.set_knob(name, value)
        touched.append(name)
    yield set_knob
    for name in touched:
        abi.set_knob(name, -1)
