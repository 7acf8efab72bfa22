import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
FIX = os.path.join(ROOT, "tests", "fixtures")
GOLD = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libkmz.so on the device)")


def fixture(name):
    with open(os.path.join(FIX, name + ".json")) as f:
        return json.load(f)


def golden(name):
    with open(os.path.join(GOLD, name + ".json")) as f:
        return json.load(f)


def have_gpu():
    try:
        import ctypes

        from kmamiz_amd import _lib

        ctx = _lib.lib().kmz_create(0, None)
        if ctx:
            _lib.lib().kmz_destroy(ctx)
            return True
    except Exception:
        return False
    return False


@pytest.fixture(scope="session")
def engine():
    # -m gpu runs on an MI355X: a missing libkmz.so or device is an ERROR here,
    # never a skip (the engine has no CPU path)
    from kmamiz_amd import Engine

    e = Engine(0)
    yield e
    e.close()
