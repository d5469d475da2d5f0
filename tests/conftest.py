import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


_cache = {}


def golden(name):
    if name not in _cache:
        with open(os.path.join(GOLDEN, name)) as f:
            _cache[name] = json.load(f)
    return _cache[name]


@pytest.fixture(scope="session")
def codecs():
    return golden("codecs.json")


@pytest.fixture(scope="session")
def docs():
    return golden("docs.json")["scenarios"]


@pytest.fixture(scope="session")
def objmeta():
    """multi-call applyChanges histories over concurrently created objects (tests/golden/gen/make_objmeta.js)"""
    return golden("objmeta.json")["scenarios"]
