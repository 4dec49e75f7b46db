"""Shared test setup: import paths, the `gpu` marker, common fixtures."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "adlsm-tree_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def oracle():
    import oracle as O

    O.lib()
    return O


@pytest.fixture(scope="session")
def golden():
    import json

    d = os.path.join(ROOT, "tests", "golden")
    with open(os.path.join(d, "appendix_b.json")) as f:
        app = json.load(f)
    with open(os.path.join(d, "murmur3_ref.json")) as f:
        mm = json.load(f)
    return {"appendix_b": app, "murmur3": mm}


@pytest.fixture
def knobs(monkeypatch):
    """ADL_BLOOM_* switches for one test.  The library reads them once per
    process, so every change is followed by adl_bloom_reload_knobs(), and the
    teardown restores the environment and reloads it."""
    import adlbloom

    class Knobs:
        def set(self, name, value):
            monkeypatch.setenv(name, str(value))
            adlbloom.reload_knobs()

        def unset(self, name):
            monkeypatch.delenv(name, raising=False)
            adlbloom.reload_knobs()

    yield Knobs()
    monkeypatch.undo()
    adlbloom.reload_knobs()
