"""Shared test setup: import paths, the `gpu` marker, and an in-tree build if artefacts are missing.

`-m "not gpu"` runs here (no GPU): oracle vs golden fixtures, host logic, C-ABI exports.
`-m gpu` runs on an MI355X: the HIP path through the C ABI vs golden fixtures and the oracle.
"""
import json
import os
import subprocess
import sys

import pytest
import torch  # noqa: F401  (imported before rtc loads its HIP runtime: see rtc._init_torch_runtime_first)

# scenes 3 and 7 use the documented substitute earth picture (rtc/earth.py) in every test: opt-in
os.environ.setdefault("RTC_SUBSTITUTE_EARTH", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ray-tracing-c_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct MI355X (gfx950)")


def pytest_collection_modifyitems(config, items):
    """A per-test time limit (pytest-timeout, when installed) for every test without its own: a test stuck
    in a GPU call then fails with its name and stack instead of holding the run (thread method: it can
    interrupt a test blocked inside a HIP call)."""
    if not config.pluginmanager.hasplugin("timeout") or config.getoption("timeout", None):
        return
    for item in items:
        if item.get_closest_marker("timeout") is None:
            item.add_marker(pytest.mark.timeout(600, method="thread"))


def _make(path, *targets):
    subprocess.run(["make", "-s", "-C", path, "-j8", *targets], check=True)


@pytest.fixture(scope="session", autouse=True)
def built():
    if not os.path.exists(os.path.join(PKG, "librtc_amd.so")):
        _make(PKG)
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        _make(os.path.join(ROOT, "oracle"), "liboracle.so")
    if not os.path.exists(os.path.join(ROOT, "tests", "native", "bin", "libglibc_ref.so")):
        _make(os.path.join(ROOT, "tests", "native"))
    yield


@pytest.fixture(scope="session")
def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def golden_image(entry):
    """Full reference render (H, W, 3) uint8 for a manifest entry that kept its file."""
    import gzip

    import numpy as np

    with gzip.open(os.path.join(GOLDEN, entry["file"]), "rb") as f:
        data = f.read()
    return np.frombuffer(data, dtype=np.uint8).reshape(entry["height"], entry["width"], 3)
