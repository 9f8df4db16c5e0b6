import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "video-spike_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        with np.load(os.path.join(GOLDEN, name)) as f:      # allow_pickle=False (default)
            return {k: f[k] for k in f.files}
    return load


@pytest.fixture
def knobs():
    """Set libvspike A/B knobs (vspike.h VS_KNOB_*, read once from the environment at load) for one
    test: `knobs("no_wres", 1)`; every knob is restored afterwards."""
    from vspike import _lib as L
    saved = []

    def set_(name, value):
        saved.append((name, L.knob_set(name, value)))
    yield set_
    for name, prev in reversed(saved):
        L.knob_set(name, prev)
