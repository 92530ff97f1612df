import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP path)")
    config.addinivalue_line("markers", "slow: long CPU test")


def pytest_sessionstart(session):
    """Build the C oracle of the sample transform (test infrastructure, the checker only — the
    product build in __graft_entry__.build() does not touch oracle/)."""
    from oracle import augment_oracle
    augment_oracle.build()


import pytest  # noqa: E402


@pytest.fixture
def knob():
    """knob(name, value): set one of the library's kernel-selection knobs (include/psfm_knobs.h) for
    the rest of the test; every knob set this way is restored afterwards.  The environment is read
    only when the library loads, so tests switch forms through this, not through PSFM_* variables."""
    from packnet_sfm_amd import _hip
    saved = {}

    def set_(name, value):
        prev = _hip.set_knob(name, value)
        saved.setdefault(name, prev)

    yield set_
    for name, prev in saved.items():
        _hip.set_knob(name, prev)
