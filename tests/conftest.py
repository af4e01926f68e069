import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libafem.so on cuda:0)")


@pytest.fixture(scope="session")
def ctx():
    import arcanefem_amd as af

    if af.device_count() < 1:
        pytest.skip("no GPU visible")
    c = af.Context(0)
    yield c
    c.close()


@pytest.fixture
def variant():
    """Select kernel variants (afem_set_variant) for one test; every knob set
    through it returns to the default at teardown.  variant(name, None)
    returns one knob to the default at once."""
    import arcanefem_amd as af

    used = set()

    def set_(name, value):
        used.add(name)
        af.set_variant(name, value)

    yield set_
    for n in used:
        af.set_variant(n, None)
