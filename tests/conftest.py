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
