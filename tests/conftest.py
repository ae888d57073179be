import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through librbgpu on cuda:0)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import rbref
    rbref.build()
    return rbref


@pytest.fixture(scope="session")
def ctx():
    import roaringbitmap_amd as rb
    if rb.Context.device_count() < 1:
        pytest.fail("no HIP device visible: gpu tests must run on the MI355X box")
    c = rb.Context(0)
    yield c
    c.close()
