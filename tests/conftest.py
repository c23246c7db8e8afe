import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libcda on the device)")


@pytest.fixture(scope="session")
def ctx():
    import cda
    c = cda.Context(0)
    yield c
    c.close()
