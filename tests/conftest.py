import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "sofa-jraft_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and libjrq.so")


@pytest.fixture(scope="session")
def oracle():
    import jraft_oracle
    jraft_oracle.lib()
    return jraft_oracle


@pytest.fixture(scope="session")
def engine():
    """One libjrq engine on cuda:0 for the whole GPU session (fails loudly without one)."""
    from jraft_amd import Engine
    e = Engine(0)
    yield e
    e.close()
