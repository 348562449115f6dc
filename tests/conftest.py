import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; parity tests through the C ABI")
    config.addinivalue_line("markers", "slow: longer-running (full-size) case")


@pytest.fixture(scope="session")
def oracle():
    import oracle_py
    oracle_py.lib()
    return oracle_py


@pytest.fixture(scope="session")
def g2o_amd_mod():
    import g2o_amd
    return g2o_amd


def gpu_available() -> bool:
    try:
        import g2o_amd
        h = g2o_amd.lib().g2ohip_graph_create(0)
        if h:
            g2o_amd.lib().g2ohip_graph_destroy(h)
            return True
    except Exception:
        return False
    return False
